#!/bin/bash
# Build a variant libngp_hip.so whose listed sources come from git revision
# REV (the rest from the working tree's build/obj), for same-box A/B of a
# change against its parent (tools/ab_variants.sh NAME).
# usage: bash tools/variant_rev.sh NAME REV src1 [src2 ...]   (sources without .hip)
set -eo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REV=$2; shift 2
OBJ=$R/build/obj
C=$R/torch-ngp_amd/csrc
out=$R/torch-ngp_amd/variants/$NAME
mkdir -p "$out"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function"
objs=""
for o in ngp_lib gridencoder raymarching shencoder ffmlp adam nerf_fused density_grid freqencoder exchange; do
    if [[ " $* " == *" $o "* ]]; then
        git -C "$R" show "$REV:torch-ngp_amd/csrc/$o.hip" > "$C/.rev_$o.hip"
        /opt/rocm/bin/hipcc $FLAGS -c "$C/.rev_$o.hip" -o "$out/$o.o"
        rm -f "$C/.rev_$o.hip"
        objs="$objs $out/$o.o"
    else
        objs="$objs $OBJ/$o.o"
    fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libngp_hip.so" $objs
rm -f "$out"/*.o
echo "built $out/libngp_hip.so ($* from $REV)"

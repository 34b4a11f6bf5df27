#!/bin/bash
# Build variant libngp_hip.so files that differ only in compile-time -D
# defines (a change under test, or -DNGP_STAMPS), for same-box A/B via NGP_HIP_LIB (tools/ab_env.sh, tools/ab_variants.sh).
# SRCS names the sources rebuilt with the knobs (default gridencoder; e.g.
# SRCS="nerf_fused density_grid" for ngp_head.h knobs); the rest come from
# the objects of a normal build (build/obj). Runs on the CPU host.
# usage: [SRCS="a b"] bash tools/variants.sh NAME "-DNGP_STAMPS ..." [NAME2 "DEFS2" ...]
set -eo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$R/build/obj
SRCS=${SRCS:-gridencoder}
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function"
while [ $# -ge 2 ]; do
    name=$1; defs=$2; shift 2
    out=$R/torch-ngp_amd/variants/$name
    mkdir -p "$out"
    objs=""
    for o in ngp_lib gridencoder raymarching shencoder ffmlp adam nerf_fused density_grid freqencoder exchange; do
        if [[ " $SRCS " == *" $o "* ]]; then
            /opt/rocm/bin/hipcc $FLAGS $defs -c "$R/torch-ngp_amd/csrc/$o.hip" -o "$out/$o.o"
            objs="$objs $out/$o.o"
        else
            objs="$objs $OBJ/$o.o"
        fi
    done
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libngp_hip.so" $objs
    rm -f "$out"/*.o
    echo "built $out/libngp_hip.so ($defs)"
done

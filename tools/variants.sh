#!/bin/bash
# Build variant libngp_hip.so files that differ only in gridencoder.hip's
# NGP_* compile-time knobs, for same-box A/B via NGP_HIP_LIB (tools/ab_env.sh).
# Needs the objects of a normal build (build/obj). Runs on the CPU host.
# usage: bash tools/variants.sh NAME "-DNGP_SEG_ITEMS=8192 ..." [NAME2 "DEFS2" ...]
set -eo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$R/build/obj
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function"
while [ $# -ge 2 ]; do
    name=$1; defs=$2; shift 2
    out=$R/torch-ngp_amd/variants/$name
    mkdir -p "$out"
    /opt/rocm/bin/hipcc $FLAGS $defs -c "$R/torch-ngp_amd/csrc/gridencoder.hip" -o "$out/gridencoder.o"
    objs=""
    for o in ngp_lib raymarching shencoder ffmlp adam nerf_fused density_grid; do objs="$objs $OBJ/$o.o"; done
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libngp_hip.so" $objs "$out/gridencoder.o"
    rm -f "$out/gridencoder.o"
    echo "built $out/libngp_hip.so ($defs)"
done

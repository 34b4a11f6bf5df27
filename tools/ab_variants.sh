#!/bin/bash
# Same-box A/B of the variant libraries from tools/variants.sh against the
# in-tree library: grid parity tests per variant, then interleaved bench runs.
# usage (on the box): [TESTS="tests/x.py ..."] bash tools/ab_variants.sh TAG NAME [NAME ...]
set -eo pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
lib() { if [ "$1" = base ]; then echo torch-ngp_amd/libngp_hip.so; else echo torch-ngp_amd/variants/$1/libngp_hip.so; fi; }
for v in "$@"; do
    NGP_HIP_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_grid_fused.py} -x -q \
        --timeout 120 --timeout-method thread > $O/test_$v.log 2>&1
    echo "$v tests: $(tail -1 $O/test_$v.log)"
done
for i in 1 2; do
    for v in base "$@"; do
        NGP_HIP_LIB=$(lib $v) timeout -k 10 200 python -u bench.py --no-cpu --no-legs --no-dp-path --no-render --steps 200 --warmup 20 ${BENCH_ARGS:-} \
            > $O/$v$i.json 2> $O/$v$i.err
        python -c "import json; d=json.load(open('$O/$v$i.json')); print('$v', $i, d['value'], d['ms_per_step'], {k: round(v * 1000, 1) for k, v in d['kernels_ms'].items()}, d.get('density_update_ms'))"
    done
done

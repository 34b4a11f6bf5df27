#!/bin/bash
# Same-box check of the in-tree library against variant libraries
# (tools/variant_rev.sh / tools/variants.sh): the parity tests on the in-tree
# library, then interleaved bench runs per workload.
# usage (on the box): [TESTS="..."] [WORKLOADS="lego truck"] [ROUNDS=2] bash tools/gpu_ab_lib.sh TAG NAME [NAME ...]
set -eo pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
lib() { if [ "$1" = base ]; then echo torch-ngp_amd/libngp_hip.so; else echo torch-ngp_amd/variants/$1/libngp_hip.so; fi; }
if [ "${TESTS:-x}" != none ]; then
    timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_grid_fused.py tests/test_gpu_e2e_oracle.py tests/test_gpu_fused.py} \
        -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
    echo "tests: $(tail -1 $O/tests.log)"
fi
for w in ${WORKLOADS:-lego}; do
    for i in $(seq 1 ${ROUNDS:-2}); do
        for v in base "$@"; do
            NGP_HIP_LIB=$(lib $v) timeout -k 10 200 python -u bench.py --no-cpu --workload $w --steps 200 --warmup 20 \
                > $O/${w}_$v$i.json 2> $O/${w}_$v$i.err
            python -c "import json; d=json.load(open('$O/${w}_$v$i.json')); r=d['roofline']; print('$w', '$v', $i, d['value'], d['ms_per_step'], 'gbwd', r['avg_launch_ms'], r['frac'], {k: round(v * 1000, 1) for k, v in d['kernels_ms'].items()})" | tee -a $O/ab.txt
        done
    done
done

#!/bin/bash
# Round-7 A/B pass: the in-tree library's grid / fused / e2e tests, then
# tools/ab_variants.sh over the named variants (interleaved bench runs).
# usage (on the box): bash tools/gpu_r07_ab.sh TAG NAME [NAME ...]
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 500 python -u -m pytest ${BASE_TESTS:-tests/test_gpu_grid_fused.py tests/test_gpu_fused.py tests/test_gpu_e2e_oracle.py} \
    -x -v --timeout 200 --timeout-method thread > $O/base_tests.log 2>&1
rc=$?; echo "base tests: rc $rc $(tail -1 $O/base_tests.log)"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 1500 bash tools/ab_variants.sh $TAG "$@"

#!/bin/bash
# Round-6 GPU pass: the grid / density / e2e files first (the changed paths),
# the whole -m gpu suite without -x (every failure named), smoke, the driver's
# bench command. usage (on the box): bash tools/gpu_r06.sh TAG
set -o pipefail
TAG=${1:-r06}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid_fused.py tests/test_density_golden.py \
    tests/test_gpu_e2e_oracle.py -v --timeout 120 --timeout-method thread > $O/first.log 2>&1
rc=$?; echo "first: rc $rc $(tail -1 $O/first.log)"
[ $rc -gt 1 ] && exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "gpu: rc $rc $(tail -1 $O/pytest_gpu.log)"
[ $rc -gt 1 ] && exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke: rc $rc $(tail -1 $O/smoke.log)"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench: rc $rc"; head -c 600 $O/bench.json
exit $rc

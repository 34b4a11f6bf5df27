#!/bin/bash
# One GPU-box check of a grid-kernel change: the grid / end-to-end parity
# tests, two 200-step bench lines and a kernel trace summary.
# usage (on the box): bash tools/gpu_check.sh TAG
set -eo pipefail
TAG=${1:-chk}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid_fused.py tests/test_gpu_e2e_oracle.py -x -q \
    --timeout 120 --timeout-method thread > $O/t.log 2>&1
for i in 1 2; do
    timeout -k 10 200 python -u bench.py --no-cpu --steps 200 --warmup 20 > $O/b$i.json 2> $O/b$i.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --no-cpu --steps 30 --warmup 10 > $O/trace.log 2>&1
python tools/prof_summary.py $O $O/step.json > /dev/null

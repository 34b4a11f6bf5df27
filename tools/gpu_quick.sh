#!/bin/bash
# Quick GPU check of the fused step: its tests, a bench line and a kernel trace.
# usage (on the box): bash tools/gpu_quick.sh TAG
set -eo pipefail
TAG=${1:-q}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fused_dp.py tests/test_gpu_grid_fused.py \
    -x -v --timeout 200 --timeout-method thread > $O/t.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu > $O/b.json 2> $O/b.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --no-cpu --steps 30 --warmup 10 > $O/trace.log 2>&1

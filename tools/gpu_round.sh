#!/bin/bash
# One GPU-box pass: parity tests, smoke, full bench line, rocprof stats + PMC.
# usage (on the box): bash tools/gpu_round.sh TAG
set -eo pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/$TAG/pytest_gpu.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > gpurun_out/$TAG/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
bash tools/prof.sh $TAG/prof

#!/bin/bash
# GPU tests + smoke + the driver's bench command, each step under its own limit.
# usage (on the box): bash tools/gpu_tests.sh TAG
set -eo pipefail
TAG=${1:-t}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > $O/smoke.log 2>&1
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err

#!/bin/bash
# Changed-path tests then the driver's bench command. usage: bash tools/gpu_quick2.sh TAG "TESTS"
set -o pipefail
TAG=${1:-q}; TESTS=${2:-tests/test_gpu_grid_fused.py}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest $TESTS -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests: rc $rc $(tail -1 $O/tests.log)"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu --no-legs --no-dp-path --no-render --steps 200 --warmup 20 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench: rc $rc"; python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d.get('kernels_ms'), d.get('live_rows_frac'), d.get('roofline_grid_encode', {}).get('avg_launch_ms'))"

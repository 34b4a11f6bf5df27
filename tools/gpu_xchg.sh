#!/bin/bash
# Exchange tests + the bench's dp_path probe. usage (on the box): bash tools/gpu_xchg.sh TAG
set -o pipefail
TAG=${1:-x}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_exchange.py tests/test_gpu_rccl.py tests/test_gpu_fused_dp.py tests/test_gpu_fused.py \
    tests/test_bench.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests: rc $rc $(tail -1 $O/tests.log)"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python -u bench.py --no-cpu --no-legs --no-render --steps 100 --warmup 20 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench: rc $rc"; python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], json.dumps(d.get('touched'))); dp=d.get('dp_path') or {}; print(dp.get('ms_per_step'), json.dumps(dp.get('three_graphs')), json.dumps(dp.get('sparse_exchange')))"

#!/bin/bash
# Density-update tests + the bench's density cadence numbers. usage (on the box): bash tools/gpu_dens.sh TAG
set -o pipefail
TAG=${1:-d}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_density.py tests/test_density_golden.py tests/test_gpu_fused_dp.py tests/test_gpu_rccl.py tests/test_gpu_fused.py \
    -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests: rc $rc $(tail -1 $O/tests.log)"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu --no-legs --no-dp-path --no-render --steps 100 --warmup 20 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench: rc $rc"; python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], json.dumps(d.get('density_update_ms')), json.dumps(d.get('with_density_update')))"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 tools/density_fused_probe.py > $O/probe.log 2>&1
echo "trace: rc $?"

#!/bin/bash
# Round-7 final pass: the whole -m gpu suite, smoke, the driver's bench
# command, then the evidence pass (tools/gpu_r07_evidence.sh: traces + PMC of
# every workload, MFMA). Each step under its own limit.
# usage (on the box): bash tools/gpu_r07_final.sh TAG
set -o pipefail
TAG=${1:-r07f}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "gpu tests: rc $rc $(tail -1 $O/pytest_gpu.log)"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke: rc $rc $(tail -1 $O/smoke.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench: rc $rc"; head -c 400 $O/bench.json; echo; [ $rc -ne 0 ] && exit $rc
timeout -k 10 950 bash tools/gpu_r07_evidence.sh ${TAG}ev
exit 0

#!/bin/bash
# Round-7 pass: the driver's bench command, then a kernel trace of the Lego
# bench (tools/prof_summary.py), each step under its own limit.
# usage (on the box): bash tools/gpu_r07_base.sh TAG [bench args...]
set -o pipefail
TAG=${1:-r07}
shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 "$@" > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench: rc $rc"; head -c 400 $O/bench.json; echo
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --no-cpu --no-legs --no-dp-path --no-render --steps 30 --warmup 10 "$@" > $O/trace.log 2>&1
rc=$?; echo "trace: rc $rc"; [ $rc -ne 0 ] && exit $rc
python tools/prof_summary.py $O $O/step_kernels.json > $O/summary.txt && echo summary ok
find $O/trace -type f -size +8M -delete
exit 0

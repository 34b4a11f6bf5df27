#!/bin/bash
# One GPU-box pass: parity tests, smoke, the bench line (+ the dense-occupancy,
# Config-5 truck and Config-3 fox workloads), rocprof stats + PMC.
# usage (on the box): bash tools/gpu_round.sh TAG [noprof]
set -eo pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest_gpu.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > gpurun_out/$TAG/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
timeout -k 10 200 python -u bench.py --no-cpu --workload lego_dense > gpurun_out/$TAG/bench_dense.json \
    2> gpurun_out/$TAG/bench_dense.err
timeout -k 10 200 python -u bench.py --no-cpu --workload truck > gpurun_out/$TAG/bench_truck.json \
    2> gpurun_out/$TAG/bench_truck.err
timeout -k 10 200 python -u bench.py --no-cpu --workload fox > gpurun_out/$TAG/bench_fox.json \
    2> gpurun_out/$TAG/bench_fox.err
if [ "$2" != "noprof" ]; then bash tools/prof.sh $TAG/prof; fi

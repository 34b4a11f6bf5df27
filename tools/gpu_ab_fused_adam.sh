#!/bin/bash
# Fused-table-Adam check on the GPU box: its tests, then a same-box A/B of the
# bench with it (NGP_FUSED_ADAM=1) and without it (the default), then a kernel trace.
# usage (on the box): bash tools/gpu_ab_fused_adam.sh TAG
set -eo pipefail
TAG=${1:-fa}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_rccl.py tests/test_gpu_fused_dp.py \
    tests/test_gpu_e2e_oracle.py tests/test_gpu_grid_fused.py tests/test_gpu_density.py -x -v --timeout 250 \
    --timeout-method thread > $O/t.log 2>&1
for i in 1 2; do
  NGP_FUSED_ADAM=1 timeout -k 10 300 python -u bench.py --no-cpu > $O/b_on_$i.json 2> $O/b_on_$i.err
  timeout -k 10 300 python -u bench.py --no-cpu > $O/b_off_$i.json 2> $O/b_off_$i.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --no-cpu --steps 30 --warmup 10 > $O/trace.log 2>&1

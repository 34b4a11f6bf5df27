#!/bin/bash
# Same-box A/B of an environment switch over the four bench workloads.
# usage (on the box): bash tools/gpu_ab_workloads.sh TAG "ENV_A" "ENV_B"
set -eo pipefail
TAG=$1; EA=$2; EB=$3
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
for w in lego truck fox lego_dense; do
  for n in A B; do
    e=$EA; [ $n = B ] && e=$EB
    env $e timeout -k 10 200 python -u bench.py --no-cpu --workload $w --steps 100 --warmup 10 > $O/${w}_$n.json 2> $O/${w}_$n.err
    python -c "import json; d=json.load(open('$O/${w}_$n.json')); print('$w', '$n', d['value'], d['ms_per_step'], d.get('density_update_ms'))" >> $O/ab.txt
  done
done

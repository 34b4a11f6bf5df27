#!/bin/bash
# A/B of an environment switch on one box: alternating bench runs + one
# kernel trace each. usage: bash tools/ab_env.sh TAG "ENV_A" "ENV_B" [ROUNDS]
set -eo pipefail
TAG=$1; EA=$2; EB=$3; R=${4:-3}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
for i in $(seq 1 $R); do
  for n in A B; do
    e=$EA; [ $n = B ] && e=$EB
    env $e timeout -k 10 200 python -u bench.py --no-cpu --steps 200 --warmup 20 > $O/$n$i.json 2> $O/$n$i.err
    python -c "import json; d=json.load(open('$O/$n$i.json')); print('$n', $i, d['value'], d['ms_per_step'])"
  done
done
for n in A B; do
  e=$EA; [ $n = B ] && e=$EB
  timeout -k 10 300 env $e rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$n/trace -o run -- \
      python3 bench.py --no-cpu --steps 30 --warmup 10 > $O/trace$n.log 2>&1
  python tools/prof_summary.py $O/p$n $O/step_$n.json > /dev/null
  python -c "import json; d=json.load(open('$O/step_$n.json')); print('$n', d['kernel_busy_us_per_step'], d['kernels_us_per_step'])"
done

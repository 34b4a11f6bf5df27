#!/bin/bash
# Same-box A/B of two bench argument sets (interleaved rounds).
# usage (on the box): [ROUNDS=2] [WORKLOAD=lego] bash tools/gpu_ab_args.sh TAG "ARGS_A" "ARGS_B"
set -eo pipefail
TAG=$1; AA=$2; AB=$3
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
for i in $(seq 1 ${ROUNDS:-2}); do
    for n in A B; do
        a=$AA; [ $n = B ] && a=$AB
        timeout -k 10 200 python -u bench.py --no-cpu --workload ${WORKLOAD:-lego} --steps 200 --warmup 20 $a \
            > $O/$n$i.json 2> $O/$n$i.err
        python -c "import json; d=json.load(open('$O/$n$i.json')); print('$n', $i, '$a', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" | tee -a $O/ab.txt
    done
done

#!/bin/bash
# A/B of two builds of the library on one box: alternating bench runs.
# usage (on the box): bash tools/ab.sh TAG LIB_A LIB_B [ROUNDS]
set -eo pipefail
TAG=$1; A=$2; B=$3; R=${4:-3}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/$TAG; mkdir -p $O
for i in $(seq 1 $R); do
  for n in A B; do
    lib=$A; [ $n = B ] && lib=$B
    NGP_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --no-cpu --steps 200 --warmup 20 > $O/$n$i.json 2> $O/$n$i.err
    python -c "import json,sys; d=json.load(open('$O/$n$i.json')); print('$n', $i, d['value'], {k: round(v*1000,1) for k,v in d['kernels_ms'].items()})"
  done
done

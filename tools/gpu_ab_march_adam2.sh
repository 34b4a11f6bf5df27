#!/bin/bash
# Same-box A/B: Adam in the head launch (A) vs inside the march launch with 8
# (B) or 4 (C, variant mw4) march waves per workgroup.
set -eo pipefail
TAG=${1:-ma2}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
NGP_MARCH_ADAM=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1
for i in 1 2; do
  for v in A B C; do
    e="NGP_MARCH_ADAM=0"; lib=torch-ngp_amd/libngp_hip.so
    [ $v != A ] && e="NGP_MARCH_ADAM=1"
    [ $v = C ] && lib=torch-ngp_amd/variants/mw4/libngp_hip.so
    env $e NGP_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --no-cpu --steps 200 --warmup 20 > $O/$v$i.json 2> $O/$v$i.err
    python -c "import json; d=json.load(open('$O/$v$i.json')); print('$v', $i, d['value'], d['ms_per_step'])" >> $O/ab.txt
  done
done
for v in B C; do
  lib=torch-ngp_amd/libngp_hip.so; [ $v = C ] && lib=torch-ngp_amd/variants/mw4/libngp_hip.so
  timeout -k 10 300 env NGP_MARCH_ADAM=1 NGP_HIP_LIB=$PWD/$lib rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$v/trace -o run -- \
      python3 bench.py --no-cpu --steps 30 --warmup 10 > $O/trace$v.log 2>&1
  python tools/prof_summary.py $O/p$v $O/step_$v.json > /dev/null
  python -c "import json; d=json.load(open('$O/step_$v.json')); print('$v', d['kernel_busy_us_per_step'], d['kernels_us_per_step'])" >> $O/ab.txt
done

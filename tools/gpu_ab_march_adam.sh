#!/bin/bash
# GPU check + same-box A/B of Adam inside the march launch (NGP_MARCH_ADAM)
# and of the MLP backward's overlapped tile round trip (variant ovl0).
# usage (on the box): bash tools/gpu_ab_march_adam.sh TAG
set -eo pipefail
TAG=${1:-ma}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
NGP_MARCH_ADAM=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_e2e_oracle.py tests/test_gpu_rccl.py \
    -x -v --timeout 200 --timeout-method thread > $O/t.log 2>&1
bash tools/ab_env.sh $TAG/env "NGP_MARCH_ADAM=0" "NGP_MARCH_ADAM=1" 2 > $O/env_ab.txt 2>&1
for i in 1 2; do
  for v in base ovl0; do
    lib=torch-ngp_amd/libngp_hip.so; [ $v = ovl0 ] && lib=torch-ngp_amd/variants/ovl0/libngp_hip.so
    NGP_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --no-cpu --steps 200 --warmup 20 > $O/$v$i.json 2> $O/$v$i.err
    python -c "import json; d=json.load(open('$O/$v$i.json')); print('$v', $i, d['value'], d['ms_per_step'], {k: round(x * 1000, 1) for k, x in d['kernels_ms'].items()})" >> $O/ovl_ab.txt
  done
done

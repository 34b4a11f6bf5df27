#!/bin/bash
# GPU check of the march / freq changes: their parity tests, the fox e2e
# oracle test and the fox + Lego bench legs.
# usage (on the box): bash tools/gpu_check_march.sh TAG
set -eo pipefail
TAG=${1:-m}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_freq.py tests/test_gpu_parity.py tests/test_gpu_e2e_oracle.py \
    -x -v --timeout 200 --timeout-method thread > $O/t.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu --workload fox > $O/fox.json 2> $O/fox.err
timeout -k 10 200 python -u bench.py --no-cpu > $O/lego.json 2> $O/lego.err

#!/bin/bash
# Stamps (trained regime) + a kernel trace of the bench, each step under its
# own limit. usage (on the box): bash tools/gpu_r06_prof.sh TAG
set -o pipefail
TAG=${1:-r06p}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_density_golden.py -v --timeout 120 --timeout-method thread \
    > $O/density_golden.log 2>&1
echo "density golden: rc $? $(tail -1 $O/density_golden.log)"
NGP_HIP_LIB=torch-ngp_amd/variants/stamps/libngp_hip.so timeout -k 10 200 python -u tools/accum_stamps.py 600 \
    > $O/accum_stamps.json 2> $O/accum_stamps.err
rc=$?; echo "accum stamps: rc $rc"; [ $rc -gt 1 ] && exit $rc
NGP_HIP_LIB=torch-ngp_amd/variants/stamps/libngp_hip.so timeout -k 10 200 python -u tools/bwd_stamps.py 600 \
    > $O/bwd_stamps.json 2> $O/bwd_stamps.err
rc=$?; echo "bwd stamps: rc $rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --no-cpu --no-legs --no-dp-path --no-render --steps 30 --warmup 10 > $O/trace.log 2>&1
rc=$?; echo "trace: rc $rc"; [ $rc -ne 0 ] && exit $rc
python tools/prof_summary.py $O/trace $O/step_kernels.json > /dev/null && echo summary ok

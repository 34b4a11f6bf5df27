#!/bin/bash
# Phase clocks of the grid backward (tools/accum_stamps.py) for stamps variant
# libraries. usage (on the box): bash tools/gpu_stamps.sh TAG NAME[:BIN_PTS] ...
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
for v in "$@"; do
    n=${v%%:*}; bp=${v#*:}; [ "$bp" = "$v" ] && bp=512
    BIN_PTS=$bp NGP_HIP_LIB=torch-ngp_amd/variants/$n/libngp_hip.so timeout -k 10 200 python -u tools/accum_stamps.py 600 \
        > $O/$n.json 2> $O/$n.err
    rc=$?; echo "$n: rc $rc"; [ $rc -gt 1 ] && exit $rc
done
exit 0

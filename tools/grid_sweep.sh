#!/bin/bash
# Sweep debug knobs of the fused grid backward (tools/grid_bwd_micro.py), kernel times by rocprofv3.
# usage: bash tools/grid_sweep.sh "NGP_DBG_ACCUM=1" "NGP_MERGE_RES=512" ...
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd "$R"
mkdir -p gpurun_out/sweep
for cfg in "$@"; do
    name=$(echo "$cfg" | tr ' =' '_-')
    (
        for kv in $cfg; do export "$kv"; done
        timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/sweep/$name" -o run -- \
            python3 tools/grid_bwd_micro.py > "gpurun_out/sweep/$name.log" 2>&1
    )
done

#!/bin/bash
# Round-7 evidence pass over the final tree: kernel trace + FETCH/WRITE PMC of
# every bench workload (tools/prof.sh, tools/prof_summary.py: the legs'
# roofline `traffic` reads these), then the MFMA passes on Lego and
# lego_dense (tools/pmc_mlp.sh, tools/mfma_busy.py). Each step under its own
# limit. usage (on the box): bash tools/gpu_r07_evidence.sh TAG [workloads...]
set -o pipefail
TAG=${1:-r07e}
shift
WLS=${*:-lego lego_dense truck fox}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
for w in $WLS; do
    args=""; [ "$w" != lego ] && args="--workload $w"
    BENCH_ARGS="$args" timeout -k 10 900 bash tools/prof.sh ${TAG}_$w; echo "prof $w: rc $?"
    WORKLOAD=$w python tools/prof_summary.py gpurun_out/${TAG}_$w gpurun_out/${TAG}_${w}_step_kernels.json > /dev/null
    echo "summary $w: rc $?"
done
if [ -z "${SKIP_MFMA:-}" ]; then
    timeout -k 10 500 bash tools/pmc_mlp.sh ${TAG}_pmc_lego; echo "pmc lego: rc $?"
    BENCH_ARGS='--workload lego_dense' timeout -k 10 500 bash tools/pmc_mlp.sh ${TAG}_pmc_dense; echo "pmc dense: rc $?"
    python tools/mfma_busy.py gpurun_out/${TAG}_pmc_lego gpurun_out/${TAG}_pmc_dense > gpurun_out/${TAG}_mfma.txt
    cat gpurun_out/${TAG}_mfma.txt
fi
exit 0

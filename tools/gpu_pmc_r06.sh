#!/bin/bash
# Final-tree evidence: kernel trace + FETCH/WRITE passes of the Lego bench
# (tools/prof.sh), then the MFMA passes on Lego and lego_dense (tools/pmc_mlp.sh).
# usage (on the box): bash tools/gpu_pmc_r06.sh TAG
set -o pipefail
TAG=${1:-r06o}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
timeout -k 10 900 bash tools/prof.sh ${TAG}_prof; echo "prof: rc $?"
python tools/prof_summary.py gpurun_out/${TAG}_prof gpurun_out/${TAG}_step_kernels.json > /dev/null; echo "summary: rc $?"
timeout -k 10 500 bash tools/pmc_mlp.sh ${TAG}_pmc_lego; echo "pmc lego: rc $?"
BENCH_ARGS='--workload lego_dense' timeout -k 10 500 bash tools/pmc_mlp.sh ${TAG}_pmc_dense; echo "pmc dense: rc $?"
python tools/mfma_busy.py gpurun_out/${TAG}_pmc_lego gpurun_out/${TAG}_pmc_dense > gpurun_out/${TAG}_mfma.txt; cat gpurun_out/${TAG}_mfma.txt

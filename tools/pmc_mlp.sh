#!/bin/bash
# MFMA evidence for the FFMLP kernels: separate --pmc passes over a short
# bench (one counter group each), kernel names filtered to the MLP kernels.
# usage (on the box): bash tools/pmc_mlp.sh TAG
set -o pipefail
TAG=${1:-pmc_mlp}
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
KRE='k_mlp|k_nerf_fwd|k_nerf_bwd|k_density_fwd|k_grid_bwd_bin|k_grid_bin_accum|k_grid_fwd|k_adam'
i=0
for PMC in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_BUSY_CU_CYCLES" "SQ_WAVE_CYCLES SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv --kernel-include-regex "$KRE" -d "$O/p$i" -o run -- \
      python3 bench.py --no-cpu --no-legs --no-dp-path --no-render ${BENCH_ARGS:-} --steps 5 --warmup 3 --settle-steps 0 --kernel-steps 2 > "$O/p$i.log" 2>&1 || echo "pass $i ($PMC) failed rc=$?" >> "$O/failed.txt"
done
exit 0

#!/bin/bash
# Round-5 pass e on the GPU box: the 6-byte item variant A/B (grid parity tests
# + interleaved bench legs), then the MLP MFMA PMC passes on Lego and lego_dense.
# usage (on the box): bash tools/gpu_r05e.sh
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
TESTS="tests/test_gpu_grid_fused.py" bash tools/ab_variants.sh r05e_soa soa > gpurun_out/r05e_soa.txt 2>&1
bash tools/pmc_mlp.sh r05e_pmc_lego
BENCH_ARGS="--workload lego_dense" bash tools/pmc_mlp.sh r05e_pmc_dense

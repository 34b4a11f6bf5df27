#!/bin/bash
# SQ counters for the fused grid backward kernels (tools/grid_bwd_micro.py).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd "$R"
O=gpurun_out/pmc_grid
mkdir -p $O
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT \
    --output-format csv --kernel-include-regex "k_grid_b" -d $O/a -o run -- python3 tools/grid_bwd_micro.py > $O/a.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE \
    --output-format csv --kernel-include-regex "k_grid_b" -d $O/b -o run -- python3 tools/grid_bwd_micro.py > $O/b.log 2>&1

#!/bin/bash
# Round-5 pass e on the GPU box: the driver's bench command (every object of
# the line: legs, dp_path, render, cpu_baseline), the RCCL capture probe, the
# 6-byte item variant A/B (grid parity tests + interleaved bench legs), then
# the MLP MFMA PMC passes on Lego and lego_dense.
# usage (on the box): bash tools/gpu_r05e.sh
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
timeout -k 10 200 python -u tools/rccl_capture_probe.py > $O/rccl_capture_probe.json 2> $O/rccl_capture_probe.err
TESTS="tests/test_gpu_grid_fused.py" bash tools/ab_variants.sh r05e_soa soa > $O/soa_ab.txt 2>&1
bash tools/pmc_mlp.sh r05e_pmc_lego
BENCH_ARGS="--workload lego_dense" bash tools/pmc_mlp.sh r05e_pmc_dense

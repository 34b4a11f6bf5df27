#!/bin/bash
# Profile the default bench on the GPU box: kernel trace + stats, then two
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) for the step's big kernels.
# usage (on the box): bash tools/prof.sh TAG
set -eo pipefail
trap 'du -ah "$O" 2>/dev/null | sort -h | tail -20 > "$O/sizes.txt"; find "$O" -type f -size +8M -delete' EXIT
TAG=${1:-prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
[ -n "${SKIP_TRACE:-}" ] || timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
    python3 bench.py --no-cpu --no-legs --no-dp-path --no-render ${BENCH_ARGS:-} --steps 30 --warmup 10 > "$O/trace.log" 2>&1
# PMC passes on eager steps (--no-graph). The per-launch bytes follow the
# training state: as the field trains, samples behind early-terminated rays get
# a zero gradient (r05m: the bin launch writes 52-59 MB in the first steps, 2-6
# MB after a few hundred), and the backwards walk only the live rows. The
# summary's median is over the whole run, so the passes settle 300 steps
# first: the median is the trained regime the bench times
KRE='k_grid_bwd|k_grid_bin|k_grid_fwd|k_adam|k_mlp|k_nerf_fwd|k_nerf_bwd|k_march|k_composite|k_glue|k_live'
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv --kernel-include-regex "$KRE" -d "$O/fetch" -o run -- \
    python3 bench.py --no-cpu --no-legs --no-dp-path --no-render ${BENCH_ARGS:-} --no-graph --steps 5 --warmup 3 --settle-steps ${PMC_SETTLE:-300} > "$O/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv --kernel-include-regex "$KRE" -d "$O/write" -o run -- \
    python3 bench.py --no-cpu --no-legs --no-dp-path --no-render ${BENCH_ARGS:-} --no-graph --steps 5 --warmup 3 --settle-steps ${PMC_SETTLE:-300} > "$O/write.log" 2>&1

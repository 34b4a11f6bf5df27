#!/bin/bash
# Kernel-trace stats of the bench step for the in-tree library and variants,
# one rocprofv3 run each (same box).
# usage (on the box): [WORKLOADS="lego truck"] bash tools/gpu_prof_libs.sh TAG NAME [NAME ...]
set -eo pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
lib() { if [ "$1" = base ]; then echo torch-ngp_amd/libngp_hip.so; else echo torch-ngp_amd/variants/$1/libngp_hip.so; fi; }
for w in ${WORKLOADS:-lego}; do
    for v in base "$@"; do
        NGP_HIP_LIB=$(lib $v) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${w}_$v -o run -- \
            python3 bench.py --no-cpu --workload $w --steps 100 --warmup 10 > $O/${w}_$v.log 2>&1
        f=$(find $O/${w}_$v -name run_kernel_stats.csv | sort | tail -n 1)
        python3 - "$f" "$w" "$v" <<'PY' | tee -a $O/prof.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print(sys.argv[2], sys.argv[3])
for r in rows[:14]:
    print("  %-60s %6s %9.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1000))
PY
    done
done

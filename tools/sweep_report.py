import csv, glob, os, statistics, sys
# median duration of each grid-backward kernel over its last 50 launches (the back-to-back timed calls)
for d in sorted(glob.glob("gpurun_out/sweep/*/")):
    f = os.path.join(d, "run_kernel_trace.csv")
    if not os.path.exists(f):
        continue
    per = {}
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        for k in ("k_grid_bin_accum", "k_grid_bwd_bin", "k_grid_bwd<"):
            if k in n:
                per.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(os.path.basename(d.rstrip("/")), {k: round(statistics.median(v[-50:]), 1) for k, v in per.items()})

"""Per-update kernel makeup of the partial density-grid updates in a rocprofv3
kernel trace of tools/density_trace.py: each update is the span from the
flush's Adam sweep (k_adam_multi) to the occupancy rebuild (k_occ_compact);
prints each kernel's mean duration, the mean gap between launches and the
mean span (device time, no host overhead) over the last `n` updates.
    python tools/density_span.py run_kernel_trace.csv [n]"""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    for key in ("k_grid_fwd_tail", "k_grid_fwd_pair", "k_density_fwd", "k_adam_multi"):
        if key in n:
            return key
    return n.split("(")[0][:40]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ups, cur = [], None
    for r in rows:
        k = short(r["Kernel_Name"])
        if k == "k_adam_multi":
            cur = [(k, int(r["Start_Timestamp"]), int(r["End_Timestamp"]))]
        elif cur is not None:
            cur.append((k, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
            if k == "k_occ_compact":
                ups.append(cur)
                cur = None
    ups = [u for u in ups if any(k == "k_ostat_points" for k, _, _ in u)][-n:]  # partial updates
    dur, order = defaultdict(float), []
    span = gaps = 0.0
    for u in ups:
        for k, a, b in u:
            if k not in order:
                order.append(k)
            dur[k] += (b - a) / 1e3
        span += (u[-1][2] - u[0][1]) / 1e3
        gaps += sum(max(0, u[i + 1][1] - u[i][2]) for i in range(len(u) - 1)) / 1e3
    m = len(ups)
    print(f"{m} partial updates: span {span / m:.1f} us, kernels {sum(dur.values()) / m:.1f} us, gaps {gaps / m:.1f} us")
    for k in order:
        print(f"  {dur[k] / m:7.1f} us  {k}")


if __name__ == "__main__":
    main()

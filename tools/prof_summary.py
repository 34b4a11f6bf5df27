"""Summarise a tools/prof.sh run: per-kernel device time inside the timed
graph replays of bench.py (steps delimited by k_lego_rays), and per-launch
FETCH_SIZE / WRITE_SIZE from the two PMC passes.

usage: python tools/prof_summary.py gpurun_out/TAG [profiles/OUT.json]
FETCH_SIZE / WRITE_SIZE are reported raw (KB x 1024). On gfx950 FETCH_SIZE
counts half the bytes of wide coalesced streaming reads (MI355X_MICROARCH.md,
HBM section): `fetch_bytes_x2` carries the doubled figure for those kernels.
"""
import collections
import csv
import json
import os
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    if n.startswith("_ZN"):  # mangled template instance: keep the kernel identifier
        import re
        m = re.search(r"(k_[a-z0-9_]+)", n)
        n = (m.group(1) if m else n[:40]) + "<" + n[-40:].split("EEv")[0][-12:] + ">"
    return n


def main(tag, out=None):
    rows = list(csv.DictReader(open(os.path.join(tag, "trace", "run_kernel_trace.csv"))))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # bench.py order: ... timed graph replays (STEPS), each one step body
    # [k_adam_multi (previous grads; the inf check comes from the backward's
    # kernels), k_step_head, ...,
    # grid backward]; then FusedTrainer.timed_steps: flush() (3 optimizer
    # kernels) and eager steps behind torch's spin kernel.
    steps = int(os.environ.get("STEPS", "30"))
    spin = next((i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]), len(rows))
    name = lambda i: rows[i]["Kernel_Name"] if i < len(rows) else ""  # noqa: E731
    # a step starts with k_adam_head (merged optimizer + batch launch) or, with
    # options split_head / older builds, k_adam_multi followed by k_step_head
    # or (march_adam, Adam inside the march launch) k_step_head alone, or
    # (draw_ahead: the batch drawn in the previous bin launch) the march +
    # Adam launch k_march_train<4> itself
    starts = [i for i in range(spin) if "k_adam_head" in name(i) or
              ("k_adam_multi" in name(i) and "k_step_head" in name(i + 1)) or
              ("k_step_head" in name(i) and "k_adam_multi" not in name(i - 1) and "k_march_train" in name(i + 1)) or
              ("k_march_train<" in name(i) and "k_march_train<16" not in name(i) and
               "k_step_head" not in name(i - 1))]
    sel = starts[-steps:]
    per = collections.defaultdict(list)
    spans = []
    bwd_spans = []  # grid backward: start of k_grid_bwd_bin to end of k_grid_bin_accum (what the bench's events bracket)
    for i in sel:
        j = next(k for k in range(i, len(rows)) if "k_grid_bin_accum" in name(k)) + 1
        seg = rows[i:j]
        t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
        spans.append((t1 - t0) / 1e3)
        b0 = next((r for r in seg if "k_grid_bwd_bin" in r["Kernel_Name"]), None)
        if b0 is not None:
            bwd_spans.append((int(seg[-1]["End_Timestamp"]) - int(b0["Start_Timestamp"])) / 1e3)
        cnt = collections.Counter()
        for r in seg:
            key = short(r["Kernel_Name"])
            cnt[key] += 1
            per[key + ("" if cnt[key] == 1 else f"#{cnt[key]}")].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    kern = {k: round(sum(v) / len(v), 2) for k, v in per.items()}
    busy = sum(kern.values())
    pmc = {}
    for which in ("fetch", "write"):
        p = os.path.join(tag, which, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(p)):
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024)
        for k, v in acc.items():
            # median: the bench's density-grid update also launches the grid
            # forward (2M points), a few outliers among the step's launches
            v = sorted(v)
            pmc.setdefault(k, {})[which + "_bytes"] = round(v[len(v) // 2])
    # the bench line printed by the profiled command (samples of its timed steps)
    bench = None
    try:
        for line in open(os.path.join(tag, "trace.log")):
            if line.startswith("{") and '"metric"' in line:
                bench = json.loads(line)
    except OSError:
        pass
    bwd_kernels = sum(v for k, v in kern.items() if k.startswith(("k_grid_bwd_bin", "k_grid_bin_accum")))
    res = {
        "workload": os.environ.get("WORKLOAD", "lego"),
        "steps": len(sel),
        "step_span_us_mean": round(sum(spans) / len(spans), 1),
        "kernel_busy_us_per_step": round(busy, 1),
        "kernels_us_per_step": dict(sorted(kern.items(), key=lambda t: -t[1])),
        "pmc_per_launch": pmc,
    }
    if bwd_spans:
        res["grid_backward_us"] = {"kernels_sum": round(bwd_kernels, 2),
                                   "span_bin_start_to_accum_end": round(sum(bwd_spans) / len(bwd_spans), 2)}
    if bench is not None and bwd_spans:
        # the roofline recomputed from this trace: SURVEY 8(d) 1100 B per sample
        # x the mean samples of the bench's timed steps / the trace's time
        r = bench.get("roofline", {})
        if r.get("samples_timed"):  # device-clock timing: the samples of the timed launches themselves
            samples = r["samples_timed"] / r["launches_timed"]
        else:
            counts = r.get("samples_per_timed_launch") or [bench["config"]["samples_per_step"]]
            samples = sum(counts) / len(counts)
        res["roofline_recomputed"] = {
            "samples_per_step": round(samples, 1),
            "frac_from_kernels_sum": round(1100 * samples / (bwd_kernels * 1e-6) / 8e12, 4),
            "frac_from_span": round(1100 * samples / (res["grid_backward_us"]["span_bin_start_to_accum_end"] * 1e-6)
                                    / 8e12, 4),
            "bench_frac": r.get("frac"), "bench_avg_launch_ms": r.get("avg_launch_ms"),
            "bench_timing": r.get("timing")}
        if r.get("frac"):
            rr = res["roofline_recomputed"]
            rr["bench_vs_kernels_sum"] = round(r["frac"] / rr["frac_from_kernels_sum"] - 1, 4)
    txt = json.dumps(res, indent=1)
    print(txt)
    if out:
        open(out, "w").write(txt + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])

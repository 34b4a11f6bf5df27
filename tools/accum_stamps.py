"""Phase clocks of the grid backward (bin + accumulate kernels) in the
trained regime (diagnostic build with -DNGP_STAMPS:
SRCS="gridencoder ffmlp" bash tools/variants.sh stamps "-DNGP_STAMPS"):
runs [steps] fused steps of the bench's Lego workload, then one more, and
summarises the per-workgroup s_memtime stamps (step 1 / retire / per unit:
zero, adds, flush; bin phases).
    NGP_HIP_LIB=torch-ngp_amd/variants/stamps/libngp_hip.so python tools/accum_stamps.py [steps]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _ngp_native as nat  # noqa: E402
from nerf.fused import FusedTrainer  # noqa: E402
from nerf.network_ff import NeRFNetwork  # noqa: E402
from nerf.provider import SyntheticLego, lego_bitfield  # noqa: E402

dev = torch.device("cuda:0")
import bench  # noqa: E402
_argv, sys.argv = sys.argv, sys.argv[:1]
_args = bench.parse()
sys.argv = _argv
STEPS = int(_argv[1]) if len(_argv) > 1 else 300  # the trained regime (live rows) by default
model, data, *_ = bench.make_workload("lego", dev, 1, 4096)
ft, _ = bench.make_trainer(_args, model, data, 1, dev, 0.0, grid_timing=False)
stamps = torch.zeros(4096 * 64, dtype=torch.int64, device=dev)
lib = nat.lib()
assert lib.ngp_debug_stamps(ctypes.c_void_p(nat.ptr(stamps))) == 0
# k_mlp_bwd / k_nerf_bwd: (NH - 1) * 2048 + wave rows of 16 (ffmlp.hip MSTAMP); set before any step
ms = torch.zeros(3 * 2048 * 16 + 4096 * 16, dtype=torch.int64, device=dev)
if hasattr(lib, "ngp_debug_mlp_stamps"):
    assert lib.ngp_debug_mlp_stamps(ctypes.c_void_p(nat.ptr(ms))) == 0
for _ in range(STEPS):
    ft.step()
torch.cuda.synchronize()
stamps.zero_()  # one more step on a clean buffer: no stale stamps of workgroups that exited early
ms.zero_()
ft.step()
torch.cuda.synchronize()
print(json.dumps({"steps": STEPS, "samples": ft.sample_count(), "live_frac": ft.live_fraction()}))
st = stamps[:32768].view(-1, 64).cpu().numpy().astype(np.int64)  # accumulate: 2 workgroups per CU
nwg = int((st[:, 0] > 0).sum())
st = st[:nwg]
wr = st[:, 10] > 0  # wave-bin workgroups (gridencoder.hip wave_bin): their own phase clocks
st_all, wr_all = st.copy(), wr.copy()
ws = stamps[131072:131072 + 4096 * 4].view(-1, 4).cpu().numpy().astype(np.int64)
ws = ws[ws[:, 1] > 0]
if len(ws):
    n, lvw, dur = ws[:, 0] & 0xffffffff, (ws[:, 0] >> 32) & 0xff, ws[:, 2] - ws[:, 1]
    order = np.argsort(dur)[::-1][:12]
    print(json.dumps({"wave_bins": {"bins": int(len(ws)), "dur_pct": [int(x) for x in np.percentile(dur, [10, 50, 90, 99, 100])],
                                    "n_pct": [int(x) for x in np.percentile(n, [10, 50, 90, 100])],
                                    "spilled": int(((ws[:, 0] >> 40) & 1).sum()),
                                    "slowest": [[int(dur[i]), int(n[i]), int(lvw[i]), int(ws[i, 3])] for i in order],
                                    "corr_n_dur": float(np.corrcoef(n, dur)[0, 1])}}))
if wr.any():
    w = st[wr]
    t0w = st[:, 0].min()
    print(json.dumps({"wave_role": {
        "workgroups": int(wr.sum()),
        "entry_med": int(np.median(w[:, 0] - t0w)), "entry_max": int(np.max(w[:, 0] - t0w)),
        "lds_zero_med": int(np.median(w[:, 10] - w[:, 0])),
        "count_load_med": int(np.median(w[w[:, 11] > 0, 11] - w[w[:, 11] > 0, 10])) if (w[:, 11] > 0).any() else None,
        "bitmap_med": int(np.median(w[w[:, 12] > 0, 12] - w[w[:, 12] > 0, 11])) if (w[:, 12] > 0).any() else None,
        "passes_med": int(np.median(w[w[:, 13] > 0, 13] - w[w[:, 13] > 0, 12])) if (w[:, 13] > 0).any() else None,
        "wave0_total_med": int(np.median(w[:, 14] - w[:, 0])), "wave0_total_max": int(np.max(w[:, 14] - w[:, 0])),
        "end_med_rel": int(np.median(w[:, 14] - t0w)), "end_max_rel": int(np.max(w[:, 14] - t0w))}}))
    if (~wr).any():
        im = st[~wr]
        print(json.dumps({"image_role": {"workgroups": int((~wr).sum()),
                                         "entry_med": int(np.median(im[:, 0] - t0w)),
                                         "prologue_med": int(np.median(im[:, 1] - im[:, 0]))}}))
    st = st[~wr] if (~wr).any() else st
    nwg = len(st)
t0 = st[:, 0].min()
res = {"workgroups": nwg, "kernel_cycles": int(max(st[i, 4 + 5 * (int(st[i, 3]) - 1) + 2] if st[i, 3] else st[i, 2]
                                                    for i in range(nwg)) - t0)}
res["entry_spread"] = int(st[:, 0].max() - t0)
res["step1_med"] = int(np.median(st[:, 1] - st[:, 0]))
res["retire_med"] = int(np.median(st[:, 2] - st[:, 1]))
res["retire_max"] = int(np.max(st[:, 2] - st[:, 1]))
units = []
for i in range(nwg):
    prev = st[i, 2]
    for u in range(int(min(st[i, 3], 11))):
        a, b, c, info, d = st[i, 4 + 5 * u: 9 + 5 * u]
        # d: after the barrier that drains the adds (0 in builds without that stamp)
        dr, fl = (d - b, c - d) if d else (0, c - b)
        units.append((a - prev, b - a, c - b, info & 0xffffffff, (info >> 32) & 0xff, (info >> 40) & 0xff, dr, fl))
        prev = c
u = np.array(units, dtype=np.int64)
res["units"] = len(u)
res["units_per_wg_max"] = int(st[:, 3].max())
for k, name in ((0, "gap_to_start"), (1, "adds"), (2, "drain_and_flush"), (6, "drain"), (7, "flush")):
    res[name + "_med"] = int(np.median(u[:, k]))
    res[name + "_p90"] = int(np.percentile(u[:, k], 90))
    res[name + "_sum_per_wg"] = int(u[:, k].sum() / nwg)
res["items_med"] = int(np.median(u[:, 3]))
res["owner_frac"] = float(u[:, 4].mean())
by_level = {}
for lv in np.unique(u[:, 5]):
    m = u[:, 5] == lv
    by_level[int(lv)] = {"units": int(m.sum()), "items_med": int(np.median(u[m, 3])),
                         "adds_med": int(np.median(u[m, 1])), "drain_med": int(np.median(u[m, 6])),
                         "flush_med": int(np.median(u[m, 7]))}
res["by_level"] = by_level
print(json.dumps(res, indent=1))

# k_grid_bwd_bin: per (point block, level) workgroup, 5 stamps: after the
# counter init, after corners + ranks, after reservation + scan, after
# staging, end
b = stamps[32768:32768 + 16 * 4096].view(-1, 16).cpu().numpy().astype(np.int64)
BP = int(os.environ.get("BIN_PTS", "512"))
gx = (ft.M + BP - 1) // BP  # bin-kernel workgroups per level (kBinPts samples each)
blevel = np.arange(len(b)) // gx
bidx = np.arange(len(b))[b[:, 0] > 0]  # linear workgroup id: XCD = id % 8 (each XCD has its own clock)
blevel = blevel[b[:, 0] > 0]  # workgroups past the sample count leave before stamping
b = b[b[:, 0] > 0]
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "bin_stamps.npz"), b=b, level=blevel, bidx=bidx,
                    acc=st)  # raw clocks for offline timelines
d = np.diff(b[:, :5], axis=1)
if (b[:, 5] > 0).all():  # builds with the in-phase stamps: loads | corners + merge | rank
    d = np.concatenate([np.stack([b[:, 5] - b[:, 0], b[:, 6] - b[:, 5], b[:, 1] - b[:, 6]], 1), d[:, 1:]], 1)
print(json.dumps({"bin_workgroups": int(len(b)),
                  "bin_phase_med": [int(x) for x in np.median(d, axis=0)],
                  "bin_phase_p90": [int(x) for x in np.percentile(d, 90, axis=0)],
                  "bin_phases": (["loads", "corners+merge", "rank"] if d.shape[1] == 6 else ["corners+rank"])
                  + ["reserve+scan", "stage", "write-out"]}))
# chip-wide 100 MHz realtime clock: the bin workgroups' [start, end] (slots
# 8, 9) and the accumulate workgroups' (60, 61), relative to the first bin start
if (b[:, 8] > 0).all() and (st_all[:, 60] > 0).all():
    r0 = b[:, 8].min()
    tl = {"bin_start_us": [round((x - r0) / 100, 2) for x in np.percentile(b[:, 8], [0, 50, 100])],
          "bin_end_us": [round((x - r0) / 100, 2) for x in np.percentile(b[:, 9], [0, 50, 90, 100])],
          "bin_wg_dur_us": [round(x / 100, 2) for x in np.percentile(b[:, 9] - b[:, 8], [10, 50, 90, 100])],
          "acc_start_us": [round((x - r0) / 100, 2) for x in np.percentile(st_all[:, 60], [0, 50, 100])],
          "acc_end_us": [round((x - r0) / 100, 2) for x in np.percentile(st_all[:, 61], [0, 50, 90, 100])]}
    if wr.any():
        for nm, sel in (("wave", wr_all), ("image", ~wr_all)):
            if sel.any():
                tl[nm + "_end_us"] = [round((x - r0) / 100, 2) for x in np.percentile(st_all[sel, 61], [0, 50, 90, 100])]
    # the bin launch's extra columns (XSTAMP: role 0 the MLP dW reduce, role 1
    # the next batch's sampler): start / end per block
    xs = stamps[200000:200000 + 2 * 4096 * 2].view(2, 4096, 2).cpu().numpy().astype(np.int64)
    for role, nm in ((0, "reduce"), (1, "sampler")):
        r = xs[role][xs[role][:, 0] > 0]
        if len(r):
            tl[nm + "_blocks"] = int(len(r))
            tl[nm + "_start_us"] = [round((x - r0) / 100, 2) for x in np.percentile(r[:, 0], [0, 50, 100])]
            tl[nm + "_end_us"] = [round((x - r0) / 100, 2) for x in np.percentile(r[:, 1], [0, 50, 90, 100])]
    print(json.dumps({"timeline": tl}))
per = {}
for lv in np.unique(blevel):
    per[int(lv)] = [int(x) for x in np.median(d[blevel == lv], axis=0)]
print(json.dumps({"bin_phase_med_by_level": per}))

# k_mlp_bwd (sigma NH=1, colour NH=2): per wave, 16 stamps: entry, after the
# fragment image copy, after each chunk, after the loop, after the dW fold,
# after the slab row
if hasattr(lib, "ngp_debug_mlp_stamps"):
    ms.zero_()
    ft.step()
    torch.cuda.synchronize()
    mm = ms[:2 * 2048 * 16].view(2, 2048, 16).cpu().numpy().astype(np.int64)
    out = {}
    for nh, name in ((0, "sigma"), (1, "colour")):
        w = mm[nh][mm[nh][:, 0] > 0]
        chunk_t = []
        for r in w:
            prev = r[1]
            for k in range(2, 12):
                if r[k] == 0:
                    break
                chunk_t.append(r[k] - prev)
                prev = r[k]
        if not chunk_t:
            continue
        out[name] = {"waves": int(len(w)), "frag_copy_med": int(np.median(w[:, 1] - w[:, 0])),
                     "chunk_med": int(np.median(chunk_t)), "chunk_p90": int(np.percentile(chunk_t, 90)),
                     "chunks_per_wave_max": int(max(np.count_nonzero(r[2:12]) for r in w)),
                     "loop_med": int(np.median(w[:, 12] - w[:, 1])), "fold_med": int(np.median(w[:, 13] - w[:, 12])),
                     "slab_med": int(np.median(w[:, 14] - w[:, 13])), "total_med": int(np.median(w[:, 14] - w[:, 0]))}
    print(json.dumps({"mlp_bwd": out}))

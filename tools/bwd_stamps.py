"""Phase clocks of the one-launch NeRF backward (k_nerf_bwd) in the trained
regime (live rows only, options live_rows), diagnostic build with -DNGP_STAMPS
(SRCS=ffmlp bash tools/variants.sh stamps "-DNGP_STAMPS"): per wave and pass,
s_memtime at entry, after the first loads + fragment copy, after each chunk,
after the half chunk, after the fold, after the slab row.
    NGP_HIP_LIB=torch-ngp_amd/variants/stamps/libngp_hip.so python tools/bwd_stamps.py [steps]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _ngp_native as nat  # noqa: E402
import bench  # noqa: E402


def summarize(f, name):
    f = f[f[:, 0] > 0]
    if not len(f):
        return {"pass": name, "waves": 0}
    ent, pre, done_chunks, fold, slab = f[:, 0], f[:, 1], f[:, 12], f[:, 13], f[:, 14]
    # waves that ran a chunk or a half: their chunk phase took time
    work = done_chunks - pre
    return {"pass": name, "waves": int(len(f)),
            "entry_to_loads_med": int(np.median(pre - ent)),
            "chunks_med": int(np.median(work)), "chunks_p90": int(np.percentile(work, 90)),
            "chunks_max": int(work.max()),
            "fold_med": int(np.median(fold - done_chunks)), "slab_med": int(np.median(slab - fold)),
            "total_med": int(np.median(slab - ent)), "total_max": int((slab - ent).max())}


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    argv, sys.argv = sys.argv, sys.argv[:1]
    args = bench.parse()
    sys.argv = argv
    dev = torch.device("cuda:0")
    model, data, bits, *_, dt_gamma = bench.make_workload("lego", dev, 1, 4096)
    ft, _ = bench.make_trainer(args, model, data, 1, dev, dt_gamma, grid_timing=False)
    ms = torch.zeros(3 * 2048 * 16, dtype=torch.int64, device=dev)
    lib = nat.lib()
    assert lib.ngp_debug_mlp_stamps(ctypes.c_void_p(nat.ptr(ms))) == 0
    for _ in range(steps):
        ft.step()
    torch.cuda.synchronize()
    ms.zero_()
    ft.step()
    torch.cuda.synchronize()
    a = ms.view(-1, 16).cpu().numpy().astype(np.int64)
    out = {"steps": steps, "live_frac": ft.live_fraction(), "samples": ft.sample_count(),
           "clock": "s_memtime cycles",
           "sigma": summarize(a[:2048], "sigma"), "color": summarize(a[2048:4096], "color")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

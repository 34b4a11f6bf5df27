"""Histogram of the marched samples per ray after 1,000 bench steps (lego, lego_dense, fox): how many rays a 32- or 16-lane segment of a wave would hold.
    python tools/ray_lengths.py"""
import os, sys
ROOT = "/root/repo" if os.path.exists("/root/repo") else os.getcwd()
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch
import bench
argv, sys.argv = sys.argv, sys.argv[:1]
args = bench.parse(); sys.argv = argv
dev = torch.device("cuda:0")
for w in ("lego", "lego_dense", "fox"):
    m, d, *_, dtg = bench.make_workload(w, dev, 1, args.num_rays)
    ft, _ = bench.make_trainer(args, m, d, 1, dev, dtg, grid_timing=False)
    ft.capture(multi=args.graph_steps)
    ft.run(1000)
    ft.step(); torch.cuda.synchronize()
    ns = ft.rays[:, 2].cpu()
    import numpy as np
    a = ns.numpy()
    print(w, "rays", len(a), "zero", int((a == 0).sum()), "<=16", int(((a > 0) & (a <= 16)).sum()), "17-32", int(((a > 16) & (a <= 32)).sum()),
          "33-64", int(((a > 32) & (a <= 64)).sum()), ">64", int((a > 64).sum()), "mean", float(a.mean()), flush=True)

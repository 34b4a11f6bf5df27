"""Items per bin of the grid backward's bin kernel in the bench's Lego regime
(after `settle` steps): the bin cursors hold the last backward's counts until
the next step's march launch clears them. Prints a histogram of the nonempty
bins' item counts and the share of items in bins up to 64 / 128 / 256 items.
    python tools/bin_hist.py [settle]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    settle = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    argv, sys.argv = sys.argv, sys.argv[:1]
    args = bench.parse()
    sys.argv = argv
    dev = torch.device("cuda:0")
    model, data, bits, *_, dt_gamma = bench.make_workload("lego", dev, 1, args.num_rays)
    ft, _ = bench.make_trainer(args, model, data, 1, dev, dt_gamma, grid_timing=False)
    ft.capture(multi=args.graph_steps)
    ft.run(settle)
    out = []
    for _ in range(4):
        ft.step()
        torch.cuda.synchronize()
        c = ft.grid_ws[:ft._grid_counter_bytes].view(torch.int32).cpu().numpy().astype(np.int64)
        out.append(c)
    c = np.concatenate(out)
    nz = c[c > 0]
    res = {"settle": settle, "bins": int(len(out[0])), "nonempty_per_step": round(len(nz) / 4, 1),
           "items_per_step": round(float(nz.sum()) / 4, 1),
           "quantiles": {q: int(np.quantile(nz, q)) for q in (0.1, 0.25, 0.5, 0.75, 0.9, 0.99)},
           "max": int(nz.max())}
    for lim in (64, 128, 256, 512):
        res[f"bins_le_{lim}"] = round(float((nz <= lim).mean()), 4)
        res[f"items_in_bins_le_{lim}"] = round(float(nz[nz <= lim].sum() / nz.sum()), 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

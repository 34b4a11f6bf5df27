"""Kernel makeup of the partial density-grid update (FusedTrainer.update_density
after 16 full ones) on the bench's Lego workload: run it under
`rocprofv3 --kernel-trace --stats` and read the per-kernel stats; the script
prints the mean wall time of `reps` updates each followed by a training step
(the bench's cadence work between two updates is 16 steps).
    rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 tools/density_trace.py [reps] [options-json]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    opts = json.loads(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2] else None
    argv, sys.argv = sys.argv, sys.argv[:1]
    args = bench.parse()
    sys.argv = argv
    dev = torch.device("cuda:0")
    model, data, bits, *_, dt_gamma = bench.make_workload("lego", dev, 1, args.num_rays)
    ft, _ = bench.make_trainer(args, model, data, 1, dev, dt_gamma, grid_timing=False, options=opts)
    ft.capture(multi=args.graph_steps)
    ft.run(200)
    while model.iter_density < 16:
        ft.update_density()
        ft.run(2)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        ft.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ft.update_density()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"partial update wall ms: median {1e3 * ts[len(ts) // 2]:.3f} min {1e3 * ts[0]:.3f}", flush=True)


if __name__ == "__main__":
    main()

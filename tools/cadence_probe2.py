"""The bench's density cadence (`with_density_update`) in the bench's own order
-- trainer with the grid timing ring, timed region, eager body steps, the
density update timings, then the cadence twice -- and a trainer without the
timing ring that goes straight to the cadence, to find which precondition
makes the unsynchronised cycles slower than their synchronised parts.

    python tools/cadence_probe2.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    args = bench.parse()
    dev = torch.device("cuda:0")
    out = {}
    model, data, bits, *_, dt_gamma = bench.make_workload("lego", dev, 1, 4096)
    ft, _ = bench.make_trainer(args, model, data, 1, dev, dt_gamma, grid_timing=True)
    bench.timed_run(args, ft, 1, dev, 20, 5, args.settle_steps, args.graph_steps)
    out["a_cadence_after_timed_run"] = bench.density_cadence(ft, bits, args)
    ft.timed_body_steps(args.kernel_steps)
    out["b_after_body_steps"] = bench.density_cadence(ft, bits, args)
    out["density_update_times"] = bench.density_update_times(model, bits, ft)
    out["c_after_update_times"] = bench.density_cadence(ft, bits, args)
    out["d_again"] = bench.density_cadence(ft, bits, args)
    del ft, model
    torch.cuda.empty_cache()
    model, data, bits, *_, dt_gamma = bench.make_workload("lego", dev, 1, 4096)
    ft, _ = bench.make_trainer(args, model, data, 1, dev, dt_gamma, grid_timing=False)
    bench.timed_run(args, ft, 1, dev, 20, 5, args.settle_steps, args.graph_steps)
    out["e_no_timing_ring"] = bench.density_cadence(ft, bits, args)
    for k, v in out.items():
        print(k, json.dumps(v))


if __name__ == "__main__":
    main()

"""Same-box A/B of FusedTrainer attributes on the bench's density cadence line
(bench.density_cadence: 6 x [partial update_density + fixture restore +
run(16)]), alternating rounds. Prints ms/step and the synced parts per cycle.
    python tools/cadence_ab.py '{"_dens_sorted": false}' [rounds]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    variant = json.loads(sys.argv[1])
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    argv, sys.argv = sys.argv, sys.argv[:1]
    args = bench.parse()
    sys.argv = argv
    dev = torch.device("cuda:0")
    model, data, bits, *_, dt_gamma = bench.make_workload("lego", dev, 1, args.num_rays)
    ft, _ = bench.make_trainer(args, model, data, 1, dev, dt_gamma, grid_timing=False)
    bench.timed_run(args, ft, 1, dev, 50, 5, 300, args.graph_steps)
    base = {k: getattr(ft, k) for k in variant}
    for r in range(rounds):
        for name, attrs in (("base", base), ("variant", variant)):
            for k, v in attrs.items():
                setattr(ft, k, v)
            ft.capture(warmup=0, multi=args.graph_steps)  # the graphs again, in this form
            c = bench.density_cadence(ft, bits, args)
            print(r, name, c["ms_per_step"], c["parts_ms_per_cycle_synced"], flush=True)


if __name__ == "__main__":
    main()

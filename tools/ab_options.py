"""Same-box A/B of FusedTrainer options (per-trainer `options=`) on bench
workloads: for each workload, alternating rounds of [baseline, variant] timed
runs (bench.timed_run: warmup, capture, clock settle, `steps` graph steps),
ms/step each, plus the eager per-launch times of the step body.
    python tools/ab_options.py '{"table16": true}' [lego,lego_dense] [rounds] [steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    variant = json.loads(sys.argv[1])
    workloads = (sys.argv[2] if len(sys.argv) > 2 else "lego,lego_dense").split(",")
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 200
    argv, sys.argv = sys.argv, sys.argv[:1]
    args = bench.parse()
    sys.argv = argv
    dev = torch.device("cuda:0")
    out = {"variant": variant, "steps": steps, "runs": []}
    for w in workloads:
        for r in range(rounds):
            for name, opts in (("base", None), ("variant", variant)):
                model, data, bits, *_, dt_gamma = bench.make_workload(w, dev, 1, args.num_rays)
                ft, _ = bench.make_trainer(args, model, data, 1, dev, dt_gamma, grid_timing=False, options=opts)
                el, used_graph, _ = bench.timed_run(args, ft, 1, dev, steps, 5, 300, args.graph_steps)
                ms = el / steps * 1e3
                per, _, _ = ft.timed_body_steps(8)
                out["runs"].append({"workload": w, "round": r, "name": name, "ms_per_step": round(ms, 4),
                                    "graph": used_graph, "body_ms": {k: round(v, 4) for k, v in per.items()}})
                print(w, r, name, round(ms, 4), {k: round(v * 1e3, 1) for k, v in per.items()}, flush=True)
                del ft, model
                torch.cuda.empty_cache()
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "ab_options.json"), "w"), indent=1)


if __name__ == "__main__":
    main()

"""How much of the Adam sweep is idle: the share of table entries whose
moments are still exactly zero (never touched: Adam leaves p, m, v as they
are) and whose gradient is zero in a step, on the bench's Lego workload after
increasing numbers of training steps. Prints one JSON object.
    python tools/adam_idle_frac.py [steps,...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    marks = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "300,1000,3000").split(",")]
    argv, sys.argv = sys.argv, sys.argv[:1]
    args = bench.parse()
    sys.argv = argv
    dev = torch.device("cuda:0")
    model, data, bits, *_, dt_gamma = bench.make_workload("lego", dev, 1, args.num_rays)
    ft, _ = bench.make_trainer(args, model, data, 1, dev, dt_gamma, grid_timing=False)
    ft.capture(multi=args.graph_steps)
    done, out = 0, {}
    for mark in marks:
        while done < mark:
            n = min(64, mark - done)
            ft.run(n)
            done += n
            if done % 640 < 64:  # the bench's density cadence, roughly
                ft.update_density()
                ft.refresh_occupancy()
        ft.step()  # leaves this step's gradient pending
        torch.cuda.synchronize()
        n_tab = ft.params[0].numel()
        g = ft.flat_grad[:n_tab]
        zero_g = float((g == 0).float().mean())
        ft.flush()
        m, v = ft.exp_avg[:n_tab], ft.exp_avg_sq[:n_tab]
        idle = float(((m == 0) & (v == 0)).float().mean())
        out[mark] = {"table_entries": n_tab, "moments_zero": round(idle, 4), "grad_zero": round(zero_g, 4)}
        print(mark, out[mark], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

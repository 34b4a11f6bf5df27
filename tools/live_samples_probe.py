"""How many of a step's samples carry a nonzero gradient as the Lego bench
trains (samples behind a ray's early termination, T < T_thresh, get none:
the reference's composite backward stops there too)? Counts rows of the
composite's output gradients (g_h column 0 = the density gradient, g_color_out
= the colour logits' gradient) after 0..N steps.

    python tools/live_samples_probe.py
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
    model, data, bits, *_, dt_gamma = bench.make_workload("lego", dev, 1, 4096)
    ft, _ = bench.make_trainer(args, model, data, 1, dev, dt_gamma, grid_timing=False)
    out = []
    done = 0
    for target in (1, 10, 100, 300, 1000, 2000):
        while done < target:
            ft.step()
            done += 1
        torch.cuda.synchronize()
        n = ft.sample_count()
        gh = ft.g_h[:n].float()
        gc = ft.g_color_out[:n].float()
        ge = ft.g_enc.view(-1, 2)  # [16][M][2]
        live_sigma = int((gh[:, 0] != 0).sum())
        live_color = int((gc != 0).any(dim=1).sum())
        live_any = int(((gh != 0).any(dim=1) | (gc != 0).any(dim=1)).sum())
        enc = ft.g_enc.view(16, -1, 2)[:, :n].float()
        live_enc = int((enc != 0).any(dim=2).any(dim=0).sum())
        out.append({"steps": done, "samples": n, "live_sigma_grad": live_sigma, "live_color_grad": live_color,
                    "live_any": live_any, "live_enc_grad": live_enc, "live_frac": round(live_any / max(n, 1), 4),
                    "loss": ft.last_loss})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()

"""Test-image rendering speed: the reference's inference
path, run_cuda with training off (renderer.py:376-426: march_rays /
network / composite_rays over the alive rays, compacted each iteration),
one 800x800 synthetic-Lego image per iteration. The reference's published
figure is 7.8 it/s on a V100 (readme.md:211).

    python tools/render_bench.py [--train-steps 300] [--images 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch  # noqa: E402

from nerf.fused import FusedTrainer  # noqa: E402
from nerf.network_ff import NeRFNetwork  # noqa: E402
from nerf.provider import SyntheticLego, lego_bitfield  # noqa: E402
from nerf.utils import get_rays  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--train-steps", type=int, default=300)
    ap.add_argument("--images", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = NeRFNetwork(bound=1, cuda_ray=True).to(dev)
    model.density_bitfield.copy_(torch.from_numpy(lego_bitfield()).to(dev))
    data = SyntheticLego(dev, num_rays=4096)
    ft = FusedTrainer(model, data, M=101762)
    for _ in range(a.train_steps):  # a partly trained field, so rays terminate as in a test render
        ft.step()
    ft.flush()
    torch.cuda.synchronize()
    model.eval()
    pose = data.poses[7:8]
    rays = get_rays(pose, data.intrinsics, data.H, data.W, -1)
    times, iters = [], None
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        for k in range(a.warmup + a.images):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = model.render(rays["rays_o"], rays["rays_d"], staged=True, bg_color=1, perturb=False,
                               dt_gamma=0.0, max_steps=1024)
            torch.cuda.synchronize()
            if k >= a.warmup:
                times.append(time.perf_counter() - t0)
    img = out["image"].float()
    res = {"metric": "test render it/s (one 800x800 image per it, inference march/composite loop)",
           "value": round(len(times) / sum(times), 3), "unit": "it/s",
           "ms_per_image": round(1e3 * sum(times) / len(times), 2), "images": len(times),
           "train_steps_before": a.train_steps, "image_mean": round(float(img.mean()), 4),
           "image_finite": bool(torch.isfinite(img).all()),
           "baseline_ref": "V100 7.8 it/s test speed (readme.md:211)"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()

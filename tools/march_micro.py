"""Micro-benchmark of march_rays_train on the bench workload (4096 Lego rays,
analytic bitfield fixture, perturb): HIP events over back-to-back calls.
    python tools/march_micro.py [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch  # noqa: E402

import raymarching  # noqa: E402
from nerf.provider import SyntheticLego, lego_bitfield  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
dev = torch.device("cuda:0")
torch.manual_seed(0)
data = SyntheticLego(dev, num_rays=N)
batch = data.sample()
rays_o, rays_d = batch["rays_o"].view(-1, 3), batch["rays_d"].view(-1, 3)
aabb = torch.tensor([-1, -1, -1, 1, 1, 1.0], device=dev)
bits = torch.from_numpy(lego_bitfield()).to(dev)
nears, fars = raymarching.near_far_from_aabb(rays_o, rays_d, aabb, 0.2)
counter = torch.zeros(16, 2, dtype=torch.int32, device=dev)


def run():
    counter.zero_()
    return raymarching.march_rays_train(rays_o, rays_d, 1.0, bits, 1, 128, nears, fars, counter[0],
                                        120000, True, 128, False, 0.0, 1024)


for _ in range(3):
    out = run()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20):
    run()
e.record()
torch.cuda.synchronize()
print({"N": N, "samples": int(counter[0, 0].item()), "march_rays_train_us": round(s.elapsed_time(e) / 20 * 1e3, 1)})

"""Config 1: the pure-PyTorch CPU NeRF train step -- TEST INFRASTRUCTURE /
CPU BASELINE ONLY (bench.py's cpu_baseline leg and tests/ import it).

BASELINE.json configs[0] is "nerf_synthetic/lego 200x200 fp32 on CPU: PyTorch
ray marching (no --cuda_ray), torch.nn MLP, encoding.py hashgrid". The
reference has no CPU-capable path (near_far_from_aabb and the hash grid are
CUDA-only), so this module restates it in torch ops:

  * near_far_from_aabb          raymarching.cu:91-145 (slab test, min_near)
  * hash-grid encoder           gridencoder.cu:87-242 (fp32, linear interp,
                                hash / dense index, offsets of grid.py:776-789),
                                autograd supplies kernel_grid_backward's scatter
  * SH degree 4                 shencoder.cu:49-121
  * sigma / colour MLPs         nerf/network.py:63-105 (nn.Linear, bias-free,
                                ReLU; 32-64-16 and 31-64-64-3)
  * run()                       nerf/renderer.py:126-254 (uniform sampling,
                                num_steps 512, upsample_steps 0, perturb)
  * train step                  nerf/utils.py:453-497 (random background,
                                MSE .mean(-1).mean()), Adam(0.9, 0.99, 1e-15)
"""
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

_PRIMES = (1, 2654435761, 805459861)


def near_far_from_aabb(rays_o, rays_d, aabb, min_near=0.2):
    """raymarching.cu:91-145 in torch (misses: near = far = FLT_MAX)."""
    inv = 1.0 / rays_d
    t0 = (aabb[:3] - rays_o) * inv
    t1 = (aabb[3:] - rays_o) * inv
    tmin = torch.minimum(t0, t1)
    tmax = torch.maximum(t0, t1)
    near = tmin.amax(-1)
    far = tmax.amin(-1)
    miss = near > far
    big = torch.full_like(near, 3.4028234663852886e38)
    near = torch.where(miss, big, torch.clamp(near, min=min_near))
    far = torch.where(miss, big, far)
    return near, far


class TorchHashGrid(nn.Module):
    """GridEncoder (hash, linear, align_corners=False) in torch ops."""

    def __init__(self, num_levels=16, level_dim=2, base_resolution=16, log2_hashmap_size=19,
                 desired_resolution=2048):
        super().__init__()
        self.L, self.C, self.H = num_levels, level_dim, base_resolution
        self.per_level_scale = float(np.exp2(np.log2(desired_resolution / base_resolution) / (num_levels - 1)))
        offsets, off = [], 0
        for i in range(num_levels):
            res = int(np.ceil(base_resolution * self.per_level_scale ** i))
            n = int(np.ceil(min(2 ** log2_hashmap_size, (res + 1) ** 3) / 8) * 8)
            offsets.append(off)
            off += n
        offsets.append(off)
        self.offsets = offsets
        self.embeddings = nn.Parameter(torch.empty(off, level_dim).uniform_(-1e-4, 1e-4))
        S = np.float32(np.log2(self.per_level_scale))
        # gridencoder.cu:138-139: scale = exp2f(l * S) * H - 1, res = ceil(scale) + 1
        self.scales = [float(np.float32(np.exp2(np.float64(np.float32(l * S)))) * np.float32(base_resolution)
                             - np.float32(1.0)) for l in range(num_levels)]
        self.res = [int(math.ceil(s)) + 1 for s in self.scales]
        self.output_dim = num_levels * level_dim

    def forward(self, x, bound=1.0):
        x = (x + bound) / (2 * bound)
        outs = []
        for l in range(self.L):
            hs = self.offsets[l + 1] - self.offsets[l]
            res = self.res[l]
            pos = x * self.scales[l] + 0.5
            pg = torch.floor(pos)
            frac = pos - pg
            pg = pg.long()
            dense = (res + 1) ** 3 <= hs
            acc = 0
            for idx in range(8):
                w = 1
                corner = []
                for d in range(3):
                    bit = (idx >> d) & 1
                    w = w * (frac[:, d] if bit else 1 - frac[:, d])
                    corner.append(pg[:, d] + bit)
                if dense:
                    e = corner[0] + corner[1] * (res + 1) + corner[2] * (res + 1) ** 2
                else:
                    e = ((corner[0] * _PRIMES[0]) ^ (corner[1] * _PRIMES[1]) ^ (corner[2] * _PRIMES[2])) & 0xFFFFFFFF
                e = e % hs + self.offsets[l]
                acc = acc + w[:, None] * self.embeddings.index_select(0, e)
            outs.append(acc)
        return torch.cat(outs, -1)


def sh_encode4(d):
    """Degree-4 real SH (16 values), shencoder.cu:49-121."""
    x, y, z = d[:, 0], d[:, 1], d[:, 2]
    xy, xz, yz, x2, y2, z2 = x * y, x * z, y * z, x * x, y * y, z * z
    return torch.stack([
        torch.full_like(x, 0.28209479177387814), -0.48860251190291987 * y, 0.48860251190291987 * z,
        -0.48860251190291987 * x, 1.0925484305920792 * xy, -1.0925484305920792 * yz,
        0.94617469575755997 * z2 - 0.31539156525251999, -1.0925484305920792 * xz,
        0.54627421529603959 * x2 - 0.54627421529603959 * y2, 0.59004358992664352 * y * (-3.0 * x2 + y2),
        2.8906114426405538 * xy * z, 0.45704579946446572 * y * (1.0 - 5.0 * z2),
        0.3731763325901154 * z * (5.0 * z2 - 3.0), 0.45704579946446572 * x * (1.0 - 5.0 * z2),
        1.4453057213202769 * z * (x2 - y2), 0.59004358992664352 * x * (-x2 + 3.0 * y2)], -1)


class _TruncExp(torch.autograd.Function):  # activation.py:5-18
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return torch.exp(x)

    @staticmethod
    def backward(ctx, g):
        x, = ctx.saved_tensors
        return g * torch.exp(x.clamp(-15, 15))


class TorchNeRF(nn.Module):
    """nerf/network.py's NeRFNetwork (hashgrid + SH + bias-free nn.Linear MLPs)."""

    def __init__(self, bound=1.0, num_steps=512):
        super().__init__()
        self.bound, self.num_steps, self.min_near, self.density_scale = bound, num_steps, 0.2, 1.0
        self.encoder = TorchHashGrid(desired_resolution=2048 * bound)
        self.sigma_net = nn.Sequential(nn.Linear(32, 64, bias=False), nn.ReLU(), nn.Linear(64, 16, bias=False))
        self.color_net = nn.Sequential(nn.Linear(31, 64, bias=False), nn.ReLU(), nn.Linear(64, 64, bias=False),
                                       nn.ReLU(), nn.Linear(64, 3, bias=False))
        self.register_buffer("aabb", torch.tensor([-bound] * 3 + [bound] * 3, dtype=torch.float32))

    def run(self, rays_o, rays_d, bg_color, perturb=True):
        """renderer.py:126-254 with upsample_steps = 0."""
        N, T = rays_o.shape[0], self.num_steps
        nears, fars = near_far_from_aabb(rays_o, rays_d, self.aabb, self.min_near)
        nears, fars = nears[:, None], fars[:, None]
        z = nears + (fars - nears) * torch.linspace(0.0, 1.0, T)[None]
        sample_dist = (fars - nears) / T
        if perturb:
            z = z + (torch.rand(z.shape) - 0.5) * sample_dist
        xyzs = rays_o[:, None] + rays_d[:, None] * z[..., None]
        xyzs = torch.min(torch.max(xyzs, self.aabb[:3]), self.aabb[3:])
        h = self.sigma_net(self.encoder(xyzs.reshape(-1, 3), bound=self.bound))
        sigma = _TruncExp.apply(h[:, 0]).view(N, T)
        deltas = torch.cat([z[:, 1:] - z[:, :-1], sample_dist], -1)
        alphas = 1 - torch.exp(-deltas * self.density_scale * sigma)
        shifted = torch.cat([torch.ones_like(alphas[:, :1]), 1 - alphas + 1e-15], -1)
        weights = alphas * torch.cumprod(shifted, -1)[:, :-1]
        d = rays_d[:, None].expand(N, T, 3).reshape(-1, 3)
        rgbs = torch.sigmoid(self.color_net(torch.cat([sh_encode4(d), h[:, 1:]], -1))).view(N, T, 3)
        ws = weights.sum(-1)
        image = (weights[..., None] * rgbs).sum(-2)
        return image + (1 - ws)[:, None] * bg_color


def train_step(model, opt, rays_o, rays_d, rgba):
    """One iteration of nerf/utils.py train_step (:453-497) on CPU tensors."""
    bg = torch.rand(rays_o.shape[0], 3)
    gt = rgba[:, :3] * rgba[:, 3:] + bg * (1 - rgba[:, 3:])
    pred = model.run(rays_o, rays_d, bg)
    loss = F.mse_loss(pred, gt, reduction="none").mean(-1).mean()
    opt.zero_grad(set_to_none=True)
    loss.backward()
    opt.step()
    return float(loss.detach())


def lego_batches(n_batches, num_rays=4096, H=200, W=200, seed=0):
    """Rays of the synthetic Lego scene (nerf.provider.SyntheticLego geometry)
    at H x W, drawn on the CPU: (rays_o, rays_d, rgba) per batch."""
    import sys
    import os
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "torch-ngp_amd")
    if pkg not in sys.path:
        sys.path.insert(0, pkg)
    from nerf.provider import SyntheticLego
    from nerf.utils import get_rays
    data = SyntheticLego(torch.device("cpu"), H=H, W=W, num_rays=num_rays)
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n_batches):
        k = int(torch.randint(0, data.poses.shape[0], (1,), generator=g))
        rays = get_rays(data.poses[k:k + 1], data.intrinsics, H, W, num_rays, generator=g)
        ro, rd = rays["rays_o"][0].contiguous(), rays["rays_d"][0].contiguous()
        out.append((ro, rd, data.target(ro, rd)))
    return out


def time_train_steps(threads, budget_s=20.0, warmup=1, max_steps=5, num_rays=4096, seed=0):
    """Config 1 timed on `threads` host threads: rays/s over the timed steps
    (at least one; stops once the budget is spent)."""
    import time
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        torch.manual_seed(seed)
        model = TorchNeRF()
        opt = torch.optim.Adam(model.parameters(), lr=1e-2, betas=(0.9, 0.99), eps=1e-15)
        batches = lego_batches(warmup + max_steps, num_rays=num_rays, seed=seed)
        for b in batches[:warmup]:
            train_step(model, opt, *b)
        t0 = time.perf_counter()
        steps = 0
        losses = []
        for b in batches[warmup:]:
            losses.append(train_step(model, opt, *b))
            steps += 1
            if time.perf_counter() - t0 > budget_s:
                break
        dt = time.perf_counter() - t0
    finally:
        torch.set_num_threads(prev)
    return steps * num_rays / dt, steps, dt, losses

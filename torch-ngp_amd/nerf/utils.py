"""get_rays + a slim trainer around the hot path (reference nerf/utils.py:52-136,
453-609, 912-1072). Only what the train step needs: AMP, Adam(0.9, 0.99,
1e-15), LambdaLR 0.1^(iter/iters), density-grid update every 16 steps,
MSE on RGB with a pixel-wise random background for RGBA targets, optional
ray-sharded data parallelism (torch.distributed, RCCL)."""
import torch


def custom_meshgrid(*args):
    return torch.meshgrid(*args, indexing="ij")


@torch.amp.autocast("cuda", enabled=False)
def get_rays(poses, intrinsics, H, W, N=-1, error_map=None, patch_size=1, generator=None):
    """poses [B, 4, 4] cam2world -> rays_o, rays_d [B, N, 3], inds [B, N]."""
    device = poses.device
    B = poses.shape[0]
    fx, fy, cx, cy = [float(v) for v in intrinsics]
    results = {}
    if N > 0:
        N = min(N, H * W)
        if patch_size > 1:
            num_patch = N // (patch_size ** 2)
            ix = torch.randint(0, H - patch_size, size=[num_patch], device=device, generator=generator)
            iy = torch.randint(0, W - patch_size, size=[num_patch], device=device, generator=generator)
            inds = torch.stack([ix, iy], dim=-1)
            pi, pj = custom_meshgrid(torch.arange(patch_size, device=device),
                                     torch.arange(patch_size, device=device))
            offsets = torch.stack([pi.reshape(-1), pj.reshape(-1)], dim=-1)
            inds = (inds.unsqueeze(1) + offsets.unsqueeze(0)).view(-1, 2)
            inds = (inds[:, 0] * W + inds[:, 1]).expand([B, N])
        else:
            inds = torch.randint(0, H * W, size=[N], device=device, generator=generator).expand([B, N])
        results["inds"] = inds
    else:
        inds = torch.arange(H * W, device=device).expand([B, H * W])
    i = (inds % W).float() + 0.5
    j = torch.div(inds, W, rounding_mode="floor").float() + 0.5
    zs = torch.ones_like(i)
    xs = (i - cx) / fx * zs
    ys = (j - cy) / fy * zs
    directions = torch.stack((xs, ys, zs), dim=-1)
    directions = directions / torch.norm(directions, dim=-1, keepdim=True)
    rays_d = directions @ poses[:, :3, :3].transpose(-1, -2)
    rays_o = poses[..., :3, 3][..., None, :].expand_as(rays_d)
    results["rays_o"] = rays_o
    results["rays_d"] = rays_d
    return results

"""Ray-marching autograd ops (mirror of the reference raymarching/raymarching.py).

Same public functions, arguments, defaults and return values as the
reference (:19-374). The kernels behind `_backend` are the gfx950 HIP ones in
csrc/raymarching.hip; the only observable difference is that
`march_rays_train` lays rays out in ray order (deterministic offsets) where
the reference's atomics give a run-dependent order (raymarching.cu:405-406).
"""
import torch
from torch.autograd import Function

from .backend import _backend

_fwd32 = torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
_bwd = torch.amp.custom_bwd(device_type="cuda")


class _near_far_from_aabb(Function):
    @staticmethod
    @_fwd32
    def forward(ctx, rays_o, rays_d, aabb, min_near=0.2):
        """rays_o/rays_d [N, 3], aabb [6] -> nears, fars [N] (miss: FLT_MAX)."""
        if not rays_o.is_cuda: rays_o = rays_o.cuda()
        if not rays_d.is_cuda: rays_d = rays_d.cuda()
        rays_o = rays_o.contiguous().view(-1, 3)
        rays_d = rays_d.contiguous().view(-1, 3)
        N = rays_o.shape[0]
        nears = torch.empty(N, dtype=rays_o.dtype, device=rays_o.device)
        fars = torch.empty(N, dtype=rays_o.dtype, device=rays_o.device)
        _backend.near_far_from_aabb(rays_o, rays_d, aabb.contiguous(), N, min_near, nears, fars)
        return nears, fars


near_far_from_aabb = _near_far_from_aabb.apply


class _sph_from_ray(Function):
    @staticmethod
    @_fwd32
    def forward(ctx, rays_o, rays_d, radius):
        """Background-sphere coordinates in [-1, 1]^2, [N, 2]."""
        if not rays_o.is_cuda: rays_o = rays_o.cuda()
        if not rays_d.is_cuda: rays_d = rays_d.cuda()
        rays_o = rays_o.contiguous().view(-1, 3)
        rays_d = rays_d.contiguous().view(-1, 3)
        N = rays_o.shape[0]
        coords = torch.empty(N, 2, dtype=rays_o.dtype, device=rays_o.device)
        _backend.sph_from_ray(rays_o, rays_d, radius, N, coords)
        return coords


sph_from_ray = _sph_from_ray.apply


class _morton3D(Function):
    @staticmethod
    def forward(ctx, coords):
        """coords int32 [N, 3] in [0, 128) -> Morton indices int32 [N]."""
        if not coords.is_cuda: coords = coords.cuda()
        N = coords.shape[0]
        indices = torch.empty(N, dtype=torch.int32, device=coords.device)
        _backend.morton3D(coords.int().contiguous(), N, indices)
        return indices


morton3D = _morton3D.apply


class _morton3D_invert(Function):
    @staticmethod
    def forward(ctx, indices):
        """Morton indices int32 [N] -> coords int32 [N, 3]."""
        if not indices.is_cuda: indices = indices.cuda()
        N = indices.shape[0]
        coords = torch.empty(N, 3, dtype=torch.int32, device=indices.device)
        _backend.morton3D_invert(indices.int().contiguous(), N, coords)
        return coords


morton3D_invert = _morton3D_invert.apply


class _packbits(Function):
    @staticmethod
    @_fwd32
    def forward(ctx, grid, thresh, bitfield=None):
        """density grid [C, H^3] float -> occupancy bitfield uint8 [C * H^3 / 8]."""
        if not grid.is_cuda: grid = grid.cuda()
        grid = grid.contiguous()
        C = grid.shape[0]
        H3 = grid.shape[1]
        N = C * H3 // 8
        if bitfield is None:
            bitfield = torch.empty(N, dtype=torch.uint8, device=grid.device)
        _backend.packbits(grid, N, thresh, bitfield)
        return bitfield


packbits = _packbits.apply


class _march_rays_train(Function):
    @staticmethod
    @_fwd32
    def forward(ctx, rays_o, rays_d, bound, density_bitfield, C, H, nears, fars, step_counter=None,
                mean_count=-1, perturb=False, align=-1, force_all_rays=False, dt_gamma=0,
                max_steps=1024):
        """March rays through the occupancy bitfield (reference raymarching.py:161-235).

        Returns xyzs [M, 3], dirs [M, 3], deltas [M, 2], rays int32 [N, 3] =
        (ray index, point offset, point count)."""
        if not rays_o.is_cuda: rays_o = rays_o.cuda()
        if not rays_d.is_cuda: rays_d = rays_d.cuda()
        if not density_bitfield.is_cuda: density_bitfield = density_bitfield.cuda()
        rays_o = rays_o.contiguous().view(-1, 3)
        rays_d = rays_d.contiguous().view(-1, 3)
        density_bitfield = density_bitfield.contiguous()

        N = rays_o.shape[0]
        M = N * max_steps
        # running-average sizing (raymarching.py:198-203)
        if not force_all_rays and mean_count > 0:
            if align > 0:
                mean_count += align - mean_count % align
            M = mean_count

        xyzs = torch.zeros(M, 3, dtype=rays_o.dtype, device=rays_o.device)
        dirs = torch.zeros(M, 3, dtype=rays_o.dtype, device=rays_o.device)
        deltas = torch.zeros(M, 2, dtype=rays_o.dtype, device=rays_o.device)
        rays = torch.empty(N, 3, dtype=torch.int32, device=rays_o.device)
        if step_counter is None:
            step_counter = torch.zeros(2, dtype=torch.int32, device=rays_o.device)
        if perturb:
            noises = torch.rand(N, dtype=rays_o.dtype, device=rays_o.device)
        else:
            noises = torch.zeros(N, dtype=rays_o.dtype, device=rays_o.device)

        _backend.march_rays_train(rays_o, rays_d, density_bitfield, bound, dt_gamma, max_steps, N, C,
                                  H, M, nears, fars, xyzs, dirs, deltas, rays, step_counter, noises)

        if force_all_rays or mean_count <= 0:
            m = step_counter[0].item()  # D2H copy, as in the reference (:224)
            if align > 0:
                m += align - m % align
            xyzs = xyzs[:m]
            dirs = dirs[:m]
            deltas = deltas[:m]
        return xyzs, dirs, deltas, rays


march_rays_train = _march_rays_train.apply


class _composite_rays_train(Function):
    @staticmethod
    @_fwd32
    def forward(ctx, sigmas, rgbs, deltas, rays, T_thresh=1e-4):
        """Front-to-back compositing -> weights_sum [N], depth [N], image [N, 3]."""
        sigmas = sigmas.contiguous()
        rgbs = rgbs.contiguous()
        deltas = deltas.contiguous()
        M = sigmas.shape[0]
        N = rays.shape[0]
        weights_sum = torch.empty(N, dtype=sigmas.dtype, device=sigmas.device)
        depth = torch.empty(N, dtype=sigmas.dtype, device=sigmas.device)
        image = torch.empty(N, 3, dtype=sigmas.dtype, device=sigmas.device)
        _backend.composite_rays_train_forward(sigmas, rgbs, deltas, rays, M, N, T_thresh,
                                              weights_sum, depth, image)
        ctx.save_for_backward(sigmas, rgbs, deltas, rays, weights_sum, depth, image)
        ctx.dims = [M, N, T_thresh]
        return weights_sum, depth, image

    @staticmethod
    @_bwd
    def backward(ctx, grad_weights_sum, grad_depth, grad_image):
        grad_weights_sum = grad_weights_sum.contiguous()
        grad_depth = grad_depth.contiguous()
        grad_image = grad_image.contiguous()
        sigmas, rgbs, deltas, rays, weights_sum, depth, image = ctx.saved_tensors
        M, N, T_thresh = ctx.dims
        grad_sigmas = torch.zeros_like(sigmas)
        grad_rgbs = torch.zeros_like(rgbs)
        _backend.composite_rays_train_backward(grad_weights_sum, grad_depth, grad_image, sigmas,
                                               rgbs, deltas, rays, weights_sum, depth, image, M, N,
                                               T_thresh, grad_sigmas, grad_rgbs)
        return grad_sigmas, grad_rgbs, None, None, None


composite_rays_train = _composite_rays_train.apply


class _march_rays(Function):
    @staticmethod
    @_fwd32
    def forward(ctx, n_alive, n_step, rays_alive, rays_t, rays_o, rays_d, bound, density_bitfield,
                C, H, near, far, align=-1, perturb=False, dt_gamma=0, max_steps=1024):
        """Inference marching: n_step samples for each alive ray (raymarching.py:298-349)."""
        if not rays_o.is_cuda: rays_o = rays_o.cuda()
        if not rays_d.is_cuda: rays_d = rays_d.cuda()
        rays_o = rays_o.contiguous().view(-1, 3)
        rays_d = rays_d.contiguous().view(-1, 3)
        M = n_alive * n_step
        if align > 0:
            M += align - (M % align)
        xyzs = torch.zeros(M, 3, dtype=rays_o.dtype, device=rays_o.device)
        dirs = torch.zeros(M, 3, dtype=rays_o.dtype, device=rays_o.device)
        deltas = torch.zeros(M, 2, dtype=rays_o.dtype, device=rays_o.device)
        if perturb:
            noises = torch.rand(n_alive, dtype=rays_o.dtype, device=rays_o.device)
        else:
            noises = torch.zeros(n_alive, dtype=rays_o.dtype, device=rays_o.device)
        _backend.march_rays(n_alive, n_step, rays_alive, rays_t, rays_o, rays_d, bound, dt_gamma,
                            max_steps, C, H, density_bitfield, near, far, xyzs, dirs, deltas, noises)
        return xyzs, dirs, deltas


march_rays = _march_rays.apply


class _composite_rays(Function):
    @staticmethod
    @_fwd32
    def forward(ctx, n_alive, n_step, rays_alive, rays_t, sigmas, rgbs, deltas, weights_sum, depth,
                image, T_thresh=1e-2):
        """In-place inference compositing; terminated rays get rays_alive = -1."""
        _backend.composite_rays(n_alive, n_step, T_thresh, rays_alive, rays_t, sigmas.contiguous(),
                                rgbs.contiguous(), deltas.contiguous(), weights_sum, depth, image)
        return tuple()


composite_rays = _composite_rays.apply

__all__ = ["near_far_from_aabb", "sph_from_ray", "morton3D", "morton3D_invert", "packbits",
           "march_rays_train", "composite_rays_train", "march_rays", "composite_rays"]

"""`_backend` for raymarching: the reference's pybind11 surface
(raymarching/src/bindings.cpp:5-18, raymarching.h:7-18) bound to
libngp_hip.so via ctypes. Same names, positional arguments and in-place
outputs; float32 tensors only (every reference wrapper casts to float32).
"""
import types

import torch

import _ngp_native as nat

_F = (torch.float32,)
_I = (torch.int32,)
_U8 = (torch.uint8,)


def _f(t, name):
    nat.check_tensor(t, name, _F, "float32")


def _i(t, name):
    nat.check_tensor(t, name, _I, "int")


def near_far_from_aabb(rays_o, rays_d, aabb, N, min_near, nears, fars):
    for t, n in ((rays_o, "rays_o"), (rays_d, "rays_d"), (aabb, "aabb"), (nears, "nears"), (fars, "fars")):
        _f(t, n)
    nat.check(nat.lib().ngp_near_far_from_aabb(
        nat.ptr(rays_o), nat.ptr(rays_d), nat.ptr(aabb), N, float(min_near), nat.ptr(nears),
        nat.ptr(fars), nat.stream_of(rays_o)), "near_far_from_aabb")


def sph_from_ray(rays_o, rays_d, radius, N, coords):
    for t, n in ((rays_o, "rays_o"), (rays_d, "rays_d"), (coords, "coords")):
        _f(t, n)
    nat.check(nat.lib().ngp_sph_from_ray(nat.ptr(rays_o), nat.ptr(rays_d), float(radius), N,
                                         nat.ptr(coords), nat.stream_of(rays_o)), "sph_from_ray")


def morton3D(coords, N, indices):
    _i(coords, "coords")
    _i(indices, "indices")
    nat.check(nat.lib().ngp_morton3D(nat.ptr(coords), N, nat.ptr(indices), nat.stream_of(coords)),
              "morton3D")


def morton3D_invert(indices, N, coords):
    _i(indices, "indices")
    _i(coords, "coords")
    nat.check(nat.lib().ngp_morton3D_invert(nat.ptr(indices), N, nat.ptr(coords),
                                            nat.stream_of(indices)), "morton3D_invert")


def packbits(grid, N, density_thresh, bitfield):
    _f(grid, "grid")
    nat.check_tensor(bitfield, "bitfield", _U8, "uint8")
    nat.check(nat.lib().ngp_packbits(nat.ptr(grid), N, float(density_thresh), nat.ptr(bitfield),
                                     nat.stream_of(grid)), "packbits")


def march_rays_train(rays_o, rays_d, grid, bound, dt_gamma, max_steps, N, C, H, M, nears, fars,
                     xyzs, dirs, deltas, rays, counter, noises):
    for t, n in ((rays_o, "rays_o"), (rays_d, "rays_d"), (nears, "nears"), (fars, "fars"),
                 (xyzs, "xyzs"), (dirs, "dirs"), (deltas, "deltas"), (noises, "noises")):
        _f(t, n)
    nat.check_tensor(grid, "grid", _U8, "uint8")
    _i(rays, "rays")
    _i(counter, "counter")
    # per-sample t scratch of the single marching pass (caching allocator:
    # reused across steps and hipGraph-capture safe)
    ws_bytes = nat.lib().ngp_march_rays_train_workspace_bytes(N, max_steps, C, H)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=rays_o.device)
    nat.check(nat.lib().ngp_march_rays_train(
        nat.ptr(rays_o), nat.ptr(rays_d), nat.ptr(grid), float(bound), float(dt_gamma), max_steps,
        N, C, H, M, nat.ptr(nears), nat.ptr(fars), nat.ptr(xyzs), nat.ptr(dirs), nat.ptr(deltas),
        nat.ptr(rays), nat.ptr(counter), nat.ptr(noises), nat.ptr(ws), ws.numel(),
        nat.stream_of(rays_o)), "march_rays_train")


def composite_rays_train_forward(sigmas, rgbs, deltas, rays, M, N, T_thresh, weights_sum, depth, image):
    for t, n in ((sigmas, "sigmas"), (rgbs, "rgbs"), (deltas, "deltas"), (weights_sum, "weights_sum"),
                 (depth, "depth"), (image, "image")):
        _f(t, n)
    _i(rays, "rays")
    nat.check(nat.lib().ngp_composite_rays_train_forward(
        nat.ptr(sigmas), nat.ptr(rgbs), nat.ptr(deltas), nat.ptr(rays), M, N, float(T_thresh),
        nat.ptr(weights_sum), nat.ptr(depth), nat.ptr(image), nat.stream_of(sigmas)),
        "composite_rays_train_forward")


def composite_rays_train_backward(grad_weights_sum, grad_depth, grad_image, sigmas, rgbs, deltas,
                                  rays, weights_sum, depth, image, M, N, T_thresh, grad_sigmas,
                                  grad_rgbs):
    for t, n in ((grad_weights_sum, "grad_weights_sum"), (grad_depth, "grad_depth"),
                 (grad_image, "grad_image"), (sigmas, "sigmas"), (rgbs, "rgbs"),
                 (deltas, "deltas"), (weights_sum, "weights_sum"), (depth, "depth"),
                 (image, "image"), (grad_sigmas, "grad_sigmas"), (grad_rgbs, "grad_rgbs")):
        _f(t, n)
    _i(rays, "rays")
    nat.check(nat.lib().ngp_composite_rays_train_backward(
        nat.ptr(grad_weights_sum), nat.ptr(grad_depth), nat.ptr(grad_image), nat.ptr(sigmas),
        nat.ptr(rgbs), nat.ptr(deltas), nat.ptr(rays), nat.ptr(weights_sum), nat.ptr(depth),
        nat.ptr(image), M, N, float(T_thresh), nat.ptr(grad_sigmas), nat.ptr(grad_rgbs),
        nat.stream_of(sigmas)), "composite_rays_train_backward")


def march_rays(n_alive, n_step, rays_alive, rays_t, rays_o, rays_d, bound, dt_gamma, max_steps, C,
               H, grid, near, far, xyzs, dirs, deltas, noises):
    for t, n in ((rays_t, "rays_t"), (rays_o, "rays_o"), (rays_d, "rays_d"), (near, "nears"),
                 (far, "fars"), (xyzs, "xyzs"), (dirs, "dirs"), (deltas, "deltas"), (noises, "noises")):
        _f(t, n)
    _i(rays_alive, "rays_alive")
    nat.check_tensor(grid, "grid", _U8, "uint8")
    nat.check(nat.lib().ngp_march_rays(
        n_alive, n_step, nat.ptr(rays_alive), nat.ptr(rays_t), nat.ptr(rays_o), nat.ptr(rays_d),
        float(bound), float(dt_gamma), max_steps, C, H, nat.ptr(grid), nat.ptr(near), nat.ptr(far),
        nat.ptr(xyzs), nat.ptr(dirs), nat.ptr(deltas), nat.ptr(noises), nat.stream_of(rays_o)),
        "march_rays")


def composite_rays(n_alive, n_step, T_thresh, rays_alive, rays_t, sigmas, rgbs, deltas, weights,
                   depth, image):
    for t, n in ((rays_t, "rays_t"), (sigmas, "sigmas"), (rgbs, "rgbs"), (deltas, "deltas"),
                 (weights, "weights_sum"), (depth, "depth"), (image, "image")):
        _f(t, n)
    _i(rays_alive, "rays_alive")
    nat.check(nat.lib().ngp_composite_rays(
        n_alive, n_step, float(T_thresh), nat.ptr(rays_alive), nat.ptr(rays_t), nat.ptr(sigmas),
        nat.ptr(rgbs), nat.ptr(deltas), nat.ptr(weights), nat.ptr(depth), nat.ptr(image),
        nat.stream_of(rays_t)), "composite_rays")


_backend = types.SimpleNamespace(
    near_far_from_aabb=near_far_from_aabb, sph_from_ray=sph_from_ray, morton3D=morton3D,
    morton3D_invert=morton3D_invert, packbits=packbits, march_rays_train=march_rays_train,
    composite_rays_train_forward=composite_rays_train_forward,
    composite_rays_train_backward=composite_rays_train_backward, march_rays=march_rays,
    composite_rays=composite_rays,
)

__all__ = ["_backend"]

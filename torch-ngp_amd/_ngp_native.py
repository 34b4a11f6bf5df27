"""Loader for libngp_hip.so, the gfx950 C-ABI library behind every op package.

The reference packages bind their CUDA sources through pybind11 (AOT
`_gridencoder`/`_raymarching`/... or JIT `backend.py`, e.g.
gridencoder/backend.py:31-38). Here a single prebuilt shared library exports
the C functions declared in include/ngp_hip.h and each package's backend.py
binds them with ctypes. There is deliberately NO fallback: if the library or
a GPU is missing, every op raises.
"""
import ctypes
import os

import torch  # noqa: F401  (must load libamdhip64 before the library below)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NGP_HIP_LIB", os.path.join(_HERE, "libngp_hip.so"))

c_u32 = ctypes.c_uint32
c_i32 = ctypes.c_int32
c_f32 = ctypes.c_float
c_vp = ctypes.c_void_p
c_sz = ctypes.c_size_t

# name -> argtypes (restype int unless listed in _RESTYPES). Mirrors ngp_hip.h.
SIGNATURES = {
    "ngp_abi_version": [],
    "ngp_last_error": [],
    "ngp_grid_encode_forward": [c_vp, c_vp, c_vp, c_vp, c_u32, c_u32, c_u32, c_u32, c_f32, c_u32,
                                c_vp, c_u32, c_i32, c_u32, c_i32, c_i32, c_vp],
    "ngp_grid_encode_backward": [c_vp, c_vp, c_vp, c_vp, c_vp, c_u32, c_u32, c_u32, c_u32, c_f32,
                                 c_u32, c_vp, c_vp, c_u32, c_i32, c_u32, c_i32, c_i32, c_vp],
    "ngp_grad_total_variation": [c_vp, c_vp, c_vp, c_vp, c_f32, c_u32, c_u32, c_u32, c_u32, c_f32,
                                 c_u32, c_u32, c_i32, c_i32, c_vp],
    "ngp_near_far_from_aabb": [c_vp, c_vp, c_vp, c_u32, c_f32, c_vp, c_vp, c_vp],
    "ngp_sph_from_ray": [c_vp, c_vp, c_f32, c_u32, c_vp, c_vp],
    "ngp_morton3D": [c_vp, c_u32, c_vp, c_vp],
    "ngp_morton3D_invert": [c_vp, c_u32, c_vp, c_vp],
    "ngp_packbits": [c_vp, c_u32, c_f32, c_vp, c_vp],
    "ngp_march_rays_train_workspace_bytes": [c_u32, c_u32, c_u32, c_u32],
    "ngp_march_rays_train_error_offset": [c_u32, c_u32, c_u32, c_u32],
    "ngp_march_occupancy_build": [c_vp, c_u32, c_u32, c_u32, c_u32, c_vp, c_sz, c_vp],
    "ngp_march_rays_train_prebuilt": [c_vp, c_vp, c_vp, c_f32, c_f32, c_u32, c_u32, c_u32, c_u32, c_u32,
                                      c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp],
    "ngp_march_rays_train_prebuilt_tail": [c_vp, c_vp, c_vp, c_f32, c_f32, c_u32, c_u32, c_u32, c_u32, c_u32,
                                           c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz,
                                           c_vp, c_f32, c_f32, c_i32, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp,
                                           c_vp, c_vp, c_vp],
    "ngp_march_rays_train_prebuilt_adam": [c_vp, c_vp, c_vp, c_f32, c_f32, c_u32, c_u32, c_u32, c_u32, c_u32,
                                           c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz,
                                           c_vp, c_f32, c_f32, c_i32, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp,
                                           c_vp, c_vp, c_vp, c_vp],
    "ngp_grid_encode_backward_fused_reduce_batch": [c_vp, c_vp, c_f32, c_vp, c_vp, c_u32, c_vp, c_u32, c_u32,
                                                    c_u32, c_f32, c_u32, c_u32, c_i32, c_u32, c_vp, c_vp, c_sz,
                                                    c_i32, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                                    c_vp, c_vp],
    "ngp_grid_encode_backward_fused_reduce_batch_live": [c_vp, c_vp, c_f32, c_vp, c_vp, c_u32, c_vp, c_vp,
                                                         c_u32, c_u32, c_u32, c_f32, c_u32, c_u32, c_i32, c_u32,
                                                         c_vp, c_vp, c_sz, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp,
                                                         c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "ngp_march_rays_train": [c_vp, c_vp, c_vp, c_f32, c_f32, c_u32, c_u32, c_u32, c_u32, c_u32,
                             c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp],
    "ngp_composite_rays_train_forward": [c_vp, c_vp, c_vp, c_vp, c_u32, c_u32, c_f32, c_vp, c_vp,
                                         c_vp, c_vp],
    "ngp_composite_rays_train_backward": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                          c_vp, c_u32, c_u32, c_f32, c_vp, c_vp, c_vp],
    "ngp_march_rays": [c_u32, c_u32, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32, c_u32, c_u32, c_u32,
                       c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "ngp_grid_encode_forward_fused_tail": [c_vp, c_f32, c_vp, c_i32, c_vp, c_vp, c_u32, c_vp, c_u32, c_u32, c_u32,
                                           c_f32, c_u32, c_u32, c_i32, c_u32, c_vp, c_f32, c_f32, c_i32, c_i32, c_vp,
                                           c_u32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "ngp_render_state_bytes": [],
    "ngp_render_count": [c_vp, c_u32],
    "ngp_render_init": [c_u32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "ngp_render_march": [c_u32, c_u32, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32, c_u32, c_u32, c_u32, c_vp,
                         c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "ngp_render_composite": [c_u32, c_u32, c_u32, c_vp, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                             c_vp, c_vp],
    "ngp_composite_rays": [c_u32, c_u32, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                           c_vp],
    "ngp_sh_encode_forward": [c_vp, c_vp, c_u32, c_u32, c_u32, c_vp, c_i32, c_vp],
    "ngp_sh_encode_backward": [c_vp, c_vp, c_u32, c_u32, c_u32, c_vp, c_vp, c_i32, c_vp],
    "ngp_freq_encode_forward": [c_vp, c_u32, c_u32, c_u32, c_u32, c_vp, c_vp],
    "ngp_freq_encode_backward": [c_vp, c_vp, c_u32, c_u32, c_u32, c_u32, c_vp, c_vp],
    "ngp_ffmlp_forward": [c_vp, c_vp, c_u32, c_u32, c_u32, c_u32, c_u32, c_u32, c_u32, c_vp, c_vp,
                          c_vp],
    "ngp_ffmlp_inference": [c_vp, c_vp, c_u32, c_u32, c_u32, c_u32, c_u32, c_u32, c_u32, c_vp,
                            c_vp, c_vp],
    "ngp_ffmlp_backward_workspace_bytes": [c_u32, c_u32, c_u32, c_u32, c_u32],
    "ngp_ffmlp_backward": [c_vp, c_vp, c_vp, c_vp, c_u32, c_u32, c_u32, c_u32, c_u32, c_u32, c_u32,
                           c_i32, c_vp, c_vp, c_vp, c_i32, c_vp, c_sz, c_vp],
    "ngp_ffmlp_allocate_splitk": [c_sz],
    "ngp_ffmlp_free_splitk": [],
    "ngp_adam_step": [c_vp, c_vp, c_i32, c_vp, c_vp, c_sz, c_f32, c_f32, c_f32, c_f32, c_f32,
                      c_i32, c_f32, c_vp],
    "ngp_grid_encode_forward_fused": [c_vp, c_f32, c_vp, c_i32, c_vp, c_vp, c_u32, c_vp, c_u32, c_u32,
                                      c_u32, c_f32, c_u32, c_u32, c_i32, c_u32, c_i32, c_vp],
    "ngp_grid_encode_backward_fused_workspace_bytes": [c_u32, c_u32, c_u32, c_u32, c_f32, c_u32, c_i32,
                                                       c_vp],
    "ngp_grid_encode_backward_fused": [c_vp, c_vp, c_f32, c_vp, c_vp, c_u32, c_vp, c_u32, c_u32,
                                       c_u32, c_f32, c_u32, c_u32, c_i32, c_u32, c_vp, c_vp, c_sz, c_i32,
                                       c_vp, c_vp],
    "ngp_ffmlp_image_bytes": [c_u32, c_u32, c_u32],
    "ngp_grad_guard": [c_vp, ctypes.c_uint64, ctypes.c_uint64, c_i32, c_vp, c_vp],
    "ngp_fused_inf_flag": [c_vp, c_i32],
    "ngp_grid_encode_backward_fused_counter_bytes": [c_u32, c_u32, c_u32, c_u32, c_f32, c_u32, c_i32, c_vp],
    "ngp_fused_optimizer_update": [c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32, c_f32, c_f32,
                                   c_i32, c_i32, c_f32, c_i32, c_vp, c_vp],
    "ngp_fused_step_head": [c_vp, c_u32, c_vp, c_u32, c_u32, c_u32, c_vp, c_i32, c_vp, c_f32, c_u32, c_vp,
                            c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32, c_i32, c_i32,
                            c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_u32, c_vp],
    "ngp_fused_optimizer_update_head": [c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32, c_f32, c_f32,
                                        c_i32, c_i32, c_f32, c_i32, c_vp,
                                        c_vp, c_u32, c_vp, c_u32, c_u32, c_u32, c_vp, c_i32, c_vp, c_f32, c_u32,
                                        c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_u32, c_vp],
    "ngp_ffmlp_pack": [c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "ngp_ffmlp_forward_rows": [c_vp, c_vp, c_vp, c_u32, c_vp, c_u32, c_u32, c_u32, c_u32, c_u32, c_u32,
                               c_vp, c_vp],
    "ngp_nerf_sigma_forward": [c_vp, c_vp, c_vp, c_u32, c_vp, c_u32, c_u32, c_u32, c_vp, c_vp, c_vp, c_vp,
                               c_f32, c_u32, c_vp],
    "ngp_nerf_forward": [c_vp, c_vp, c_vp, c_u32, c_vp, c_u32, c_u32, c_u32, c_u32, c_vp, c_vp, c_vp, c_vp,
                         c_f32, c_vp, c_vp],
    "ngp_ffmlp_backward_rows": [c_vp, c_vp, c_vp, c_vp, c_u32, c_vp, c_u32, c_u32, c_u32, c_u32, c_u32,
                                c_vp, c_vp, c_i32, c_u32, c_vp, c_sz, c_vp],
    "ngp_nerf_backward": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_u32, c_vp, c_u32, c_u32, c_u32, c_u32,
                          c_vp, c_sz, c_vp, c_sz, c_vp, c_vp],
    "ngp_nerf_backward_live": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_u32, c_vp, c_vp, c_u32, c_u32, c_u32,
                               c_u32, c_vp, c_sz, c_vp, c_sz, c_vp, c_vp],
    "ngp_ffmlp_reduce": [c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp],
    "ngp_fused_state_bytes": [],
    "ngp_fused_state_init": [c_vp, c_f32, c_vp],
    "ngp_lego_rays": [c_vp, c_u32, c_vp, c_u32, c_u32, c_u32, c_vp, c_i32, c_vp, c_f32, c_u32,
                      c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "ngp_nerf_glue_forward": [c_vp, c_vp, c_f32, c_vp, c_vp, c_u32, c_vp, c_vp],
    "ngp_nerf_glue_backward": [c_vp, c_vp, c_u32, c_vp, c_vp],
    "ngp_nerf_composite_loss": [c_vp, c_vp, c_vp, c_vp, c_vp, c_u32, c_u32, c_f32, c_f32, c_vp,
                                c_u32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "ngp_nerf_composite_loss_live": [c_vp, c_vp, c_vp, c_vp, c_vp, c_u32, c_u32, c_f32, c_f32, c_vp,
                                     c_u32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                     c_vp],
    "ngp_fused_optimizer_step": [c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32, c_f32, c_f32,
                                 c_i32, c_i32, c_f32, c_f32, c_f32, c_i32, c_i32, c_u32, c_vp, c_vp,
                                 c_vp, c_vp, c_vp],
    "ngp_density_grid_points": [c_vp, c_vp, c_u32, c_u32, c_u32, c_u32, c_f32, c_vp, c_vp, c_vp],
    "ngp_nerf_density_forward": [c_vp, c_vp, c_vp, c_u32, c_u32, c_u32, c_u32, c_f32, c_vp, c_vp, c_vp],
    "ngp_density_grid_ema_pack": [c_vp, c_vp, c_u32, c_u32, c_f32, ctypes.c_double, c_vp, c_vp, c_vp],
    "ngp_density_grid_draw_workspace_bytes": [c_u32, c_u32],
    "ngp_density_grid_sort_workspace_bytes": [c_u32, c_u32],
    "ngp_density_grid_points_sorted": [c_vp, c_vp, c_u32, c_u32, c_u32, c_u32, c_f32, c_u32, c_u32, c_vp, c_sz,
                                       c_vp, c_vp, c_vp],
    "ngp_density_grid_draw": [c_vp, c_u32, c_u32, c_u32, c_u32, c_u32, c_vp, c_vp, c_vp, c_sz, c_vp],
    "ngp_density_mean_count": [c_vp, c_vp, c_vp, c_u32, c_u32, c_vp, c_vp],
    "ngp_nerf_density_forward_rows": [c_vp, c_vp, c_u32, c_u32, c_u32, c_f32, c_vp, c_vp],
    "ngp_density_grid_run_max": [c_vp, c_vp, c_u32, c_u32, c_u32, c_u32, c_vp, c_vp],
    "ngp_density_grid_ostat_workspace_bytes": [c_u32, c_u32],
    "ngp_density_grid_draw_sorted": [c_vp, c_u32, c_u32, c_u32, c_u32, c_f32, c_u32, c_u32, c_vp, c_sz, c_vp, c_sz,
                                     c_vp, c_vp, c_vp],
    "ngp_grid_encode_backward_fused_timing_offset": [c_u32, c_u32, c_u32, c_u32, c_f32, c_u32, c_i32, c_vp],
    "ngp_grad_exchange_bins": [ctypes.c_uint64],
    "ngp_grad_exchange_words": [ctypes.c_uint64, c_u32],
    "ngp_grad_exchange_list": [c_vp, ctypes.c_uint64, c_vp, c_vp, c_u32, c_vp],
    "ngp_grad_exchange_reduce": [c_vp, c_i32, c_u32, c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp],
    "ngp_grid_encode_backward_fused_reduce": [c_vp, c_vp, c_f32, c_vp, c_vp, c_u32, c_vp, c_u32, c_u32, c_u32,
                                              c_f32, c_u32, c_u32, c_i32, c_u32, c_vp, c_vp, c_sz, c_i32, c_vp,
                                              c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
}
_RESTYPES = {
    "ngp_last_error": ctypes.c_char_p,
    "ngp_fused_inf_flag": c_vp,
    "ngp_grid_encode_backward_fused_timing_offset": c_sz,
    "ngp_grid_encode_backward_fused_counter_bytes": c_sz,
    "ngp_ffmlp_backward_workspace_bytes": c_sz,
    "ngp_march_rays_train_workspace_bytes": c_sz,
    "ngp_march_rays_train_error_offset": c_sz,
    "ngp_fused_state_bytes": c_sz,
    "ngp_render_state_bytes": c_sz,
    "ngp_render_count": c_vp,
    "ngp_grid_encode_backward_fused_workspace_bytes": c_sz,
    "ngp_ffmlp_image_bytes": c_sz,
    "ngp_density_grid_draw_workspace_bytes": c_sz,
    "ngp_density_grid_sort_workspace_bytes": c_sz,
    "ngp_density_grid_ostat_workspace_bytes": c_sz,
    "ngp_grad_exchange_bins": c_u32,
    "ngp_grad_exchange_words": ctypes.c_uint64,
}

DTYPE_CODE = {torch.float32: 0, torch.float16: 1, torch.float64: 2}
DENSITY_STATS_LEN = 1025  # include/ngp_hip.h NGP_DENSITY_STATS_LEN (doubles of ngp_density_grid_ema_pack's stats)


class AdamJob(ctypes.Structure):
    """ngp_adam_job (include/ngp_hip.h): the optimizer update a march launch
    carries (ngp_march_rays_train_prebuilt_adam)."""
    _fields_ = [("n_tensors", c_i32), ("params", c_vp * 8), ("grads", c_vp * 8), ("exp_avg", c_vp * 8),
                ("exp_avg_sq", c_vp * 8), ("half_params", c_vp * 8), ("sizes", ctypes.c_uint64 * 8),
                ("lr", c_f32), ("beta1", c_f32), ("beta2", c_f32), ("eps", c_f32), ("iters", c_i32),
                ("zero_grads", c_i32), ("grad_mult", c_f32), ("clear", c_vp), ("clear_bytes", c_u32),
                ("flags", c_u32)]


ADAM_JOB_TAIL_LATER = 2  # NGP_ADAM_JOB_TAIL_LATER
ADAM_JOB_EMIT_LAUNCH = 4  # NGP_ADAM_JOB_EMIT_LAUNCH


class BatchJob(ctypes.Structure):
    """ngp_batch_job (include/ngp_hip.h): the fused step's next batch, drawn by
    ngp_grid_encode_backward_fused_reduce_batch."""
    _fields_ = [("poses", c_vp), ("n_poses", c_u32), ("intrinsics4", c_vp), ("H", c_u32), ("W", c_u32),
                ("N", c_u32), ("boxes", c_vp), ("nboxes", c_i32), ("aabb6", c_vp), ("min_near", c_f32),
                ("seed", c_u32), ("state", c_vp), ("rays_o", c_vp), ("rays_d", c_vp), ("rgba", c_vp), ("bg", c_vp),
                ("nears", c_vp), ("fars", c_vp), ("noises", c_vp), ("counter", c_vp), ("step_counter", c_vp)]

_lib = None


def lib():
    """Load (once) and return the ctypes handle; raises if the .so is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libngp_hip.so not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.argtypes = argtypes
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _lib = handle
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().ngp_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def ptr(t):
    """Raw device pointer of a tensor (or NULL for None)."""
    return None if t is None else t.data_ptr()


def stream_of(t):
    """hipStream_t handle of the current torch stream on the tensor's device."""
    return torch.cuda.current_stream(t.device).cuda_stream


def require_cuda(t, name):
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")


def require_contiguous(t, name):
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be a contiguous tensor")


def require_dtype(t, name, dtypes, what):
    if t.dtype not in dtypes:
        raise RuntimeError(f"{name} must be a {what} tensor")


FLOATING = (torch.float32, torch.float16, torch.float64)


def check_tensor(t, name, dtypes=FLOATING, what="floating", contiguous=True):
    require_cuda(t, name)
    if contiguous:
        require_contiguous(t, name)
    if dtypes is not None:
        require_dtype(t, name, dtypes, what)

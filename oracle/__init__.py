"""CPU oracle for the instant-ngp hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker / the timed CPU baseline. The
product code under torch-ngp_amd/ never imports it (tests/test_boundary.py
checks that), and has no CPU fallback.

Contents:
  * ctypes bindings to ngp_oracle.c (sequential C restatements of the
    reference CUDA kernels, bit-exact contract with the HIP kernels);
  * numpy restatements of shencoder (values, float32 op order of
    shencoder.cu:49-121), of the fused MLP (ffmlp.cu layer semantics), of
    trunc_exp (activation.py:5-18) and of the frequency encoder
    (freqencoder.cu:30-94);
  * `pipeline` (oracle/pipeline.py): an end-to-end CPU train step built from
    the above, used for bench.py's cpu_baseline.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "ngp_oracle.c")
BUILD_DIR = os.path.join(HERE, "build")
LIB = os.path.join(BUILD_DIR, "libngp_oracle.so")

_lib = None


def build(force=False):
    """Compile ngp_oracle.c with gcc (no FMA contraction)."""
    os.makedirs(BUILD_DIR, exist_ok=True)
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.check_call(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-fno-fast-math",
                               "-fPIC", "-shared", SRC, "-o", LIB, "-lm"])
    return LIB


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB)
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _u(x):
    return ctypes.c_uint32(int(x))


def _f(x):
    return ctypes.c_float(float(x))


_DT = {np.dtype(np.float32): 0, np.dtype(np.float16): 1, np.dtype(np.float64): 2}


def f2h(x):
    """float32 -> float16 with the C oracle's RNE conversion (as uint16 view)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty(x.shape, dtype=np.uint16)
    lib().oracle_f2h_array(_p(x), _p(out), ctypes.c_size_t(x.size))
    return out.view(np.float16)


# --------------------------------------------------------------------------- grid

def grid_offsets(D, L, C, H, per_level_scale, log2T, align_corners=False):
    """Level table offsets exactly as GridEncoder.__init__ (grid.py:776-789)."""
    offsets, off = [], 0
    for i in range(L):
        res = int(np.ceil(H * per_level_scale ** i))
        n = min(2 ** log2T, (res if align_corners else res + 1) ** D)
        n = int(np.ceil(n / 8) * 8)
        offsets.append(off)
        off += n
    offsets.append(off)
    return np.array(offsets, dtype=np.int32)


def grid_encode_forward(inputs, embeddings, offsets, per_level_scale, H, calc_dy_dx=False,
                        gridtype=0, align_corners=False, interp=0, out_layout=1):
    """Returns outputs ([B, L*C] if out_layout else [L, B, C]) and dy_dx or None."""
    inputs = np.ascontiguousarray(inputs, dtype=np.float32)
    emb = np.ascontiguousarray(embeddings)
    offsets = np.ascontiguousarray(offsets, dtype=np.int32)
    B, D = inputs.shape
    C = emb.shape[1]
    L = offsets.shape[0] - 1
    S = np.float32(np.log2(per_level_scale))
    out = np.empty((B, L * C) if out_layout else (L, B, C), dtype=emb.dtype)
    dy = np.empty((B, L * D * C), dtype=emb.dtype) if calc_dy_dx else None
    rc = lib().oracle_grid_encode_forward(_p(inputs), _p(emb), _p(offsets), _p(out), _u(B), _u(D),
                                          _u(C), _u(L), _f(S), _u(H), _p(dy), _u(gridtype),
                                          ctypes.c_int(int(align_corners)), _u(interp),
                                          ctypes.c_int(_DT[emb.dtype]), ctypes.c_int(out_layout))
    assert rc == 0
    return out, dy


def grid_encode_backward(grad, inputs, offsets, C, per_level_scale, H, gridtype=0,
                         align_corners=False, interp=0, grad_layout=1):
    """float64 [sum_T, C] scatter of the per-corner contributions."""
    grad = np.ascontiguousarray(grad)
    inputs = np.ascontiguousarray(inputs, dtype=np.float32)
    offsets = np.ascontiguousarray(offsets, dtype=np.int32)
    B, D = inputs.shape
    L = offsets.shape[0] - 1
    S = np.float32(np.log2(per_level_scale))
    out = np.zeros((int(offsets[-1]), C), dtype=np.float64)
    rc = lib().oracle_grid_encode_backward(_p(grad), _p(inputs), _p(offsets), _p(out), _u(B), _u(D),
                                           _u(C), _u(L), _f(S), _u(H), _u(gridtype),
                                           ctypes.c_int(int(align_corners)), _u(interp),
                                           ctypes.c_int(_DT[grad.dtype]), ctypes.c_int(grad_layout))
    assert rc == 0
    return out


def grad_total_variation(inputs, embeddings, offsets, weight, per_level_scale, H, gridtype=0,
                         align_corners=False):
    """float64 image of the TV gradient kernel_grad_tv adds (gridencoder.cu:503-607);
    inputs and embeddings float32 or float64 (the reference's type)."""
    emb = np.ascontiguousarray(embeddings)
    x = np.ascontiguousarray(inputs, dtype=emb.dtype)
    offsets = np.ascontiguousarray(offsets, dtype=np.int32)
    B, D = x.shape
    C = emb.shape[1]
    L = offsets.shape[0] - 1
    S = np.float32(np.log2(per_level_scale))
    out = np.zeros((int(offsets[-1]), C), dtype=np.float64)
    rc = lib().oracle_grad_tv(_p(x), _p(emb), _p(out), _p(offsets), _f(weight), _u(B), _u(D), _u(C), _u(L),
                              _f(S), _u(H), _u(gridtype), ctypes.c_int(int(align_corners)),
                              ctypes.c_int(_DT[emb.dtype]))
    assert rc == 0
    return out


def grid_input_backward(grad, dy_dx, B, D, C, L, grad_layout=1):
    grad = np.ascontiguousarray(grad)
    dy_dx = np.ascontiguousarray(dy_dx, dtype=grad.dtype)
    out = np.empty((B, D), dtype=grad.dtype)
    lib().oracle_grid_input_backward(_p(grad), _p(dy_dx), _p(out), _u(B), _u(D), _u(C), _u(L),
                                     ctypes.c_int(_DT[grad.dtype]), ctypes.c_int(grad_layout))
    return out


# ---------------------------------------------------------------------- raymarch

def near_far_from_aabb(rays_o, rays_d, aabb, min_near=0.2):
    ro = np.ascontiguousarray(rays_o, dtype=np.float32).reshape(-1, 3)
    rd = np.ascontiguousarray(rays_d, dtype=np.float32).reshape(-1, 3)
    aabb = np.ascontiguousarray(aabb, dtype=np.float32)
    N = ro.shape[0]
    nears = np.empty(N, np.float32)
    fars = np.empty(N, np.float32)
    lib().oracle_near_far_from_aabb(_p(ro), _p(rd), _p(aabb), _u(N), _f(min_near), _p(nears), _p(fars))
    return nears, fars


def morton3D(coords):
    c = np.ascontiguousarray(coords, dtype=np.int32)
    out = np.empty(c.shape[0], np.int32)
    lib().oracle_morton3D(_p(c), _u(c.shape[0]), _p(out))
    return out


def morton3D_invert(indices):
    i = np.ascontiguousarray(indices, dtype=np.int32)
    out = np.empty((i.shape[0], 3), np.int32)
    lib().oracle_morton3D_invert(_p(i), _u(i.shape[0]), _p(out))
    return out


def packbits(grid, thresh):
    g = np.ascontiguousarray(grid, dtype=np.float32)
    N = g.size // 8
    out = np.empty(N, np.uint8)
    lib().oracle_packbits(_p(g), _u(N), _f(thresh), _p(out))
    return out


def march_rays_train(rays_o, rays_d, bound, bitfield, C, H, nears, fars, noises, M=None,
                     dt_gamma=0.0, max_steps=1024, counter=(0, 0)):
    """Returns xyzs, dirs, deltas (zero-filled [M, *]), rays [N, 3], counter [2]."""
    ro = np.ascontiguousarray(rays_o, dtype=np.float32).reshape(-1, 3)
    rd = np.ascontiguousarray(rays_d, dtype=np.float32).reshape(-1, 3)
    N = ro.shape[0]
    if M is None:
        M = N * max_steps
    xyzs = np.zeros((M, 3), np.float32)
    dirs = np.zeros((M, 3), np.float32)
    deltas = np.zeros((M, 2), np.float32)
    rays = np.empty((N, 3), np.int32)
    cnt = np.array(counter, dtype=np.int32)
    bf = np.ascontiguousarray(bitfield, dtype=np.uint8)
    nears = np.ascontiguousarray(nears, np.float32)
    fars = np.ascontiguousarray(fars, np.float32)
    noises = np.ascontiguousarray(noises, np.float32)
    lib().oracle_march_rays_train(_p(ro), _p(rd), _p(bf), _f(bound), _f(dt_gamma), _u(max_steps),
                                  _u(N), _u(C), _u(H), _u(M), _p(nears), _p(fars), _p(xyzs), _p(dirs),
                                  _p(deltas), _p(rays), _p(cnt), _p(noises))
    return xyzs, dirs, deltas, rays, cnt


def march_rays(n_alive, n_step, rays_alive, rays_t, rays_o, rays_d, bound, bitfield, C, H, nears,
               fars, noises, dt_gamma=0.0, max_steps=1024, align=-1):
    M = n_alive * n_step
    if align > 0:
        M += align - (M % align)
    xyzs = np.zeros((M, 3), np.float32)
    dirs = np.zeros((M, 3), np.float32)
    deltas = np.zeros((M, 2), np.float32)
    args = [np.ascontiguousarray(a, dt) for a, dt in
            ((rays_alive, np.int32), (rays_t, np.float32), (rays_o, np.float32), (rays_d, np.float32),
             (bitfield, np.uint8), (nears, np.float32), (fars, np.float32), (noises, np.float32))]
    ra, rt, ro, rd, bf, ne, fa, no = args
    lib().oracle_march_rays(_u(n_alive), _u(n_step), _p(ra), _p(rt), _p(ro), _p(rd), _f(bound),
                            _f(dt_gamma), _u(max_steps), _u(C), _u(H), _p(bf), _p(ne), _p(fa),
                            _p(xyzs), _p(dirs), _p(deltas), _p(no))
    return xyzs, dirs, deltas


def composite_rays_train_forward(sigmas, rgbs, deltas, rays, T_thresh=1e-4):
    s = np.ascontiguousarray(sigmas, np.float32)
    c = np.ascontiguousarray(rgbs, np.float32)
    d = np.ascontiguousarray(deltas, np.float32)
    r = np.ascontiguousarray(rays, np.int32)
    M, N = s.shape[0], r.shape[0]
    ws = np.empty(N, np.float32)
    dp = np.empty(N, np.float32)
    img = np.empty((N, 3), np.float32)
    lib().oracle_composite_rays_train_forward(_p(s), _p(c), _p(d), _p(r), _u(M), _u(N), _f(T_thresh),
                                              _p(ws), _p(dp), _p(img))
    return ws, dp, img


def composite_rays_train_backward(grad_ws, grad_depth, grad_image, sigmas, rgbs, deltas, rays, ws,
                                  depth, image, T_thresh=1e-4):
    arrs = [np.ascontiguousarray(a, np.float32) for a in
            (grad_ws, grad_depth, grad_image, sigmas, rgbs, deltas)]
    r = np.ascontiguousarray(rays, np.int32)
    outs = [np.ascontiguousarray(a, np.float32) for a in (ws, depth, image)]
    M, N = arrs[3].shape[0], r.shape[0]
    gs = np.zeros(M, np.float32)
    gc = np.zeros((M, 3), np.float32)
    lib().oracle_composite_rays_train_backward(*[_p(a) for a in arrs], _p(r), *[_p(a) for a in outs],
                                               _u(M), _u(N), _f(T_thresh), _p(gs), _p(gc))
    return gs, gc


def composite_rays(n_alive, n_step, rays_alive, rays_t, sigmas, rgbs, deltas, weights_sum, depth,
                   image, T_thresh=1e-2):
    """In place on the given numpy arrays (like the reference)."""
    s = np.ascontiguousarray(sigmas, np.float32)
    c = np.ascontiguousarray(rgbs, np.float32)
    d = np.ascontiguousarray(deltas, np.float32)
    lib().oracle_composite_rays(_u(n_alive), _u(n_step), _f(T_thresh), _p(rays_alive), _p(rays_t),
                                _p(s), _p(c), _p(d), _p(weights_sum), _p(depth), _p(image))


# ------------------------------------------------------------------------- SH

_f32 = np.float32


def sh_encode(inputs, degree):
    """Values of the first degree^2 real SH (shencoder.cu:49-121), float32 op order."""
    v = np.ascontiguousarray(inputs, dtype=np.float32)
    x, y, z = v[:, 0], v[:, 1], v[:, 2]
    return _sh_values(x, y, z, degree, _f32).astype(np.float32)


def sh_encode_jacobian(inputs, degree, eps=1e-4):
    """d SH / d(x, y, z) as [B, 3, degree^2] (float64 central differences of the
    same polynomials; the reference writes the analytic derivatives,
    shencoder.cu:122-355)."""
    v = np.asarray(inputs, dtype=np.float64)
    out = np.empty((v.shape[0], 3, degree * degree))
    for d in range(3):
        hi = v.copy(); hi[:, d] += eps
        lo = v.copy(); lo[:, d] -= eps
        fh = _sh_values(hi[:, 0], hi[:, 1], hi[:, 2], degree, np.float64)
        fl = _sh_values(lo[:, 0], lo[:, 1], lo[:, 2], degree, np.float64)
        out[:, d, :] = (fh - fl) / (2 * eps)
    return out


def _sh_values(x, y, z, degree, T):
    c = lambda a: T(a)  # noqa: E731
    xy, xz, yz, x2, y2, z2 = x * y, x * z, y * z, x * x, y * y, z * z
    x4, y4, z4 = x2 * x2, y2 * y2, z2 * z2
    x6, y6, z6 = x4 * x2, y4 * y2, z4 * z2
    B = x.shape[0]
    o = np.zeros((B, degree * degree), dtype=T)
    o[:, 0] = c(0.28209479177387814)
    if degree <= 1: return o
    o[:, 1] = c(-0.48860251190291987) * y
    o[:, 2] = c(0.48860251190291987) * z
    o[:, 3] = c(-0.48860251190291987) * x
    if degree <= 2: return o
    o[:, 4] = c(1.0925484305920792) * xy
    o[:, 5] = c(-1.0925484305920792) * yz
    o[:, 6] = c(0.94617469575755997) * z2 - c(0.31539156525251999)
    o[:, 7] = c(-1.0925484305920792) * xz
    o[:, 8] = c(0.54627421529603959) * x2 - c(0.54627421529603959) * y2
    if degree <= 3: return o
    o[:, 9] = c(0.59004358992664352) * y * (c(-3.0) * x2 + y2)
    o[:, 10] = c(2.8906114426405538) * xy * z
    o[:, 11] = c(0.45704579946446572) * y * (c(1.0) - c(5.0) * z2)
    o[:, 12] = c(0.3731763325901154) * z * (c(5.0) * z2 - c(3.0))
    o[:, 13] = c(0.45704579946446572) * x * (c(1.0) - c(5.0) * z2)
    o[:, 14] = c(1.4453057213202769) * z * (x2 - y2)
    o[:, 15] = c(0.59004358992664352) * x * (-x2 + c(3.0) * y2)
    if degree <= 4: return o
    o[:, 16] = c(2.5033429417967046) * xy * (x2 - y2)
    o[:, 17] = c(1.7701307697799304) * yz * (c(-3.0) * x2 + y2)
    o[:, 18] = c(0.94617469575756008) * xy * (c(7.0) * z2 - c(1.0))
    o[:, 19] = c(0.66904654355728921) * yz * (c(3.0) - c(7.0) * z2)
    o[:, 20] = c(-3.1735664074561294) * z2 + c(3.7024941420321507) * z4 + c(0.31735664074561293)
    o[:, 21] = c(0.66904654355728921) * xz * (c(3.0) - c(7.0) * z2)
    o[:, 22] = c(0.47308734787878004) * (x2 - y2) * (c(7.0) * z2 - c(1.0))
    o[:, 23] = c(1.7701307697799304) * xz * (-x2 + c(3.0) * y2)
    o[:, 24] = c(-3.7550144126950569) * x2 * y2 + c(0.62583573544917614) * x4 + c(0.62583573544917614) * y4
    if degree <= 5: return o
    o[:, 25] = c(0.65638205684017015) * y * (c(10.0) * x2 * y2 - c(5.0) * x4 - y4)
    o[:, 26] = c(8.3026492595241645) * xy * z * (x2 - y2)
    o[:, 27] = c(-0.48923829943525038) * y * (c(3.0) * x2 - y2) * (c(9.0) * z2 - c(1.0))
    o[:, 28] = c(4.7935367849733241) * xy * z * (c(3.0) * z2 - c(1.0))
    o[:, 29] = c(0.45294665119569694) * y * (c(14.0) * z2 - c(21.0) * z4 - c(1.0))
    o[:, 30] = c(0.1169503224534236) * z * (c(-70.0) * z2 + c(63.0) * z4 + c(15.0))
    o[:, 31] = c(0.45294665119569694) * x * (c(14.0) * z2 - c(21.0) * z4 - c(1.0))
    o[:, 32] = c(2.3967683924866621) * z * (x2 - y2) * (c(3.0) * z2 - c(1.0))
    o[:, 33] = c(-0.48923829943525038) * x * (x2 - c(3.0) * y2) * (c(9.0) * z2 - c(1.0))
    o[:, 34] = c(2.0756623148810411) * z * (c(-6.0) * x2 * y2 + x4 + y4)
    o[:, 35] = c(0.65638205684017015) * x * (c(10.0) * x2 * y2 - x4 - c(5.0) * y4)
    if degree <= 6: return o
    o[:, 36] = c(1.3663682103838286) * xy * (c(-10.0) * x2 * y2 + c(3.0) * x4 + c(3.0) * y4)
    o[:, 37] = c(2.3666191622317521) * yz * (c(10.0) * x2 * y2 - c(5.0) * x4 - y4)
    o[:, 38] = c(2.0182596029148963) * xy * (x2 - y2) * (c(11.0) * z2 - c(1.0))
    o[:, 39] = c(-0.92120525951492349) * yz * (c(3.0) * x2 - y2) * (c(11.0) * z2 - c(3.0))
    o[:, 40] = c(0.92120525951492349) * xy * (c(-18.0) * z2 + c(33.0) * z4 + c(1.0))
    o[:, 41] = c(0.58262136251873131) * yz * (c(30.0) * z2 - c(33.0) * z4 - c(5.0))
    o[:, 42] = c(6.6747662381009842) * z2 - c(20.024298714302954) * z4 + c(14.684485723822165) * z6 - c(0.31784601133814211)
    o[:, 43] = c(0.58262136251873131) * xz * (c(30.0) * z2 - c(33.0) * z4 - c(5.0))
    o[:, 44] = c(0.46060262975746175) * (x2 - y2) * (c(11.0) * z2 * (c(3.0) * z2 - c(1.0)) - c(7.0) * z2 + c(1.0))
    o[:, 45] = c(-0.92120525951492349) * xz * (x2 - c(3.0) * y2) * (c(11.0) * z2 - c(3.0))
    o[:, 46] = c(0.50456490072872406) * (c(11.0) * z2 - c(1.0)) * (c(-6.0) * x2 * y2 + x4 + y4)
    o[:, 47] = c(2.3666191622317521) * xz * (c(10.0) * x2 * y2 - x4 - c(5.0) * y4)
    o[:, 48] = c(10.247761577878714) * x2 * y4 - c(10.247761577878714) * x4 * y2 + c(0.6831841051919143) * x6 - c(0.6831841051919143) * y6
    if degree <= 7: return o
    o[:, 49] = c(0.70716273252459627) * y * (c(-21.0) * x2 * y4 + c(35.0) * x4 * y2 - c(7.0) * x6 + y6)
    o[:, 50] = c(5.2919213236038001) * xy * z * (c(-10.0) * x2 * y2 + c(3.0) * x4 + c(3.0) * y4)
    o[:, 51] = c(-0.51891557872026028) * y * (c(13.0) * z2 - c(1.0)) * (c(-10.0) * x2 * y2 + c(5.0) * x4 + y4)
    o[:, 52] = c(4.1513246297620823) * xy * z * (x2 - y2) * (c(13.0) * z2 - c(3.0))
    o[:, 53] = c(-0.15645893386229404) * y * (c(3.0) * x2 - y2) * (c(13.0) * z2 * (c(11.0) * z2 - c(3.0)) - c(27.0) * z2 + c(3.0))
    o[:, 54] = c(0.44253269244498261) * xy * z * (c(-110.0) * z2 + c(143.0) * z4 + c(15.0))
    o[:, 55] = c(0.090331607582517306) * y * (c(-135.0) * z2 + c(495.0) * z4 - c(429.0) * z6 + c(5.0))
    o[:, 56] = c(0.068284276912004949) * z * (c(315.0) * z2 - c(693.0) * z4 + c(429.0) * z6 - c(35.0))
    o[:, 57] = c(0.090331607582517306) * x * (c(-135.0) * z2 + c(495.0) * z4 - c(429.0) * z6 + c(5.0))
    o[:, 58] = c(0.07375544874083044) * z * (x2 - y2) * (c(143.0) * z2 * (c(3.0) * z2 - c(1.0)) - c(187.0) * z2 + c(45.0))
    o[:, 59] = c(-0.15645893386229404) * x * (x2 - c(3.0) * y2) * (c(13.0) * z2 * (c(11.0) * z2 - c(3.0)) - c(27.0) * z2 + c(3.0))
    o[:, 60] = c(1.0378311574405206) * z * (c(13.0) * z2 - c(3.0)) * (c(-6.0) * x2 * y2 + x4 + y4)
    o[:, 61] = c(-0.51891557872026028) * x * (c(13.0) * z2 - c(1.0)) * (c(-10.0) * x2 * y2 + x4 + c(5.0) * y4)
    o[:, 62] = c(2.6459606618019) * z * (c(15.0) * x2 * y4 - c(15.0) * x4 * y2 + x6 - y6)
    o[:, 63] = c(0.70716273252459627) * x * (c(-35.0) * x2 * y4 + c(21.0) * x4 * y2 - x6 + c(7.0) * y6)
    return o


# ------------------------------------------------------------------------ MLP

def _act(a, x):
    if a == 0: return np.maximum(x, 0)
    if a == 1: return np.exp(x)
    if a == 2: return np.sin(x)
    if a == 3: return 1 / (1 + np.exp(-x))
    if a == 4:
        y = x * 10.0
        return 0.5 * (y + np.sqrt(y * y + 4)) / 10.0
    if a == 5: return np.log(np.exp(x * 10.0) + 1.0) / 10.0
    return x


def _act_bwd(a, g, y):
    if a == 0: return g * (y > 0)
    if a == 1: return g * y
    if a == 3: return g * y * (1 - y)
    if a == 4:
        t = y * 10.0
        return g * (t * t / (t * t + 1))
    if a == 5: return g * (1 - np.exp(-y * 10.0))
    return g


def mlp_layers(weights, input_dim, output_dim, hidden_dim, num_layers):
    """Split the flat FFMLP weight vector into per-layer [out, in] matrices
    (ffmlp.py:115; num_layers hidden activations -> num_layers + 1 matmuls)."""
    w = np.asarray(weights)
    mats, off = [], 0
    shapes = [(hidden_dim, input_dim)] + [(hidden_dim, hidden_dim)] * (num_layers - 1) + [(output_dim, hidden_dim)]
    for o, i in shapes:
        mats.append(w[off:off + o * i].reshape(o, i))
        off += o * i
    return mats


def mlp_forward(x, weights, input_dim, output_dim, hidden_dim, num_layers, act=0, out_act=6,
                fp16=True):
    """fp16 storage between layers (like the fused kernel; fp16=False keeps
    float64), float64 accumulation. Returns (outputs [B, output_dim], list of
    hidden post-activations)."""
    st = np.float16 if fp16 else np.float64
    mats = mlp_layers(np.asarray(weights, st).astype(np.float64), input_dim, output_dim,
                      hidden_dim, num_layers)
    h = np.asarray(x, st)
    hs = []
    for li, W in enumerate(mats):
        z = h.astype(np.float64) @ W.T
        if li < len(mats) - 1:
            h = _act(act, z).astype(st)
            hs.append(h)
        else:
            h = _act(out_act, z).astype(st)
    return h, hs


def mlp_backward(grad, x, weights, input_dim, output_dim, hidden_dim, num_layers, act=0,
                 fp16=True):
    """float64 backward with fp16-rounded deltas (like the fused kernel; fp16=False
    keeps float64). Returns (grad_inputs [B, in], grad_weights float64 flat)."""
    st = np.float16 if fp16 else np.float64
    mats = mlp_layers(np.asarray(weights, st).astype(np.float64), input_dim, output_dim,
                      hidden_dim, num_layers)
    _, hs = mlp_forward(x, weights, input_dim, output_dim, hidden_dim, num_layers, act, fp16=fp16)
    ins = [np.asarray(x, st).astype(np.float64)] + [h.astype(np.float64) for h in hs]
    d = np.asarray(grad, st).astype(np.float64)
    gws = [None] * len(mats)
    for li in range(len(mats) - 1, -1, -1):
        gws[li] = d.T @ ins[li]
        g_in = d @ mats[li]
        if li > 0:
            d = _act_bwd(act, g_in, ins[li]).astype(st).astype(np.float64)
        else:
            grad_inputs = g_in.astype(st)
    return grad_inputs, np.concatenate([g.reshape(-1) for g in gws])


def mlp_backward_error_bound(grad, x, weights, input_dim, output_dim, hidden_dim, num_layers):
    """Per-element error scale of mlp_backward's grad_inputs for a kernel that
    accumulates in fp32 instead of float64 (ReLU hidden layers). Returns
    (mag, flip):
      * mag: |grad| pushed back through |W| with the fp16 forward's ReLU masks,
        the sum of the absolute terms each grad_input is made of; an fp16
        rounding of a delta on the way moves the result by at most 2^-11 of it
        per rounded layer;
      * flip: what ReLU units whose pre-activation sits within the accumulation
        error of zero (|z| <= 2^-14 sum|terms| + 2^-24: fp32 vs float64 sums,
        and fp16's flush of tiny positives to zero) can add when their mask
        differs -- their whole delta, pushed back through |W|.
    A grad_input within  layers * 2^-11 * mag + flip  (+ the fp16 ulps of the
    value) of the oracle is consistent with it."""
    st = np.float16
    W = mlp_layers(np.asarray(weights, st).astype(np.float64), input_dim, output_dim, hidden_dim, num_layers)
    A = [np.abs(w) for w in W]
    h = np.asarray(x, st).astype(np.float64)
    hs, amb = [], []
    for li in range(len(W) - 1):
        z, za = h @ W[li].T, np.abs(h) @ A[li].T
        amb.append(np.abs(z) <= 2.0 ** -14 * za + 2.0 ** -24)
        h = np.maximum(z, 0).astype(st).astype(np.float64)
        hs.append(h)
    D = np.abs(np.asarray(grad, st).astype(np.float64))
    F = np.zeros_like(D)
    for li in range(len(W) - 1, -1, -1):
        G, FG = D @ A[li], F @ A[li]
        if li == 0:
            return G, FG
        opened = (hs[li - 1] > 0) | amb[li - 1]
        F = FG * opened + G * amb[li - 1]
        D = G * opened


def trunc_exp(x):
    return np.exp(np.asarray(x, np.float32))


def trunc_exp_grad(x, g):
    return np.asarray(g, np.float32) * np.exp(np.clip(np.asarray(x, np.float32), -15, 15))


# ---- freqencoder (freqencoder/src/freqencoder.cu) ---------------------------

def freq_encode_forward(inputs, degree):
    """[B, D] -> [B, D (1 + 2 degree)] (kernel_freq, freqencoder.cu:30-59):
    [x, sin(2^0 x), sin(2^0 x + pi/2), ..., sin(2^(deg-1) x + pi/2)]. The
    argument is formed in float32 as the kernel does (scalbnf(x, f) exact, then
    + float(pi / 2) rounded); the sine itself is evaluated in float64 (the
    kernel's __sinf approximation is what the tests bound). Also returns the
    float32 arguments, which the tolerance scales with."""
    x = np.asarray(inputs, np.float32)
    B, D = x.shape
    out, args = [x.astype(np.float64)], [np.zeros_like(x)]
    half_pi = np.float32(np.pi / 2)
    for f in range(degree):
        a = (x * np.float32(2.0 ** f)).astype(np.float32)
        for ph in (np.float32(0.0), half_pi):
            arg = (a + ph).astype(np.float32)
            out.append(np.sin(arg.astype(np.float64)))
            args.append(arg)
    return np.concatenate(out, axis=1), np.concatenate(args, axis=1)


def freq_encode_backward(grad, outputs, D, degree):
    """grad_inputs [B, D] = grad[:, :D] + sum_f 2^f (g_sin * out_cos - g_cos *
    out_sin), from the saved outputs (kernel_freq_backward,
    freqencoder.cu:63-94), in float64."""
    g = np.asarray(grad, np.float64)
    o = np.asarray(outputs, np.float64)
    r = g[:, :D].copy()
    for f in range(degree):
        s = D + 2 * D * f
        r += 2.0 ** f * (g[:, s:s + D] * o[:, s + D:s + 2 * D] - g[:, s + D:s + 2 * D] * o[:, s:s + D])
    return r

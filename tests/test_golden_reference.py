"""Parity against fixtures produced by the reference's own Python
(tests/golden/make_golden.py, run where /root/reference exists; the fixtures
are data and travel, the reference does not):

* renderer_run_reference.npz — NeRFRenderer.run (nerf/renderer.py:126-254) on
  an analytic field, upsample_steps=0, perturb=False: the samples the field
  saw, its sigma / rgb, and run()'s image, weights_sum and depth. The same
  samples go through the oracle's and the HIP composite_rays_train_forward
  (raymarching.cu:500-577) with T_thresh = 0 (no early stop, as run() has
  none): image (+ the white background run() mixes in) and weights_sum
  within 1e-5 of run()'s cumprod compositing, depth within 1e-5.
* get_rays_reference.npz — get_rays (nerf/utils.py:52-136) for whole images
  and a seeded random batch: this repo's torch get_rays (nerf/utils.py) and
  the device sampler of the fused step (ngp_lego_rays, csrc/ngp_head.h
  lego_ray) on the same poses / intrinsics / pixels.
* nerf_matrix_reference.npz — nerf_matrix_to_ngp (nerf/provider.py:19-27).
"""
import os

import numpy as np
import pytest
import torch

import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return dict(np.load(os.path.join(GOLDEN, name)))


def _run_samples(f):
    """run()'s uniform samples (renderer.py:148-160, 206-207) restated with the
    same torch ops: z_vals, clipped xyzs, deltas, and the normalised depths
    (:226) as the composite kernel's accumulated real deltas."""
    ro, rd = torch.from_numpy(f["rays_o"]), torch.from_numpy(f["rays_d"])
    nears, fars = torch.from_numpy(f["nears"])[:, None], torch.from_numpy(f["fars"])[:, None]
    T, N = int(f["num_steps"]), ro.shape[0]
    z = torch.linspace(0.0, 1.0, T).unsqueeze(0).expand((N, T))
    z_vals = nears + (fars - nears) * z
    sample_dist = (fars - nears) / T
    xyzs = ro.unsqueeze(-2) + rd.unsqueeze(-2) * z_vals.unsqueeze(-1)
    aabb = torch.tensor([-1.0] * 3 + [1.0] * 3)
    xyzs = torch.min(torch.max(xyzs, aabb[:3]), aabb[3:])
    deltas = z_vals[..., 1:] - z_vals[..., :-1]
    deltas = torch.cat([deltas, sample_dist * torch.ones_like(deltas[..., :1])], dim=-1)
    ori = ((z_vals - nears) / (fars - nears)).clamp(0, 1)
    real = torch.cat([ori[:, :1], ori[:, 1:] - ori[:, :-1]], -1)
    d2 = torch.stack([deltas, real], -1).reshape(-1, 2).numpy().astype(np.float32)
    rays = np.stack([np.arange(N), np.arange(N) * T, np.full(N, T)], -1).astype(np.int32)
    return xyzs.reshape(-1, 3).numpy(), d2, rays


def test_run_samples_restated_bit_exact():
    f = _load("renderer_run_reference.npz")
    xyzs, _, _ = _run_samples(f)
    assert np.array_equal(xyzs.view(np.uint32), f["xyzs"].view(np.uint32))


def _check_composite(f, ws, depth, image):
    img = image + (1 - ws)[:, None]  # bg_color = 1 (renderer.py:237-240)
    assert f["weights_sum"].max() > 0.5 and f["weights_sum"].min() < 0.5  # opaque and see-through rays
    np.testing.assert_allclose(ws, f["weights_sum"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(img, f["image"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(depth, f["depth"], rtol=1e-5, atol=1e-5)


def test_oracle_composite_matches_reference_run():
    f = _load("renderer_run_reference.npz")
    _, deltas, rays = _run_samples(f)
    sigma = (f["sigma"] * f["density_scale"]).astype(np.float32)
    ws, depth, image = oracle.composite_rays_train_forward(sigma, f["rgb"], deltas, rays, 0.0)
    _check_composite(f, ws, depth, image)


@pytest.mark.gpu
def test_hip_composite_matches_reference_run(cuda):
    import raymarching
    f = _load("renderer_run_reference.npz")
    _, deltas, rays = _run_samples(f)
    sigma = torch.from_numpy((f["sigma"] * f["density_scale"]).astype(np.float32)).to(cuda)
    rgbs = torch.from_numpy(f["rgb"]).to(cuda)
    ws, depth, image = raymarching.composite_rays_train(sigma, rgbs, torch.from_numpy(deltas).to(cuda),
                                                       torch.from_numpy(rays).to(cuda), 0.0)
    _check_composite(f, ws.cpu().numpy(), depth.cpu().numpy(), image.cpu().numpy())


# ------------------------------------------------- composite backward (autograd)

def _grad_close(got, ref, what, rel=1e-3):
    """Elementwise 1e-3 rel + 1e-3 of the largest magnitude, and 1e-3 rel-norm."""
    g, r = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    assert g.shape == r.shape and np.isfinite(g).all(), what
    err = float(np.linalg.norm(g - r) / max(np.linalg.norm(r), 1e-30))
    assert err <= rel, (what, err)
    tol = rel * np.abs(r) + rel * np.abs(r).max()
    assert (np.abs(g - r) <= tol).all(), (what, float(np.abs(g - r).max()), float(np.abs(r).max()))
    return err


def _backward_case():
    """renderer_run_backward_reference.npz: run()'s samples as the composite
    kernels' inputs, and the kernel-side gradients of the fixture's linear
    functional: run()'s image includes the white background, so
    d/d weights_sum = gW - sum_c gI (renderer.py:240)."""
    f = _load("renderer_run_backward_reference.npz")
    _, deltas, rays = _run_samples(f)
    g_ws = (f["gW"] - f["gI"].sum(-1)).astype(np.float32)
    return f, deltas, rays, g_ws


def test_oracle_composite_backward_matches_reference_autograd():
    """oracle.composite_rays_train_backward (raymarching.cu:601-691) against
    torch autograd of the reference's run() compositing (renderer.py:206-240):
    d/d sigma and d/d rgb of sum(gI image) + sum(gD depth) + sum(gW ws)."""
    f, deltas, rays, g_ws = _backward_case()
    sigma = (f["sigma"] * f["density_scale"]).astype(np.float32)
    ws, depth, image = oracle.composite_rays_train_forward(sigma, f["rgb"], deltas, rays, 0.0)
    np.testing.assert_allclose(image + (1 - ws)[:, None], f["image"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(depth, f["depth"], rtol=1e-5, atol=1e-5)
    g_sig, g_rgb = oracle.composite_rays_train_backward(g_ws, f["gD"], f["gI"], sigma, f["rgb"], deltas, rays,
                                                        ws, depth, image, 0.0)
    _grad_close(g_sig, f["d_sigma"], "d sigma")
    _grad_close(g_rgb, f["d_rgb"], "d rgb")


def test_oracle_composite_backward_is_zero_past_termination():
    """The premise of the live-row backwards (nerf/fused.py options live_rows): the
    reference's composite backward stops at a ray's early termination
    (`if (T < T_thresh) break;`, raymarching.cu:680), so every sample past it
    has an exactly zero sigma and rgb gradient. Checked on the oracle's
    restatement with dense rays that terminate inside their samples."""
    rng = np.random.default_rng(7)
    N, S, T_thresh = 64, 96, 1e-4
    counts = rng.integers(1, S + 1, N)
    offsets = np.concatenate([[0], np.cumsum(counts)[:-1]])
    rays = np.stack([np.arange(N), offsets, counts], 1).astype(np.int32)
    M = int(counts.sum())
    sigma = rng.uniform(0.0, 60.0, M).astype(np.float32)
    rgb = rng.uniform(0.0, 1.0, (M, 3)).astype(np.float32)
    deltas = np.stack([rng.uniform(0.005, 0.02, M), rng.uniform(0.005, 0.02, M)], 1).astype(np.float32)
    ws, depth, image = oracle.composite_rays_train_forward(sigma, rgb, deltas, rays, T_thresh)
    g_ws = rng.normal(size=N).astype(np.float32)
    g_sig, g_rgb = oracle.composite_rays_train_backward(g_ws, np.zeros(N, np.float32),
                                                        rng.normal(size=(N, 3)).astype(np.float32), sigma, rgb,
                                                        deltas, rays, ws, depth, image, T_thresh)
    terminated = 0
    for n in range(N):
        o, c = int(offsets[n]), int(counts[n])
        T, stop = 1.0, c
        for k in range(c):  # the first sample after which T < T_thresh (float32, as the kernel)
            T = np.float32(T) * np.float32(1.0 - (1.0 - np.exp(np.float32(-sigma[o + k] * deltas[o + k, 0]))))
            if T < T_thresh:
                stop = k + 1
                break
        terminated += stop < c
        assert not g_sig[o + stop:o + c].any() and not g_rgb[o + stop:o + c].any(), n
        assert g_rgb[o:o + stop].any(), n  # the live samples do carry a gradient
    assert terminated > N // 2  # most rays end early: the rows the live-row backwards skip


@pytest.mark.gpu
def test_hip_composite_backward_matches_reference_autograd(cuda, parity_report):
    """The HIP composite_rays_train backward through the reference-API autograd
    Function (raymarching.py:238-289) against the reference's autograd."""
    import raymarching
    f, deltas, rays, g_ws = _backward_case()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    sigma = t((f["sigma"] * f["density_scale"]).astype(np.float32)).requires_grad_(True)
    rgbs = t(f["rgb"]).requires_grad_(True)
    ws, depth, image = raymarching.composite_rays_train(sigma, rgbs, t(deltas), t(rays), 0.0)
    g_sig, g_rgb = torch.autograd.grad([ws, depth, image], [sigma, rgbs], [t(g_ws), t(f["gD"]), t(f["gI"])])
    e1 = _grad_close(g_sig.cpu().numpy(), f["d_sigma"], "d sigma")
    e2 = _grad_close(g_rgb.cpu().numpy(), f["d_rgb"], "d rgb")
    parity_report(f"vs reference run() autograd: d_sigma rel {e1:.2e}, d_rgb rel {e2:.2e}")


@pytest.mark.gpu
def test_fused_composite_loss_matches_reference_autograd(cuda, parity_report):
    """The fused step's k_composite_loss (composite + white background + MSE +
    composite backward + trunc_exp / sigmoid backward, csrc/nerf_fused.hip)
    against autograd of the reference's run() + MSE (renderer.py:206-240,
    nerf/utils.py train_step): d mse / d h0 and d mse / d (colour logits),
    loss-scaled fp16 outputs divided by the scale; loss within 1e-4."""
    import _ngp_native as nat
    f, deltas, rays, _ = _backward_case()
    N, M = rays.shape[0], deltas.shape[0]
    scale = 65536.0  # GradScaler's init_scale
    h = np.zeros((M, 16), np.float16)
    h[:, 0] = f["h0"]
    col = np.zeros((M, 16), np.float16)
    col[:, :3] = f["logit"]
    assert np.array_equal(h[:, 0].astype(np.float32), f["h0"]) and np.array_equal(col[:, :3].astype(np.float32),
                                                                                 f["logit"])
    sigma = (np.float32(f["density_scale"]) * np.exp(f["h0"])).astype(np.float32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    d_sigma, d_col, d_h, d_del, d_rays, d_gt = map(t, (sigma, col, h, deltas, rays, f["gt"]))
    d_bg = torch.ones(N, 3, device=cuda)
    state = torch.zeros(nat.lib().ngp_fused_state_bytes(), dtype=torch.uint8, device=cuda)
    nat.check(nat.lib().ngp_fused_state_init(nat.ptr(state), scale, nat.stream_of(state)), "state_init")
    g_col = torch.zeros(M, 16, dtype=torch.float16, device=cuda)
    g_h = torch.zeros(M, 16, dtype=torch.float16, device=cuda)
    img = torch.zeros(N, 3, device=cuda)
    ws = torch.zeros(N, device=cuda)
    loss = torch.zeros(N, device=cuda)
    P = nat.ptr
    nat.check(nat.lib().ngp_nerf_composite_loss(
        P(d_sigma), P(d_col), P(d_h), P(d_del), P(d_rays), M, N, 0.0, float(f["density_scale"]), P(d_gt), 3,
        P(d_bg), P(state), P(g_col), P(g_h), P(img), P(ws), P(loss), nat.stream_of(img)), "composite_loss")
    torch.cuda.synchronize()
    np.testing.assert_allclose(img.cpu().numpy(), f["image"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ws.cpu().numpy(), f["weights_sum"], rtol=1e-5, atol=1e-5)
    got_loss = float(loss.double().sum().item()) / N
    assert abs(got_loss - float(f["mse"])) <= 1e-4 * float(f["mse"]), (got_loss, float(f["mse"]))
    gh0 = g_h[:, 0].float().cpu().numpy() / scale
    gl = g_col[:, :3].float().cpu().numpy() / scale
    assert (g_col[:, 3:] == 0).all() and (g_h[:, 1:] == 0).all()
    e1 = _grad_close(gh0, f["d_h0"], "d mse / d h0")
    e2 = _grad_close(gl, f["d_logit"], "d mse / d logit")
    parity_report(f"vs reference run()+MSE autograd: d_h0 rel {e1:.2e}, d_logit rel {e2:.2e}, loss {got_loss:.6f}")


def test_torch_get_rays_matches_reference():
    from nerf.utils import get_rays
    f = _load("get_rays_reference.npz")
    poses = torch.from_numpy(f["poses"])
    H, W = int(f["H"]), int(f["W"])
    out = get_rays(poses, f["intrinsics"], H, W, -1)
    np.testing.assert_array_equal(out["rays_o"].numpy(), f["rays_o"])
    np.testing.assert_allclose(out["rays_d"].numpy(), f["rays_d"], rtol=0, atol=1e-6)
    torch.manual_seed(int(f["seed"]))
    part = get_rays(poses[:1], f["intrinsics"], H, W, int(f["N"]))
    np.testing.assert_array_equal(part["inds"].numpy(), f["inds_part"])
    np.testing.assert_allclose(part["rays_d"].numpy(), f["rays_d_part"], rtol=0, atol=1e-6)
    np.testing.assert_array_equal(part["rays_o"].numpy(), f["rays_o_part"])


def test_nerf_matrix_to_ngp_matches_reference():
    from nerf.provider import nerf_matrix_to_ngp
    f = _load("nerf_matrix_reference.npz")
    for k, (s, o) in enumerate(zip(f["scales"], f["offsets"])):
        for j, p in enumerate(f["poses"]):
            got = nerf_matrix_to_ngp(p, scale=float(s), offset=[float(v) for v in o])
            np.testing.assert_array_equal(got, f["out"][k, j])


def _mix32(x):
    with np.errstate(over="ignore"):
        x = np.asarray(x, np.uint32)
        x = x ^ (x >> np.uint32(16)); x = x * np.uint32(0x7feb352d)
        x = x ^ (x >> np.uint32(15)); x = x * np.uint32(0x846ca68b)
        return x ^ (x >> np.uint32(16))


def _rng_u32(seed, a, b, c):
    """csrc/ngp_head.h rng_u32, restated in numpy uint32."""
    with np.errstate(over="ignore"):
        inner = _mix32(np.asarray(b, np.uint32) ^ _mix32(np.uint32(c) + np.uint32(0x85ebca6b)))
        return _mix32(np.uint32(seed) ^ _mix32(np.uint32(a) + np.uint32(0x9e3779b9) * inner))


@pytest.mark.gpu
def test_device_sampler_matches_reference_get_rays(cuda):
    """The fused step's sampler on the fixture's poses and intrinsics: each
    ray equals the reference get_rays ray of the pixel and pose the counter
    RNG picked (pose = rng(seed, draw, ~0, 0) % n_poses, pixel = rng(seed,
    draw, ray, 1) % (H W))."""
    import ctypes

    import _ngp_native as nat
    f = _load("get_rays_reference.npz")
    H, W, n_poses = int(f["H"]), int(f["W"]), f["poses"].shape[0]
    N, seed = 2048, 17
    poses = torch.from_numpy(f["poses"]).to(cuda)
    z = lambda *s: torch.zeros(*s, device=cuda)  # noqa: E731
    rays_o, rays_d, rgba, bg = z(N, 3), z(N, 3), z(N, 4), z(N, 3)
    nears, fars, noises = z(N), z(N), z(N)
    counter = torch.zeros(2, dtype=torch.int32, device=cuda)
    state = torch.zeros(nat.lib().ngp_fused_state_bytes(), dtype=torch.uint8, device=cuda)
    nat.check(nat.lib().ngp_fused_state_init(nat.ptr(state), 1.0, nat.stream_of(state)), "state_init")
    intr = (ctypes.c_float * 4)(*[float(v) for v in f["intrinsics"]])
    box = (ctypes.c_float * 9)(-0.1, -0.1, -0.1, 0.1, 0.1, 0.1, 1, 1, 1)
    aabb = (ctypes.c_float * 6)(-1, -1, -1, 1, 1, 1)
    P = nat.ptr
    for draw in range(3):
        nat.check(nat.lib().ngp_lego_rays(P(poses), n_poses, intr, H, W, N, box, 1, aabb, 0.2, seed, P(state),
                                          P(rays_o), P(rays_d), P(rgba), P(bg), P(nears), P(fars), P(noises),
                                          P(counter), None, nat.stream_of(poses)), "lego_rays")
        torch.cuda.synchronize()
        pose = int(_rng_u32(seed, draw, 0xFFFFFFFF, 0) % np.uint32(n_poses))
        pix = (_rng_u32(seed, draw, np.arange(N, dtype=np.uint32), 1) % np.uint32(H * W)).astype(np.int64)
        np.testing.assert_array_equal(rays_o.cpu().numpy(), f["rays_o"][pose][pix])
        np.testing.assert_allclose(rays_d.cpu().numpy(), f["rays_d"][pose][pix], rtol=0, atol=2e-6)


# ---------------------------------------------------------------- freqencoder

def freq_forward_tol(args):
    """|sin approximation - sin| bound for a float32 argument: a 2^-22
    absolute floor plus 2^-22 of |arg| (the float32 argument reduction of
    sin(arg) and of the + pi/2 phase lose |arg| * 2^-24 each)."""
    return 2.0 ** -22 + np.abs(args.astype(np.float64)) * 2.0 ** -22


def freq_backward_tol(gy, args, D, degree, fwd_tol):
    """Per input: sum over the 2 deg terms of 2^f |grad| times the forward
    bound of the output it multiplies, plus float32 summation rounding."""
    tol = np.zeros((gy.shape[0], D))
    mag = np.abs(gy[:, :D]).astype(np.float64)
    for f in range(degree):
        s = D + 2 * D * f
        gs, gc = np.abs(gy[:, s:s + D]), np.abs(gy[:, s + D:s + 2 * D])
        tol += 2.0 ** f * (gs * fwd_tol[:, s + D:s + 2 * D] + gc * fwd_tol[:, s:s + D])
        mag += 2.0 ** f * (gs + gc)
    return tol + mag * 2.0 ** -21


@pytest.mark.parametrize("deg", [4, 10])
def test_freq_oracle_matches_reference_torch_encoder(deg):
    """oracle.freq_encode_* (freqencoder.cu:30-94) against the reference's
    pure-torch FreqEncoder (encoding.py:5-43, cos as torch.cos) and its
    autograd input gradient."""
    f = _load("freq_reference.npz")
    x, y, gy, gx = f[f"x{deg}"], f[f"y{deg}"], f[f"gy{deg}"], f[f"gx{deg}"]
    out, args = oracle.freq_encode_forward(x, deg)
    assert out.shape == y.shape == (x.shape[0], 3 * (1 + 2 * deg))
    tol = freq_forward_tol(args)
    assert np.array_equal(out[:, :3], x)
    assert (np.abs(out - y) <= tol).all(), float((np.abs(out - y) / tol).max())
    gi = oracle.freq_encode_backward(gy, out, 3, deg)
    btol = freq_backward_tol(gy, args, 3, deg, tol)
    assert (np.abs(gi - gx) <= btol).all(), float((np.abs(gi - gx) / btol).max())

"""CPU: pin the oracle against the reference's own fixtures and against
analytic properties of each restated kernel (no GPU needed)."""
import math
import os

import numpy as np
import pytest
import torch

import oracle
from helpers import box_bitfield, lego_boxes, lego_rays

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


# ---------------------------------------------------------- golden fixtures

def test_sh_matches_reference_torch_oracle():
    """oracle.sh_encode vs the reference's SHEncoder_torch (testing/test_shencoder.py)
    on unit vectors, degrees 1..5. Degree >= 3 uses identities valid only on the
    unit sphere in one of the two forms (test_shencoder.py:73), hence the tolerance."""
    f = np.load(os.path.join(GOLD, "sh_reference.npz"))
    d = f["inputs"]
    for deg in range(1, 6):
        np.testing.assert_allclose(oracle.sh_encode(d, deg), f[f"deg{deg}"], rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("name", ["sigma", "color", "small"])
def test_mlp_matches_reference_torch_oracle(name):
    """oracle MLP (FFMLP layer semantics) vs the reference's nn.Linear MLP
    (testing/test_ffmlp.py:11-43): forward, input grads, weight grads (fp64 path)."""
    f = np.load(os.path.join(GOLD, "mlp_reference.npz"))
    i, o, h, nl = (int(v) for v in f[f"{name}_dims"])
    w, x, g = f[f"{name}_weights"], f[f"{name}_x"], f[f"{name}_g"]
    y, _ = oracle.mlp_forward(x, w, i, o, h, nl, fp16=False)
    np.testing.assert_allclose(y, f[f"{name}_y"], rtol=1e-4, atol=1e-5)
    gx, gw = oracle.mlp_backward(g, x, w, i, o, h, nl, fp16=False)
    np.testing.assert_allclose(gx, f[f"{name}_gx"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(gw, f[f"{name}_gw"], rtol=1e-4, atol=1e-4)


def test_trunc_exp_matches_reference():
    f = np.load(os.path.join(GOLD, "trunc_exp_reference.npz"))
    np.testing.assert_allclose(oracle.trunc_exp(f["x"]), f["y"], rtol=1e-6)
    np.testing.assert_allclose(oracle.trunc_exp_grad(f["x"], np.ones_like(f["x"])), f["gx"], rtol=1e-6)


def test_product_trunc_exp_matches_reference_cpu():
    """activation.trunc_exp (product) on CPU tensors vs the fixture."""
    from activation import trunc_exp
    f = np.load(os.path.join(GOLD, "trunc_exp_reference.npz"))
    x = torch.from_numpy(f["x"]).requires_grad_(True)
    y = trunc_exp(x)
    y.backward(torch.ones_like(y))
    np.testing.assert_allclose(y.detach().numpy(), f["y"], rtol=1e-6)
    np.testing.assert_allclose(x.grad.numpy(), f["gx"], rtol=1e-6)


# ---------------------------------------------------------------- fp16 model

def test_half_conversion_matches_numpy():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.standard_normal(100000).astype(np.float32) * s
                        for s in (1e-8, 1e-5, 1e-2, 1, 1e3, 7e4)])
    with np.errstate(over="ignore"):
        ref = x.astype(np.float16)
    assert np.array_equal(oracle.f2h(x).view(np.uint16), ref.view(np.uint16))


# ---------------------------------------------------------------- grid encode

LEGO_S = float(np.exp2(np.log2(2048 / 16) / 15))


def test_grid_offsets_lego():
    off = oracle.grid_offsets(3, 16, 2, 16, LEGO_S, 19)
    assert off[-1] == 6119864 and off[-1] * 2 == 12239728  # SURVEY §8 table size
    # levels 0-4 dense ((res+1)^3 rounded to 8), 5-15 hashed (2^19)
    sizes = np.diff(off)
    assert list(sizes[:5]) == [int(np.ceil((int(np.ceil(16 * LEGO_S ** l)) + 1) ** 3 / 8) * 8) for l in range(5)]
    assert all(s == 2 ** 19 for s in sizes[5:])


def test_grid_module_layout_on_cpu():
    from gridencoder import GridEncoder
    enc = GridEncoder(desired_resolution=2048)
    assert enc.embeddings.shape == (6119864, 2)
    assert np.array_equal(enc.offsets.numpy(), oracle.grid_offsets(3, 16, 2, 16, enc.per_level_scale, 19))
    assert float(enc.embeddings.abs().max()) <= 1e-4
    assert set(enc.state_dict().keys()) == {"embeddings", "offsets"}


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_grid_partition_of_unity(dt):
    """A constant table interpolates to the constant (sum of corner weights = 1)."""
    off = oracle.grid_offsets(3, 8, 2, 16, 1.5, 14)
    emb = np.full((int(off[-1]), 2), 0.375, dt)
    x = np.random.default_rng(1).random((2000, 3), dtype=np.float32)
    out, _ = oracle.grid_encode_forward(x, emb, off, 1.5, 16)
    np.testing.assert_allclose(out, 0.375, rtol=1e-6)


def test_grid_backward_is_forward_transpose():
    """Forward is linear in the table: <fwd(E), G> == <E, bwd(G)> (float64)."""
    rng = np.random.default_rng(2)
    off = oracle.grid_offsets(3, 6, 2, 8, 1.6, 12)
    E = rng.standard_normal((int(off[-1]), 2))
    x = rng.random((500, 3), dtype=np.float32)
    G = rng.standard_normal((500, 12))
    out, _ = oracle.grid_encode_forward(x, E, off, 1.6, 8)
    bwd = oracle.grid_encode_backward(G, x, off, 2, 1.6, 8)
    assert abs((out * G).sum() - (E * bwd).sum()) < 1e-9 * max(1.0, abs((out * G).sum()))


def test_grid_dydx_matches_finite_differences():
    rng = np.random.default_rng(3)
    off = oracle.grid_offsets(3, 4, 2, 4, 2.0, 12)
    E = rng.standard_normal((int(off[-1]), 2))
    x = rng.uniform(0.1, 0.9, (50, 3)).astype(np.float32)
    _, dy = oracle.grid_encode_forward(x, E, off, 2.0, 4, calc_dy_dx=True)
    dy = dy.reshape(50, 4, 3, 2)
    eps = 1e-3
    for d in range(3):
        xp, xm = x.copy(), x.copy()
        xp[:, d] += eps; xm[:, d] -= eps
        fp, _ = oracle.grid_encode_forward(xp, E, off, 2.0, 4)
        fm, _ = oracle.grid_encode_forward(xm, E, off, 2.0, 4)
        fd = ((fp - fm) / (2 * eps)).reshape(50, 4, 2)
        # piecewise linear: exact away from cell boundaries; compare the median error
        err = np.abs(fd - dy[:, :, d, :])
        assert np.median(err) < 1e-3


def test_grid_out_of_bounds_zero():
    off = oracle.grid_offsets(3, 4, 2, 4, 2.0, 10)
    E = np.ones((int(off[-1]), 2), np.float32)
    x = np.array([[-0.01, 0.5, 0.5], [0.5, 1.01, 0.5], [0.5, 0.5, 0.5]], np.float32)
    out, _ = oracle.grid_encode_forward(x, E, off, 2.0, 4)
    assert np.all(out[:2] == 0) and np.allclose(out[2], 1)


# ---------------------------------------------------------------- raymarching

def test_morton_roundtrip_and_known_values():
    c = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1], [127, 127, 127], [5, 3, 9]], np.int32)
    m = oracle.morton3D(c)
    assert list(m[:4]) == [0, 1, 2, 4] and m[4] == 2 ** 21 - 1
    assert np.array_equal(oracle.morton3D_invert(m), c)


def test_packbits_bit_order():
    g = np.zeros(16, np.float32)
    g[[0, 3, 8, 15]] = 1.0
    assert list(oracle.packbits(g, 0.5)) == [0b00001001, 0b10000001]


def test_near_far_slab():
    ro = np.array([[0, 0, -3], [5, 5, 5], [0, 0, 0.5]], np.float32)
    rd = np.array([[0, 0, 1], [1, 0, 0], [0, 0, 1]], np.float32)
    n, f = oracle.near_far_from_aabb(ro, rd, np.array([-1, -1, -1, 1, 1, 1], np.float32), 0.2)
    assert n[0] == 2 and f[0] == 4
    assert n[1] == f[1] == np.finfo(np.float32).max
    assert n[2] == np.float32(0.2) and f[2] == np.float32(0.5)


def _march(N=512, C=1, bound=1.0, dt_gamma=0.0, M=None):
    ro, rd = lego_rays(N, seed=4)
    if bound > 1:
        ro = ro * (bound / 2)
    aabb = np.array([-bound] * 3 + [bound] * 3, np.float32)
    n, f = oracle.near_far_from_aabb(ro, rd, aabb)
    bits = box_bitfield(lego_boxes(), cascade=C, bound=bound)
    noise = np.random.default_rng(5).random(N, dtype=np.float32)
    return bits, oracle.march_rays_train(ro, rd, bound, bits, C, 128, n, f, noise, M=M, dt_gamma=dt_gamma)


def test_march_samples_lie_in_occupied_cells():
    bits, (xyz, dirs, dl, rays, cnt) = _march()
    m = int(cnt[0])
    assert m > 0 and cnt[1] == 512
    assert np.array_equal(rays[:, 0], np.arange(512))
    assert rays[:, 2].sum() == m
    assert np.array_equal(rays[1:, 1], np.cumsum(rays[:-1, 2]))  # ray-order prefix sum
    p = xyz[:m]
    cell = np.clip(((p + 1) / 2 * 128).astype(np.int64), 0, 127)
    idx = oracle.morton3D(cell.astype(np.int32))
    occ = (bits[idx // 8] >> (idx % 8)) & 1
    assert occ.all()
    np.testing.assert_allclose(dl[:m, 0], 2 * math.sqrt(3) / 1024, rtol=1e-6)
    assert (dl[:m, 1] > 0).all()


def test_march_overflow_drops_whole_rays():
    _, full = _march()
    _, part = _march(M=1000)
    rays, cnt = part[3], part[4]
    assert np.array_equal(rays, full[3]) and np.array_equal(cnt, full[4])
    last_ok = np.nonzero(rays[:, 1] + rays[:, 2] <= 1000)[0]
    end = int((rays[last_ok, 1] + rays[last_ok, 2]).max())
    assert np.array_equal(part[0][:end], full[0][:end])


def test_march_cascade_and_dt_gamma():
    _, (xyz, _, dl, rays, cnt) = _march(N=256, C=2, bound=2.0, dt_gamma=1 / 128)
    m = int(cnt[0])
    assert m > 0
    assert (dl[:m, 0] >= 2 * math.sqrt(3) / 1024 * (1 - 1e-6)).all()
    assert (dl[:m, 0] <= 2 * math.sqrt(3) * 2 / 128 * (1 + 1e-6)).all()


def test_composite_matches_torch_formulation():
    """Front-to-back compositing equals the cumprod formulation of renderer.run()
    (renderer.py:206-230) for rays that never hit the T threshold."""
    rng = np.random.default_rng(6)
    N, S = 64, 40
    sig = rng.random((N, S)).astype(np.float32) * 5
    rgb = rng.random((N, S, 3)).astype(np.float32)
    dl = np.stack([np.full((N, S), 0.01), rng.random((N, S)) * 0.01], -1).astype(np.float32)
    rays = np.stack([np.arange(N), np.arange(N) * S, np.full(N, S)], -1).astype(np.int32)
    ws, dp, img = oracle.composite_rays_train_forward(sig.reshape(-1), rgb.reshape(-1, 3), dl.reshape(-1, 2), rays)
    alpha = 1 - np.exp(-sig.astype(np.float64) * dl[..., 0])
    T = np.cumprod(np.concatenate([np.ones((N, 1)), 1 - alpha], 1), 1)[:, :-1]
    w = alpha * T
    np.testing.assert_allclose(ws, w.sum(1), rtol=1e-5)
    np.testing.assert_allclose(img, (w[..., None] * rgb).sum(1), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(dp, (w * np.cumsum(dl[..., 1], 1)).sum(1), rtol=1e-5, atol=1e-7)


def test_composite_backward_matches_autograd():
    rng = np.random.default_rng(7)
    N, S = 32, 25
    sig = rng.random((N, S)) * 3
    rgb = rng.random((N, S, 3))
    dl = np.stack([np.full((N, S), 0.02), rng.random((N, S)) * 0.01], -1)
    rays = np.stack([np.arange(N), np.arange(N) * S, np.full(N, S)], -1).astype(np.int32)
    ts, tc = torch.tensor(sig, requires_grad=True), torch.tensor(rgb, requires_grad=True)
    alpha = 1 - torch.exp(-ts * torch.tensor(dl[..., 0]))
    T = torch.cumprod(torch.cat([torch.ones(N, 1, dtype=torch.float64), 1 - alpha], 1), 1)[:, :-1]
    w = alpha * T
    ws, img = w.sum(1), (w[..., None] * tc).sum(1)
    dp = (w * torch.tensor(np.cumsum(dl[..., 1], 1))).sum(1)
    gws, gd, gi = rng.standard_normal(N), rng.standard_normal(N), rng.standard_normal((N, 3))
    ((ws * torch.tensor(gws)).sum() + (dp * torch.tensor(gd)).sum() + (img * torch.tensor(gi)).sum()).backward()
    f32 = lambda a: np.asarray(a, np.float32)  # noqa: E731
    ows, odp, oimg = oracle.composite_rays_train_forward(f32(sig).reshape(-1), f32(rgb).reshape(-1, 3),
                                                         f32(dl).reshape(-1, 2), rays)
    gs, gc = oracle.composite_rays_train_backward(f32(gws), f32(gd), f32(gi), f32(sig).reshape(-1),
                                                  f32(rgb).reshape(-1, 3), f32(dl).reshape(-1, 2), rays,
                                                  ows, odp, oimg)
    np.testing.assert_allclose(gc.reshape(N, S, 3), tc.grad.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(gs.reshape(N, S), ts.grad.numpy(), rtol=1e-3, atol=1e-4)


def test_composite_early_termination_and_empty_rays():
    sig = np.array([1e4, 1.0, 1.0], np.float32)
    rgb = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1]], np.float32)
    dl = np.array([[0.01, 0.01]] * 3, np.float32)
    rays = np.array([[0, 0, 3], [1, 3, 0]], np.int32)
    ws, dp, img = oracle.composite_rays_train_forward(sig, rgb, dl, rays)
    np.testing.assert_allclose(img[0], [1, 0, 0], atol=1e-6)
    assert ws[1] == 0 and np.all(img[1] == 0)


def test_sh_jacobian_matches_autograd_degree4():
    f = np.load(os.path.join(GOLD, "sh_reference.npz"))
    d = f["inputs"][:64].astype(np.float64)
    jac = oracle.sh_encode_jacobian(d, 4)
    x = torch.tensor(d, requires_grad=True)
    vals = torch.tensor(oracle._sh_values(d[:, 0], d[:, 1], d[:, 2], 4, np.float64))
    assert vals.shape == (64, 16)
    # autograd of the same polynomials in torch
    xx, yy, zz = x[:, 0], x[:, 1], x[:, 2]
    v9 = 0.59004358992664352 * yy * (-3.0 * xx * xx + yy * yy)
    g, = torch.autograd.grad(v9.sum(), x)
    np.testing.assert_allclose(jac[:, :, 9], g.numpy(), rtol=1e-6, atol=1e-8)

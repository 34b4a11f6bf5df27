"""HIP kernels (through the C ABI / _backend shims) vs the CPU oracle.

Integer work (sample counts, offsets, ray table, Morton codes, bitfields) and
the grid-encoder / marching float outputs must be bit-exact; atomically
accumulated gradients are compared to the oracle's float64 scatter with a
tolerance; the MLP (fp16 MFMA, fp32 accumulate) against the float64 oracle
within fp16 tolerances written per test.
"""
import numpy as np
import pytest
import torch

import oracle
from helpers import box_bitfield, close16, lego_boxes, lego_rays

pytestmark = pytest.mark.gpu

LEGO_SCALE = float(np.exp2(np.log2(2048 / 16) / 15))  # desired_resolution 2048, bound 1


def t(a, dev, dtype=None):
    x = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return x if dtype is None else x.to(dtype)


# ------------------------------------------------------------------ grid encode

GRID_CASES = [
    # D, L, C, H, scale, log2T, gridtype, align_corners, interp, dtype, B
    (3, 16, 2, 16, LEGO_SCALE, 19, 0, False, 0, np.float16, 8192),
    (3, 16, 2, 16, LEGO_SCALE, 19, 0, False, 0, np.float32, 8192),
    (3, 8, 2, 16, 1.5, 14, 0, False, 0, np.float64, 1000),
    (2, 4, 1, 4, 2.0, 8, 0, False, 0, np.float32, 777),
    (3, 6, 4, 8, 1.7, 12, 1, False, 0, np.float32, 513),
    (3, 5, 8, 4, 2.0, 10, 0, True, 0, np.float16, 300),
    (3, 4, 2, 4, 2.0, 9, 0, False, 1, np.float32, 256),
    (4, 3, 2, 4, 2.0, 12, 0, False, 0, np.float32, 129),
]


def _grid_inputs(B, D, seed, oob=True):
    rng = np.random.default_rng(seed)
    x = rng.random((B, D), dtype=np.float32)
    if oob and B > 8:
        x[:4] = [[-1e-3] + [0.5] * (D - 1), [1.0] * D, [0.0] * D, [1.0 + 1e-6] + [0.2] * (D - 1)]
    return x


@pytest.mark.parametrize("case", GRID_CASES, ids=lambda c: f"D{c[0]}L{c[1]}C{c[2]}{np.dtype(c[9]).name}t{c[6]}a{int(c[7])}i{c[8]}")
def test_grid_forward_bit_exact(cuda, case):
    import gridencoder.backend as gb
    D, L, C, H, s, log2T, gt, ac, it, dt, B = case
    offsets = oracle.grid_offsets(D, L, C, H, s, log2T, ac)
    rng = np.random.default_rng(1)
    emb = (rng.standard_normal((int(offsets[-1]), C)) * 0.1).astype(dt)
    x = _grid_inputs(B, D, 2)
    ref, ref_dy = oracle.grid_encode_forward(x, emb, offsets, s, H, calc_dy_dx=True, gridtype=gt,
                                             align_corners=ac, interp=it, out_layout=0)
    tdt = {np.float16: torch.float16, np.float32: torch.float32, np.float64: torch.float64}[dt]
    out = torch.empty(L, B, C, dtype=tdt, device=cuda)
    dy = torch.empty(B, L * D * C, dtype=tdt, device=cuda)
    gb._backend.grid_encode_forward(t(x, cuda), t(emb, cuda), t(offsets, cuda), out, B, D, C, L,
                                    np.log2(s), H, dy, gt, ac, it)
    got = out.cpu().numpy()
    assert np.array_equal(got.view(np.uint8), ref.view(np.uint8)), \
        f"max abs diff {np.abs(got.astype(np.float64) - ref.astype(np.float64)).max()}"
    np.testing.assert_allclose(dy.cpu().numpy().astype(np.float64), ref_dy.astype(np.float64),
                               rtol=1e-5 if dt != np.float16 else 2e-3, atol=1e-6 if dt != np.float16 else 2e-3)
    # [B, L*C] layout is the same numbers
    out_bm = torch.empty(B, L * C, dtype=tdt, device=cuda)
    gb._backend.grid_encode_forward_bm(t(x, cuda), t(emb, cuda), t(offsets, cuda), out_bm, B, D, C, L,
                                       np.log2(s), H, None, gt, ac, it)
    assert torch.equal(out_bm.cpu(), torch.from_numpy(got).permute(1, 0, 2).reshape(B, L * C))


@pytest.mark.parametrize("case", GRID_CASES, ids=lambda c: f"D{c[0]}L{c[1]}C{c[2]}{np.dtype(c[9]).name}t{c[6]}a{int(c[7])}i{c[8]}")
def test_grid_backward_vs_scatter(cuda, case):
    import gridencoder.backend as gb
    D, L, C, H, s, log2T, gt, ac, it, dt, B = case
    offsets = oracle.grid_offsets(D, L, C, H, s, log2T, ac)
    x = _grid_inputs(B, D, 3)
    rng = np.random.default_rng(4)
    grad = rng.standard_normal((B, L * C)).astype(dt)
    ref = oracle.grid_encode_backward(grad, x, offsets, C, s, H, gt, ac, it, grad_layout=1)
    tdt = {np.float16: torch.float16, np.float32: torch.float32, np.float64: torch.float64}[dt]
    gemb = torch.zeros(int(offsets[-1]), C, dtype=tdt, device=cuda)
    emb = torch.zeros_like(gemb)
    gb._backend.grid_encode_backward_bm(t(grad, cuda), t(x, cuda), emb, t(offsets, cuda), gemb, B, D,
                                        C, L, np.log2(s), H, None, None, gt, ac, it)
    got = gemb.cpu().numpy().astype(np.float64)
    # reference [L, B, C] grad layout gives the same scatter
    gemb0 = torch.zeros_like(gemb)
    g0 = np.ascontiguousarray(grad.reshape(B, L, C).transpose(1, 0, 2))
    gb._backend.grid_encode_backward(t(g0, cuda), t(x, cuda), emb, t(offsets, cuda), gemb0, B, D, C,
                                     L, np.log2(s), H, None, None, gt, ac, it)
    got0 = gemb0.cpu().numpy().astype(np.float64)
    if dt == np.float16:
        # fp16 atomics round the running sum at every add (the reference
        # rounds each w * g as well, gridencoder.cu:322-328): against the exact
        # sum, allow 2^-8 of the entry's sum of |contributions| (4 fp16 ulps of
        # the largest partial sum)
        exact = oracle.grid_encode_backward(grad.astype(np.float64), x, offsets, C, s, H, gt, ac, it, grad_layout=1)
        mag = oracle.grid_encode_backward(np.abs(grad.astype(np.float64)), x, offsets, C, s, H, gt, ac, it,
                                          grad_layout=1)
        for g_ in (got, got0):
            err = np.abs(g_ - exact)
            assert (err <= 2.0 ** -8 * mag + 1e-7).all(), float((err / np.maximum(mag, 1e-30)).max())
            assert np.linalg.norm(g_ - exact) <= 1e-3 * np.linalg.norm(exact)
    else:  # unordered atomics: fp32 / fp64 sums reassociate
        np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(got0, ref, rtol=1e-4, atol=1e-5)


def test_grid_input_backward(cuda):
    import gridencoder.backend as gb
    D, L, C, H, s = 3, 6, 2, 8, 1.6
    offsets = oracle.grid_offsets(D, L, C, H, s, 12)
    rng = np.random.default_rng(5)
    emb = (rng.standard_normal((int(offsets[-1]), C)) * 0.1).astype(np.float32)
    B = 300
    x = _grid_inputs(B, D, 6, oob=False)
    grad = rng.standard_normal((B, L * C)).astype(np.float32)
    _, dy = oracle.grid_encode_forward(x, emb, offsets, s, H, calc_dy_dx=True)
    ref = oracle.grid_input_backward(grad, dy, B, D, C, L, grad_layout=1)
    dyt = torch.empty(B, L * D * C, device=cuda)
    out = torch.empty(B, L * C, device=cuda)
    gb._backend.grid_encode_forward_bm(t(x, cuda), t(emb, cuda), t(offsets, cuda), out, B, D, C, L,
                                       np.log2(s), H, dyt, 0, False, 0)
    gi = torch.zeros(B, D, device=cuda)
    gemb = torch.zeros(int(offsets[-1]), C, device=cuda)
    gb._backend.grid_encode_backward_bm(t(grad, cuda), t(x, cuda), t(emb, cuda), t(offsets, cuda),
                                        gemb, B, D, C, L, np.log2(s), H, dyt, gi, 0, False, 0)
    np.testing.assert_allclose(gi.cpu().numpy(), ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("D,L,C,log2T,gt,ac,dt", [(3, 16, 2, 19, 0, False, np.float32),
                                                    (3, 6, 4, 12, 1, False, np.float32),
                                                    (2, 5, 1, 10, 0, True, np.float32),
                                                    (3, 8, 2, 14, 0, False, np.float64)])
def test_grad_total_variation(cuda, D, L, C, log2T, gt, ac, dt):
    """grad_total_variation (gridencoder.cu:503-607) against the oracle's
    float64 image of the same per-point contributions (atomics unordered)."""
    import gridencoder.backend as gb
    H, s = 16, LEGO_SCALE if L == 16 else 1.6
    offsets = oracle.grid_offsets(D, L, C, H, s, log2T, ac)
    rng = np.random.default_rng(11)
    emb = (rng.standard_normal((int(offsets[-1]), C)) * 0.1).astype(dt)
    B = 20000
    x = _grid_inputs(B, D, 12).astype(dt)
    ref = oracle.grad_total_variation(x, emb, offsets, 1e-4, s, H, gt, ac)
    base = (rng.standard_normal(emb.shape) * 1e-6).astype(dt)  # the grad the TV term is added into
    grad = t(base, cuda)
    gb._backend.grad_total_variation(t(x, cuda), t(emb, cuda), grad, t(offsets, cuda), 1e-4, B, D, C, L,
                                     np.log2(s), H, gt, ac)
    got = grad.cpu().numpy().astype(np.float64) - base.astype(np.float64)
    assert np.abs(ref).max() > 0 and (ref != 0).sum() > 1000
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5 * np.abs(ref).max())
    # the module method: world inputs mapped to [0, 1], added into embeddings.grad
    from gridencoder import GridEncoder
    enc = GridEncoder(input_dim=D, num_levels=L, level_dim=C, base_resolution=H, per_level_scale=s,
                      log2_hashmap_size=log2T, gridtype=["hash", "tiled"][gt], align_corners=ac).to(cuda)
    with torch.no_grad():
        enc.embeddings.data = t(emb, cuda)
    enc.embeddings.grad = torch.zeros_like(enc.embeddings)
    enc.grad_total_variation(1e-4, inputs=t(x * 2 - 1, cuda), bound=1)
    x01 = ((t(x * 2 - 1, cuda) + 1) / 2).cpu().numpy()
    ref2 = oracle.grad_total_variation(x01, emb, offsets, 1e-4, s, H, gt, ac)
    np.testing.assert_allclose(enc.embeddings.grad.cpu().numpy().astype(np.float64), ref2, rtol=1e-4,
                               atol=1e-5 * np.abs(ref2).max())


def test_grid_module_autograd_autocast(cuda):
    from gridencoder import GridEncoder
    enc = GridEncoder(input_dim=3, num_levels=16, level_dim=2, base_resolution=16,
                      log2_hashmap_size=19, desired_resolution=2048).to(cuda)
    assert enc.embeddings.shape == (6119864, 2)
    torch.manual_seed(0)
    with torch.no_grad():
        enc.embeddings.normal_(0, 0.1)
    x = (torch.rand(4096, 3, device=cuda) * 2 - 1)
    with torch.autocast("cuda", dtype=torch.float16):
        y = enc(x, bound=1)
    assert y.dtype == torch.float16 and y.shape == (4096, 32)
    ref, _ = oracle.grid_encode_forward(((x.cpu().numpy() + 1) / 2).astype(np.float32),
                                        enc.embeddings.detach().cpu().numpy().astype(np.float16),
                                        enc.offsets.cpu().numpy(), enc.per_level_scale, 16)
    assert np.array_equal(y.detach().cpu().numpy().view(np.uint16), ref.view(np.uint16))
    g = torch.randn_like(y)
    y.backward(g)
    assert enc.embeddings.grad.dtype == torch.float32
    # the fp16 table grad (autocast) against the exact float64 scatter of the
    # half-rounded output grad: per entry within 2^-8 of its sum of
    # |contributions| (the fp16 bound of test_grid_backward_vs_scatter)
    g16 = g.half().double().cpu().numpy()
    x01 = ((x + 1) / 2).cpu().numpy().astype(np.float32)
    exact = oracle.grid_encode_backward(g16, x01, enc.offsets.cpu().numpy(), 2, enc.per_level_scale, 16)
    mag = oracle.grid_encode_backward(np.abs(g16), x01, enc.offsets.cpu().numpy(), 2, enc.per_level_scale, 16)
    got = enc.embeddings.grad.cpu().numpy().astype(np.float64)
    err = np.abs(got - exact)
    assert (err <= 2.0 ** -8 * mag + 1e-7).all(), float((err / np.maximum(mag, 1e-30)).max())
    assert np.linalg.norm(got - exact) <= 1e-3 * np.linalg.norm(exact)
    assert np.all(got[mag == 0] == 0)


# ---------------------------------------------------------------- ray marching

def _rays(N, seed, dev):
    ro, rd = lego_rays(N, seed=seed)
    return ro, rd


def _march_case(cuda, N, C=1, bound=1.0, dt_gamma=0.0, M=None, perturb_seed=0, max_steps=1024,
                bits=None, H=128):
    import raymarching.backend as rb
    ro, rd = lego_rays(N, seed=perturb_seed)
    if bound > 1:
        ro = ro * (bound / 2.0)
    aabb = np.array([-bound] * 3 + [bound] * 3, np.float32)
    nears, fars = oracle.near_far_from_aabb(ro, rd, aabb, 0.2)
    if bits is None:
        bits = box_bitfield(lego_boxes(), cascade=C, bound=bound, H=H)
    noises = np.random.default_rng(perturb_seed + 100).random(N, dtype=np.float32)
    Mr = M if M is not None else N * max_steps
    ref = oracle.march_rays_train(ro, rd, bound, bits, C, H, nears, fars, noises, M=Mr,
                                  dt_gamma=dt_gamma, max_steps=max_steps)
    xyzs = torch.zeros(Mr, 3, device=cuda); dirs = torch.zeros(Mr, 3, device=cuda)
    deltas = torch.zeros(Mr, 2, device=cuda)
    rays = torch.empty(N, 3, dtype=torch.int32, device=cuda)
    counter = torch.zeros(2, dtype=torch.int32, device=cuda)
    tn, tf = torch.empty(N, device=cuda), torch.empty(N, device=cuda)
    rb._backend.near_far_from_aabb(t(ro, cuda), t(rd, cuda), t(aabb, cuda), N, 0.2, tn, tf)
    assert np.array_equal(tn.cpu().numpy(), nears) and np.array_equal(tf.cpu().numpy(), fars)
    rb._backend.march_rays_train(t(ro, cuda), t(rd, cuda), t(bits, cuda), bound, dt_gamma, max_steps,
                                 N, C, H, Mr, tn, tf, xyzs, dirs, deltas, rays, counter, t(noises, cuda))
    return ref, (xyzs, dirs, deltas, rays, counter)


def _assert_march_equal(ref, got):
    rx, rdirs, rdel, rrays, rcnt = ref
    xyzs, dirs, deltas, rays, counter = [a.cpu().numpy() for a in got]
    assert np.array_equal(rays, rrays)
    assert np.array_equal(counter, rcnt)
    m = int(rcnt[0])
    assert m > 0
    assert np.array_equal(xyzs[:m].view(np.uint32), rx[:m].view(np.uint32))
    assert np.array_equal(dirs[:m].view(np.uint32), rdirs[:m].view(np.uint32))
    assert np.array_equal(deltas[:m].view(np.uint32), rdel[:m].view(np.uint32))


@pytest.mark.parametrize("N,C,bound,dt_gamma", [(4096, 1, 1.0, 0.0), (1000, 2, 2.0, 1 / 128), (77, 1, 1.0, 0.0),
                                                (1000, 2, 2.0, 0.0), (600, 3, 4.0, 0.0), (4096, 1, 1.0, 1 / 128),
                                                (600, 3, 4.0, 1 / 256), (900, 2, 2.0, 0.01), (300, 2, 2.0, 0.5)])
def test_march_rays_train_bit_exact(cuda, N, C, bound, dt_gamma):
    # one wave per ray, 64 speculative segments stitched (multi-level
    # cascades skip across whole segments); dt_gamma == 0: segment starts in
    # closed form, dt_gamma > 0: from the wave's records of the bare chain
    # (0.01: a rounded t * dt_gamma; 0.5: every step at dt_max)
    _assert_march_equal(*_march_case(cuda, N, C, bound, dt_gamma))


@pytest.mark.parametrize("dt_gamma,max_steps,density", [(1 / 128, 1024, 0.02), (1 / 128, 1024, 0.3),
                                                        (1 / 128, 1024, 1.0), (1 / 128, 7, 0.3),
                                                        (1 / 4096, 16384, 0.3), (1 / 64, 64, 1.0)])
def test_march_rays_train_gamma_random_bitfields(cuda, dt_gamma, max_steps, density):
    """dt_gamma > 0 over irregular two-cascade occupancy: re-walks that seek
    into other lanes' chain records, truncation at max_steps, and (1/4096 with
    max_steps 16384: dt_min 2.1e-4, ~10K indices to far) chains longer than
    the 4096 indices the records cover, which the serial walk marches."""
    rng = np.random.default_rng(int(density * 100) + max_steps)
    bits = np.packbits(rng.random(2 * 128 ** 3) < density, bitorder="little")
    _assert_march_equal(*_march_case(cuda, 300, C=2, bound=2.0, dt_gamma=dt_gamma, bits=bits,
                                     perturb_seed=7, max_steps=max_steps))


@pytest.mark.parametrize("density", [0.02, 0.3, 1.0])
def test_march_rays_train_random_bitfields(cuda, density):
    """Irregular occupancy exercises the segment stitching (re-walks) and, at
    density 1, rays that sample every chain index."""
    rng = np.random.default_rng(int(density * 100))
    bits = np.packbits(rng.random(128 ** 3) < density, bitorder="little")
    _assert_march_equal(*_march_case(cuda, 700, bits=bits, perturb_seed=5))


@pytest.mark.parametrize("max_steps", [1, 7, 64])
def test_march_rays_train_max_steps(cuda, max_steps):
    _assert_march_equal(*_march_case(cuda, 500, max_steps=max_steps, perturb_seed=2))


def test_march_rays_train_grid64(cuda):
    _assert_march_equal(*_march_case(cuda, 800, H=64, perturb_seed=3))


def test_march_rays_train_overflow_drops_tail_rays(cuda):
    ref, got = _march_case(cuda, 2048, M=128 * 40)
    xyzs, dirs, deltas, rays, counter = [a.cpu().numpy() for a in got]
    assert np.array_equal(rays, ref[3]) and np.array_equal(counter, ref[4])
    assert np.array_equal(xyzs.view(np.uint32), ref[0].view(np.uint32))
    assert np.array_equal(deltas.view(np.uint32), ref[2].view(np.uint32))


def test_march_rays_train_deterministic(cuda):
    _, a = _march_case(cuda, 4096)
    _, b = _march_case(cuda, 4096)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def _composite_inputs(N, seed):
    rng = np.random.default_rng(seed)
    counts = rng.integers(0, 80, N).astype(np.int32)
    counts[:3] = [0, 1, 200]
    offs = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int32)
    M = int(counts.sum())
    rays = np.stack([np.arange(N), offs, counts], -1).astype(np.int32)
    sig = np.log1p(np.exp(rng.standard_normal(M))).astype(np.float32) * 10
    rgb = rng.random((M, 3), dtype=np.float32)
    dl = np.stack([np.full(M, 2 * 1.7320508 / 1024), rng.random(M) * 0.01], -1).astype(np.float32)
    return sig, rgb, dl, rays


def test_composite_train_forward_backward(cuda):
    import raymarching.backend as rb
    N = 2000
    sig, rgb, dl, rays = _composite_inputs(N, 7)
    M = sig.shape[0]
    ws, dp, img = oracle.composite_rays_train_forward(sig, rgb, dl, rays)
    tws, tdp, timg = torch.empty(N, device=cuda), torch.empty(N, device=cuda), torch.empty(N, 3, device=cuda)
    rb._backend.composite_rays_train_forward(t(sig, cuda), t(rgb, cuda), t(dl, cuda), t(rays, cuda), M,
                                             N, 1e-4, tws, tdp, timg)
    np.testing.assert_allclose(tws.cpu().numpy(), ws, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(tdp.cpu().numpy(), dp, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(timg.cpu().numpy(), img, rtol=1e-5, atol=1e-6)
    rng = np.random.default_rng(8)
    gws, gd, gi = rng.standard_normal(N).astype(np.float32), rng.standard_normal(N).astype(np.float32), \
        rng.standard_normal((N, 3)).astype(np.float32)
    rgs, rgc = oracle.composite_rays_train_backward(gws, gd, gi, sig, rgb, dl, rays, ws, dp, img)
    gs, gc = torch.zeros(M, device=cuda), torch.zeros(M, 3, device=cuda)
    rb._backend.composite_rays_train_backward(t(gws, cuda), t(gd, cuda), t(gi, cuda), t(sig, cuda),
                                              t(rgb, cuda), t(dl, cuda), t(rays, cuda), tws, tdp, timg,
                                              M, N, 1e-4, gs, gc)
    np.testing.assert_allclose(gc.cpu().numpy(), rgc, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(gs.cpu().numpy(), rgs, rtol=1e-4, atol=1e-5)


def test_inference_march_and_composite(cuda):
    import raymarching.backend as rb
    N = 1500
    ro, rd = lego_rays(N, seed=11)
    aabb = np.array([-1, -1, -1, 1, 1, 1], np.float32)
    nears, fars = oracle.near_far_from_aabb(ro, rd, aabb, 0.2)
    bits = box_bitfield(lego_boxes())
    alive = np.arange(0, N, 2, dtype=np.int32)
    n_alive, n_step = alive.shape[0], 8
    rays_t = nears.copy()
    noises = np.random.default_rng(12).random(n_alive, dtype=np.float32)
    rx, rdirs, rdel = oracle.march_rays(n_alive, n_step, alive, rays_t, ro, rd, 1.0, bits, 1, 128,
                                        nears, fars, noises, align=128)
    Mi = rx.shape[0]
    xyzs, dirs, deltas = (torch.zeros(Mi, 3, device=cuda), torch.zeros(Mi, 3, device=cuda),
                          torch.zeros(Mi, 2, device=cuda))
    rb._backend.march_rays(n_alive, n_step, t(alive, cuda), t(rays_t, cuda), t(ro, cuda), t(rd, cuda),
                           1.0, 0.0, 1024, 1, 128, t(bits, cuda), t(nears, cuda), t(fars, cuda), xyzs,
                           dirs, deltas, t(noises, cuda))
    assert np.array_equal(xyzs.cpu().numpy().view(np.uint32), rx.view(np.uint32))
    assert np.array_equal(deltas.cpu().numpy().view(np.uint32), rdel.view(np.uint32))
    rng = np.random.default_rng(13)
    sig = (rng.random(Mi) * 50).astype(np.float32)
    rgb = rng.random((Mi, 3), dtype=np.float32)
    ws, dp, img = np.zeros(N, np.float32), np.zeros(N, np.float32), np.zeros((N, 3), np.float32)
    ra, rt = alive.copy(), rays_t.copy()
    tws, tdp, timg = t(ws, cuda), t(dp, cuda), t(img, cuda)
    tra, trt = t(ra, cuda), t(rt, cuda)
    oracle.composite_rays(n_alive, n_step, ra, rt, sig, rgb, rdel, ws, dp, img, 1e-2)
    rb._backend.composite_rays(n_alive, n_step, 1e-2, tra, trt, t(sig, cuda), t(rgb, cuda), deltas,
                               tws, tdp, timg)
    assert np.array_equal(tra.cpu().numpy(), ra)
    np.testing.assert_allclose(trt.cpu().numpy(), rt, rtol=1e-6)
    np.testing.assert_allclose(tws.cpu().numpy(), ws, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(timg.cpu().numpy(), img, rtol=1e-5, atol=1e-6)


def test_morton_packbits(cuda):
    import raymarching as rm
    rng = np.random.default_rng(14)
    coords = rng.integers(0, 128, (10000, 3)).astype(np.int32)
    idx = rm.morton3D(t(coords, cuda))
    assert np.array_equal(idx.cpu().numpy(), oracle.morton3D(coords))
    back = rm.morton3D_invert(idx)
    assert np.array_equal(back.cpu().numpy(), coords)
    grid = rng.standard_normal((2, 128 ** 3)).astype(np.float32)
    bits = rm.packbits(t(grid, cuda), 0.3)
    assert np.array_equal(bits.cpu().numpy(), oracle.packbits(grid, 0.3))


# ----------------------------------------------------------------------- SH

@pytest.mark.parametrize("degree", [1, 2, 3, 4, 5, 8])
def test_sh_forward_backward(cuda, degree):
    from shencoder import SHEncoder
    rng = np.random.default_rng(20 + degree)
    d = rng.standard_normal((5000, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    ref = oracle.sh_encode(d, degree)
    enc = SHEncoder(degree=degree)
    x = t(d, cuda).requires_grad_(True)
    y = enc(x)
    np.testing.assert_allclose(y.detach().cpu().numpy(), ref, rtol=0, atol=2e-6)
    g = rng.standard_normal(y.shape).astype(np.float32)
    y.backward(t(g, cuda))
    jac = oracle.sh_encode_jacobian(d, degree)
    ref_gi = np.einsum("bc,bdc->bd", g.astype(np.float64), jac)
    np.testing.assert_allclose(x.grad.cpu().numpy(), ref_gi, rtol=1e-3, atol=1e-3)


# ----------------------------------------------------------------------- MLP

@pytest.mark.parametrize("in_dim,hidden,nl,out,B", [(32, 64, 2, 16, 4096 + 16), (32, 64, 3, 3, 3000),
                                                    (16, 32, 2, 8, 257), (64, 64, 4, 16, 1024)])
def test_ffmlp_forward_backward(cuda, in_dim, hidden, nl, out, B):
    from ffmlp import FFMLP
    net = FFMLP(in_dim, out, hidden, nl).to(cuda)
    rng = np.random.default_rng(30)
    x = (rng.standard_normal((B, in_dim)) * 0.5).astype(np.float16)
    xt = t(x, cuda).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.float16):
        y = net(xt)
    w16 = net.weights.detach().half().cpu().numpy()
    ref, _ = oracle.mlp_forward(x, w16, in_dim, 16, hidden, nl)
    close16(y.detach().cpu().numpy(), ref[:, :out], "ffmlp forward")
    g = rng.standard_normal((B, out)).astype(np.float16)
    y.backward(t(g, cuda))
    gpad = np.zeros((B, 16), np.float16); gpad[:, :out] = g
    ref_gi, ref_gw = oracle.mlp_backward(gpad, x, w16, in_dim, 16, hidden, nl)
    close16(xt.grad.cpu().numpy(), ref_gi, "ffmlp grad_inputs")
    # dW: an fp32 sum over the batch (fp16 deltas), rounded to fp16 once
    close16(net.weights.grad.cpu().numpy(), ref_gw, "ffmlp grad_weights", min_equal=0.9)


def test_ffmlp_forward_buffer_and_inference(cuda):
    import ffmlp.backend as fb
    B, in_dim, hidden, nl = 1000, 32, 64, 2
    rng = np.random.default_rng(31)
    nparams = hidden * (in_dim + hidden * (nl - 1) + 16)
    w = (rng.uniform(-1, 1, nparams) * np.sqrt(3 / hidden)).astype(np.float16)
    x = rng.standard_normal((B, in_dim)).astype(np.float16)
    out = torch.empty(B, 16, dtype=torch.float16, device=cuda)
    fbuf = torch.empty(nl, B, hidden, dtype=torch.float16, device=cuda)
    fb._backend.ffmlp_forward(t(x, cuda), t(w, cuda), B, in_dim, 16, hidden, nl, 0, 6, fbuf, out)
    ref, hs = oracle.mlp_forward(x, w, in_dim, 16, hidden, nl)
    for l in range(nl):
        close16(fbuf[l].cpu().numpy(), hs[l], f"forward_buffer[{l}]")
    close16(out.cpu().numpy(), ref, "ffmlp_forward output")
    out2 = torch.empty_like(out)
    fb._backend.ffmlp_inference(t(x, cuda), t(w, cuda), B, in_dim, 16, hidden, nl, 0, 6, None, out2)
    assert torch.equal(out, out2)


def test_adam_matches_torch(cuda):
    import _ngp_native as nat
    n = 10007
    torch.manual_seed(0)
    p = torch.randn(n, device=cuda)
    p_ref = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([p_ref], lr=1e-2, betas=(0.9, 0.99), eps=1e-15)
    m = torch.zeros(n, device=cuda); v = torch.zeros(n, device=cuda)
    for step in range(1, 4):
        g = torch.randn(n, device=cuda)
        p_ref.grad = g.clone()
        opt.step()
        nat.check(nat.lib().ngp_adam_step(p.data_ptr(), g.data_ptr(), 0, m.data_ptr(), v.data_ptr(), n,
                                          1e-2, 0.9, 0.99, 1e-15, 0.0, step, 1.0,
                                          torch.cuda.current_stream().cuda_stream), "adam")
    torch.testing.assert_close(p, p_ref.detach(), rtol=1e-5, atol=1e-6)

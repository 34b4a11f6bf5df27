"""GPU: the density-grid update (update_extra_state, mark_untrained_grid).

`_torch_update` below is the reference's update_extra_state (nerf/renderer.py
:498-598) restated in torch over the model's autograd density() path -- the
torch glue this build ran before the update moved to csrc/density_grid.hip. Both
are run from the same torch RNG state, so they draw the same cells and noise;
the grid must agree to fp32 exp rounding and the bitfield bit for bit. A cell
drawn twice in one partial update keeps its larger density in both (upstream's
index_put keeps an arbitrary one).
"""
import copy

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


def _model(cuda, bound=1, density_thresh=10.0, seed=0):
    from nerf.network_ff import NeRFNetwork
    from nerf.provider import lego_bitfield
    torch.manual_seed(seed)
    m = NeRFNetwork(bound=bound, cuda_ray=True, density_thresh=density_thresh).to(cuda)
    with torch.no_grad():
        m.encoder.embeddings.normal_(0, 0.3)  # densities spread around exp(0) = 1
    m.density_bitfield.copy_(torch.from_numpy(lego_bitfield(cascade=m.cascade, bound=float(bound))).to(cuda))
    return m


@torch.no_grad()
def _torch_update(m, decay=0.95, S=128):
    """Reference update_extra_state in torch (renderer.py:498-598)."""
    import raymarching
    from nerf.renderer import custom_meshgrid
    tmp_grid = -torch.ones_like(m.density_grid)
    dev = m.density_bitfield.device
    H = m.grid_size

    def put(cas, indices, xyzs):
        sig = m.density(xyzs)["sigma"].reshape(-1).detach().float() * m.density_scale
        tmp_grid[cas].view(torch.int32).scatter_reduce_(0, indices, sig.view(torch.int32), "amax")

    if m.iter_density < 16:
        X = torch.arange(H, dtype=torch.int32, device=dev).split(S)
        for xs in X:
            for ys in X:
                for zs in X:
                    xx, yy, zz = custom_meshgrid(xs, ys, zs)
                    coords = torch.cat([xx.reshape(-1, 1), yy.reshape(-1, 1), zz.reshape(-1, 1)], dim=-1)
                    indices = raymarching.morton3D(coords).long()
                    xyzs = 2 * coords.float() / (H - 1) - 1
                    for cas in range(m.cascade):
                        bound = min(2 ** cas, m.bound)
                        hgs = bound / H
                        cas_xyzs = xyzs * (bound - hgs)
                        cas_xyzs += (torch.rand_like(cas_xyzs) * 2 - 1) * hgs
                        put(cas, indices, cas_xyzs)
    else:
        N = H ** 3 // 4
        for cas in range(m.cascade):
            coords = torch.randint(0, H, (N, 3), device=dev)
            indices = raymarching.morton3D(coords.int()).long()
            occ_indices = torch.nonzero(m.density_grid[cas] > 0).squeeze(-1)
            rand_mask = torch.randint(0, occ_indices.shape[0], [N], dtype=torch.long, device=dev)
            occ_indices = occ_indices[rand_mask]
            occ_coords = raymarching.morton3D_invert(occ_indices.int())
            indices = torch.cat([indices, occ_indices], dim=0)
            coords = torch.cat([coords.int(), occ_coords], dim=0)
            xyzs = 2 * coords.float() / (H - 1) - 1
            bound = min(2 ** cas, m.bound)
            hgs = bound / H
            cas_xyzs = xyzs * (bound - hgs)
            cas_xyzs += (torch.rand_like(cas_xyzs) * 2 - 1) * hgs
            put(cas, indices, cas_xyzs)
    valid = (m.density_grid >= 0) & (tmp_grid >= 0)
    m.density_grid[valid] = torch.maximum(m.density_grid[valid] * decay, tmp_grid[valid])
    m.mean_density = torch.mean(m.density_grid.clamp(min=0)).item()
    m.iter_density += 1
    thresh = min(m.mean_density, m.density_thresh)
    m.density_bitfield = raymarching.packbits(m.density_grid, thresh, m.density_bitfield)


def _pair(cuda, **kw):
    a = _model(cuda, **kw)
    b = copy.deepcopy(a)
    return a, b


def _run_both(a, b, seed):
    with torch.autocast("cuda", dtype=torch.float16):
        torch.manual_seed(seed)
        a.update_extra_state()
        torch.manual_seed(seed)
        _torch_update(b)
    torch.cuda.synchronize()


def _compare(a, b):
    ga, gb = a.density_grid.cpu().numpy(), b.density_grid.cpu().numpy()
    assert np.array_equal(ga < 0, gb < 0)
    np.testing.assert_allclose(ga, gb, rtol=1e-6, atol=0)
    assert abs(a.mean_density - b.mean_density) <= 1e-6 * abs(b.mean_density)
    assert torch.equal(a.density_bitfield, b.density_bitfield)


@pytest.mark.parametrize("bound,thresh", [(1, 10.0), (1, 0.01), (2, 10.0)])
def test_update_extra_state_matches_torch_restatement(cuda, bound, thresh):
    """Full updates (iter_density < 16) then partial ones (occupied + uniform
    cells), one and two cascades, threshold from density_thresh or from the
    grid's mean."""
    a, b = _pair(cuda, bound=bound, density_thresh=thresh)
    for it in range(3):
        _run_both(a, b, 100 + it)
        _compare(a, b)
    occ = (a.density_grid > 0).float().mean().item()
    assert 0.01 < occ <= 1.0
    a.iter_density = b.iter_density = 16  # partial updates from here on
    for it in range(3):
        _run_both(a, b, 200 + it)
        _compare(a, b)
    bits = np.unpackbits(a.density_bitfield.cpu().numpy())
    assert bits.sum() > 0
    if a.mean_density < thresh:  # thresholded at the mean: some cells stay empty
        assert bits.sum() < bits.size


def test_update_extra_state_mean_count(cuda):
    m = _model(cuda)
    m.step_counter[:, 0] = torch.arange(16, dtype=torch.int32, device=cuda) * 100
    m.local_step = 5
    with torch.autocast("cuda", dtype=torch.float16):
        m.update_extra_state()
    assert m.mean_count == int(sum(range(5)) * 100 / 5) and m.local_step == 0


def test_update_extra_state_marks_only_valid_cells(cuda):
    """Cells marked untrained (-1) stay -1 through updates and never light up."""
    m = _model(cuda)
    m.density_grid.view(-1)[::7] = -1
    with torch.autocast("cuda", dtype=torch.float16):
        for _ in range(2):
            m.update_extra_state()
    g = m.density_grid.view(-1)
    assert torch.all(g[::7] == -1) and torch.all(g[1::7] >= 0)
    bits = np.unpackbits(m.density_bitfield.cpu().numpy(), bitorder="little")
    assert not bits[::7].any()


def test_mark_untrained_grid_matches_numpy(cuda):
    """mark_untrained_grid (renderer.py:433-496) against a numpy restatement of
    the camera-frustum test, on a ring of synthetic Lego poses."""
    from nerf.provider import SyntheticLego
    m = _model(cuda, bound=2)
    data = SyntheticLego(cuda, num_rays=16)
    poses = data.poses[::10].contiguous()
    fx, fy, cx, cy = [float(v) for v in data.intrinsics]
    m.mark_untrained_grid(poses, (fx, fy, cx, cy), S=64)
    got = (m.density_grid == -1).cpu().numpy()
    H = m.grid_size
    xs = np.arange(H)
    coords = np.stack(np.meshgrid(xs, xs, xs, indexing="ij"), -1).reshape(-1, 3).astype(np.int32)
    idx = oracle.morton3D(coords)
    world = 2 * coords.astype(np.float64) / (H - 1) - 1
    P = poses.cpu().numpy().astype(np.float64)
    want = np.zeros((m.cascade, H ** 3), bool)
    for cas in range(m.cascade):
        bound = min(2 ** cas, m.bound)
        hgs = bound / H
        cw = world * (bound - hgs)
        seen = np.zeros(H ** 3, bool)
        for p in P:
            cam = (cw - p[:3, 3]) @ p[:3, :3]
            seen |= ((cam[:, 2] > 0) & (np.abs(cam[:, 0]) < cx / fx * cam[:, 2] + hgs * 2)
                     & (np.abs(cam[:, 1]) < cy / fy * cam[:, 2] + hgs * 2))
        want[cas, idx] = ~seen
    # fp32 (torch) vs fp64 (here) frustum tests may differ exactly on a frustum plane
    assert (got != want).mean() < 1e-4 and 0 < want.mean() < 1


# ---- FusedTrainer.update_density: device-side draws -------------------------------

def _mix32(x):
    x = np.asarray(x, np.uint32)
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint32(16)); x = x * np.uint32(0x7feb352d)
        x = x ^ (x >> np.uint32(15)); x = x * np.uint32(0x846ca68b)
        x = x ^ (x >> np.uint32(16))
    return x


def _rng_u32(seed, a, b, c):
    """csrc/density_grid.hip rng_u32 (counter RNG), restated in numpy uint32."""
    with np.errstate(over="ignore"):
        inner = _mix32(np.asarray(b, np.uint32) ^ _mix32(np.uint32(c) + np.uint32(0x85ebca6b)))
        return _mix32(np.uint32(seed) ^ _mix32(np.uint32(a) + np.uint32(0x9e3779b9) * inner))


DENSITY_RNG_DOMAIN = 0xd3a5b1c7  # csrc/density_grid.hip kDensityRngDomain


def _draws(seed, update, P, ppc, H, grid=None):
    seed = np.uint32(seed ^ DENSITY_RNG_DOMAIN)
    p = np.arange(P, dtype=np.uint32)
    noise = np.stack([(_rng_u32(seed, update, p, 1 + j) >> np.uint32(8)).astype(np.float32) * np.float32(2 ** -24)
                      for j in range(3)], -1)
    if grid is None:
        return None, noise
    coords = np.stack([_rng_u32(seed, update, p, 8 + j) % np.uint32(H) for j in range(3)], -1).astype(np.int32)
    cas, k = p // ppc, p % ppc
    for c in range(grid.shape[0]):
        occ = np.nonzero(grid[c] > 0)[0].astype(np.int32)
        sel = (cas == c) & (k >= ppc // 2)
        if occ.size:
            cells = occ[_rng_u32(seed, update, p[sel], 7) % np.uint32(occ.size)]
            coords[sel] = oracle.morton3D_invert(cells)
    return coords, noise


def _exp_fixed(r):
    """csrc/density_grid.hip exp_fixed: -ln(u) of u = ((r >> 8) + 1) / 2^24 in
    2^-32 fixed point, the same IEEE double operations in the same order."""
    v = (np.asarray(r, np.uint32) >> np.uint32(8)).astype(np.uint64) + np.uint64(1)
    e = np.array([int(x).bit_length() - 1 for x in v.ravel()], np.int64).reshape(v.shape)
    m = v.astype(np.float64) / np.exp2(e.astype(np.float64))
    s = (m - 1.0) / (m + 1.0)
    s2 = s * s
    q = np.full_like(s, 1.0 / 15.0)
    for c in (1.0 / 13.0, 1.0 / 11.0, 1.0 / 9.0, 1.0 / 7.0, 1.0 / 5.0, 1.0 / 3.0, 1.0):
        q = q * s2 + c
    lnm = 2.0 * s * q
    E = (24 - e).astype(np.float64) * 0.6931471805599453 - lnm
    return np.where(E > 0, (np.maximum(E, 0) * 4294967296.0).astype(np.uint64), np.uint64(0))


def _draws_ostat(seed, update, C, H, grid):
    """ngp_density_grid_draw_sorted's draws (cells per point, uniform half then
    occupied half per cascade) restated in numpy: uniform order statistics
    S_k / S_N from the prefix sums of N + 1 fixed-point exponentials."""
    seed = np.uint32(seed ^ DENSITY_RNG_DOMAIN)
    H3, N = H ** 3, H ** 3 // 4
    j = np.arange(N + 1, dtype=np.uint32)
    cells = []
    for cas in range(C):
        occ = np.nonzero(grid[cas] > 0)[0].astype(np.int64)
        for half in range(2):
            E = _exp_fixed(_rng_u32(seed, update, j, 16 + 2 * cas + half))
            S = np.cumsum(E, dtype=np.uint64)
            t = S[:N].astype(np.float64) / np.float64(S[N])
            if half and occ.size:
                cells.append(occ[np.minimum(np.floor(t * occ.size), occ.size - 1).astype(np.int64)])
            else:
                cells.append(np.minimum(np.floor(t * H3), H3 - 1).astype(np.int64))
    cells = np.concatenate(cells)
    _, noise = _draws(int(seed ^ np.uint32(DENSITY_RNG_DOMAIN)), update, C * 2 * N, 2 * N, H)
    return oracle.morton3D_invert(cells.astype(np.int32)).astype(np.int32), noise, cells


@torch.no_grad()
def _torch_update_from(m, coords, noise, ppc, decay=0.95):
    """The reference update (:524-590) from given cells and noise (torch ops on
    the model's autograd density path); duplicates keep the larger density."""
    import raymarching
    H = m.grid_size
    tmp_grid = -torch.ones_like(m.density_grid)
    for cas in range(m.cascade):
        c = coords[cas * ppc:(cas + 1) * ppc]
        indices = raymarching.morton3D(c).long()
        xyzs = 2 * c.float() / (H - 1) - 1
        bound = min(2 ** cas, m.bound)
        hgs = bound / H
        cas_xyzs = xyzs * (bound - hgs)
        cas_xyzs += (noise[cas * ppc:(cas + 1) * ppc] * 2 - 1) * hgs
        sig = m.density(cas_xyzs)["sigma"].reshape(-1).detach().float() * m.density_scale
        tmp_grid[cas].view(torch.int32).scatter_reduce_(0, indices, sig.view(torch.int32), "amax")
    valid = (m.density_grid >= 0) & (tmp_grid >= 0)
    m.density_grid[valid] = torch.maximum(m.density_grid[valid] * decay, tmp_grid[valid])
    m.mean_density = torch.mean(m.density_grid.clamp(min=0)).item()
    m.density_bitfield = raymarching.packbits(m.density_grid, min(m.mean_density, m.density_thresh),
                                              m.density_bitfield)


@pytest.mark.parametrize("bound,ordered", [(1, True), (2, True), (1, False)], ids=["b1", "b2", "b1_draw_order"])
def test_fused_update_density_matches_restatement(cuda, bound, ordered):
    """Full updates (every cell, Morton-ordered queries) and partial ones: the
    Morton-ordered order-statistics draws (density_sort, default) or the
    counter-RNG draws in draw order, restated in numpy, through the
    reference's update on the model's autograd density path."""
    from nerf.fused import FusedTrainer
    from nerf.provider import SyntheticLego
    a = _model(cuda, bound=bound)
    b = copy.deepcopy(a)
    ft = FusedTrainer(a, SyntheticLego(cuda, num_rays=256), M=20000, seed=5, options=dict(density_sort=ordered))
    H, C = a.grid_size, a.cascade
    allc = torch.stack(torch.meshgrid(*[torch.arange(H, dtype=torch.int32, device=cuda)] * 3, indexing="ij"),
                       -1).reshape(-1, 3).repeat(C, 1)
    for it in range(4):
        partial = it >= 2
        if partial:
            a.iter_density = b.iter_density = 16
        pre = b.density_grid.cpu().numpy()
        ft.update_density()
        ppc = H ** 3 // 2 if partial else H ** 3
        d = ft._dens
        if partial and ordered:
            coords, noise, cells = _draws_ostat(5, a.iter_density - 1, C, H, pre)
            idx = (np.repeat(np.arange(C), ppc) * H ** 3 + cells).astype(np.int32)
            np.testing.assert_array_equal(d["idx"][:C * ppc].cpu().numpy(), idx)  # the draws, bit for bit
        else:
            coords, noise = _draws(5, a.iter_density - 1, C * ppc, ppc, H, pre if partial else None)
            np.testing.assert_array_equal(d["noise"][:C * ppc].cpu().numpy(), noise)
            if partial:
                np.testing.assert_array_equal(d["coords"][:C * ppc].cpu().numpy(), coords)
        with torch.autocast("cuda", dtype=torch.float16):
            _torch_update_from(b, torch.from_numpy(coords).to(cuda) if partial else allc,
                               torch.from_numpy(noise).to(cuda), ppc)
        torch.cuda.synchronize()
        ga, gb = a.density_grid.cpu().numpy(), b.density_grid.cpu().numpy()
        np.testing.assert_allclose(ga, gb, rtol=1e-6, atol=0)
        assert abs(ft.mean_density - b.mean_density) <= 1e-6 * b.mean_density
        assert torch.equal(a.density_bitfield, b.density_bitfield)
    # the marcher's occupancy image follows the new bitfield: a step still marches
    ft.step()
    assert ft.sample_count() > 0


@pytest.mark.parametrize("C,H", [(1, 128), (2, 64), (3, 32)])
def test_sorted_points_are_a_permutation_in_brick_order(cuda, C, H):
    """ngp_density_grid_points_sorted over [lo, hi) = the same (xyz, index)
    rows as ngp_density_grid_points' rows lo..hi-1, permuted into brick order
    (bucket = cascade, morton >> shift non-decreasing); two slices together
    hold every draw (the data-parallel split)."""
    import _ngp_native as nat
    lib, P_ = nat.lib(), nat.ptr
    H3 = H ** 3
    ppc = H3 // 2
    P = C * ppc
    g = torch.Generator(device="cpu").manual_seed(C * 100 + H)
    coords = torch.randint(0, H, (P, 3), dtype=torch.int32, generator=g).to(cuda)
    noise = torch.rand(P, 3, generator=g).to(cuda)
    xa, ia = torch.zeros(P, 3, device=cuda), torch.zeros(P, dtype=torch.int32, device=cuda)
    s = nat.stream_of(xa)
    nat.check(lib.ngp_density_grid_points(P_(coords), P_(noise), P, ppc, C, H, 2.0, P_(xa), P_(ia), s), "points")
    ws = torch.zeros(int(lib.ngp_density_grid_sort_workspace_bytes(C, H)), dtype=torch.uint8, device=cuda)
    split = P // 3 + 17
    xs, is_ = torch.zeros(P, 3, device=cuda), torch.zeros(P, dtype=torch.int32, device=cuda)
    for lo, hi in ((0, split), (split, P)):
        nat.check(lib.ngp_density_grid_points_sorted(P_(coords), P_(noise), P, ppc, C, H, 2.0, lo, hi, P_(ws),
                                                     ws.numel(), P_(xs) + 12 * lo, P_(is_) + 4 * lo, s), "sorted")
    torch.cuda.synchronize()
    for lo, hi in ((0, split), (split, P)):
        ref = np.concatenate([xa[lo:hi].cpu().numpy().view(np.int32), ia[lo:hi, None].cpu().numpy()], 1)
        got = np.concatenate([xs[lo:hi].cpu().numpy().view(np.int32), is_[lo:hi, None].cpu().numpy()], 1)
        order = lambda r: r[np.lexsort(r.T[::-1])]  # noqa: E731  rows as a sorted multiset
        np.testing.assert_array_equal(order(ref), order(got))
        # brick order: the bucket (cascade * H^3 + morton) >> shift never decreases
        idx = is_[lo:hi].cpu().numpy().astype(np.int64)
        cas, mort = idx // H3, idx % H3
        bits = int(np.ceil(np.log2(H)))
        shift = min(9, 3 * bits)
        while shift < 3 * bits and C << (3 * bits - shift) > 8192:
            shift += 1
        bucket = cas * (1 << (3 * bits - shift)) + (mort >> shift)
        assert np.all(np.diff(bucket) >= 0)


@pytest.mark.parametrize("C,H", [(1, 32), (2, 16)])
def test_ordered_draws_slices_and_statistics(cuda, C, H):
    """ngp_density_grid_draw_sorted: two slices [0, s) + [s, P) (the
    data-parallel split) give the numpy restatement's points bit for bit
    (xyz and index); each half's cells are in Morton order; the occupied half
    draws only occupied cells; over many updates the uniform half's cells are
    uniform (chi-square over 64 Morton blocks)."""
    import _ngp_native as nat
    from scipy import stats
    lib, P_ = nat.lib(), nat.ptr
    H3, N = H ** 3, H ** 3 // 4
    P = C * 2 * N
    g = torch.Generator(device="cpu").manual_seed(C * 10 + H)
    grid = (torch.rand(C, H3, generator=g) - 0.7).to(cuda)  # ~30 % occupied
    dws = torch.zeros(int(lib.ngp_density_grid_draw_workspace_bytes(C, H)), dtype=torch.uint8, device=cuda)
    ows = torch.zeros(int(lib.ngp_density_grid_ostat_workspace_bytes(C, H)), dtype=torch.uint8, device=cuda)
    xyz, idx = torch.zeros(P, 3, device=cuda), torch.zeros(P, dtype=torch.int32, device=cuda)
    s = nat.stream_of(xyz)
    split = P // 3 + 5
    counts = np.zeros(64)
    for upd in range(8):
        for lo, hi in ((0, split), (split, P)):
            nat.check(lib.ngp_density_grid_draw_sorted(P_(grid), C, H, 9, upd, 1.0, lo, hi, P_(dws), dws.numel(),
                                                       P_(ows), ows.numel(), P_(xyz) + 12 * lo, P_(idx) + 4 * lo, s),
                      "draw_sorted")
        torch.cuda.synchronize()
        got = idx.cpu().numpy()
        coords, noise, cells = _draws_ostat(9, upd, C, H, grid.cpu().numpy())
        np.testing.assert_array_equal(got, (np.repeat(np.arange(C), 2 * N) * H3 + cells).astype(np.int32))
        if upd == 0:
            want, wi = torch.zeros(P, 3, device=cuda), torch.zeros(P, dtype=torch.int32, device=cuda)
            tc, tn = torch.from_numpy(coords).to(cuda), torch.from_numpy(noise).to(cuda)  # (held: the pointers outlive P_)
            nat.check(lib.ngp_density_grid_points(P_(tc), P_(tn), P, 2 * N, C, H, 1.0, P_(want), P_(wi), s), "points")
            torch.cuda.synchronize()
            assert torch.equal(xyz, want)  # k_density_points' arithmetic, bit for bit
        for cas in range(C):
            u, o = cells[cas * 2 * N:cas * 2 * N + N], cells[cas * 2 * N + N:(cas + 1) * 2 * N]
            assert np.all(np.diff(u) >= 0) and np.all(np.diff(o) >= 0)
            assert np.all(grid[cas].cpu().numpy()[o] > 0)
            counts += np.bincount(u * 64 // H3, minlength=64)
    assert stats.chisquare(counts).pvalue > 1e-3


def test_fused_mean_count_kernel_matches_the_ring(cuda):
    """ngp_density_mean_count (the update's mean_count bookkeeping in one
    launch) equals int(mean) of the last `total` batches' counts gathered from
    the step-counter ring with torch ops (FusedTrainer._recent_counts), with
    the next batch drawn ahead and not, for every total in 1..16."""
    from nerf.fused import FusedTrainer
    from nerf.provider import SyntheticLego
    a = _model(cuda, bound=1)
    ft = FusedTrainer(a, SyntheticLego(cuda, num_rays=256), M=20000, seed=3)
    ft._dens = dict(mean_count=torch.zeros(1, dtype=torch.int64, device=cuda))
    seen = set()
    for it in range(20):
        ft.step()
        torch.cuda.synchronize()
        for total in range(1, 17):
            want = int(ft._recent_counts(total).sum().item()) // total
            assert int(ft._recent_count_mean(total).item()) == want, (it, total, ft._ahead)
        seen.add(ft._ahead)
    ft.flush()
    ft._sample()  # a batch drawn by the head: not ahead
    torch.cuda.synchronize()
    for total in range(1, 17):
        assert int(ft._recent_count_mean(total).item()) == int(ft._recent_counts(total).sum().item()) // total
    seen.add(ft._ahead)
    assert seen == {True, False}

"""The density-grid pipeline against the reference's own update_extra_state
and mark_untrained_grid (nerf/renderer.py:433-598), executed on a stub by
tests/golden/make_golden.py (`density_fixture`) with an analytic density
sigma = 30 exp(-|x - c|^2 / (0.35 bound^2)), grid 16^3, bound 2 (two
cascades, threshold = the grid mean) and bound 1 (one cascade, threshold =
density_thresh 0.5): the mark, then two full and two partial updates. The
fixture records every torch draw the reference made (served by a recording
proxy: distinct cells, the same noise for a cell drawn twice, so upstream's
arbitrary-duplicate index_put and this build's scatter-max agree), the grid,
bitfield, mean_density, mean_count and local_step after each update.

CPU: the fixture is self-consistent with the oracle's packbits / morton
(the oracle restatements the reference's raymarching calls were bound to).
GPU: this build's reference-API `update_extra_state` and
`mark_untrained_grid` (nerf/renderer.py, csrc/density_grid.hip) replay the
same draws on the same analytic field: the -1 mask and the bitfield bit for
bit (but for cells within the grid tolerance of the threshold), the grid
within RTOL (the analytic field's exp of an argument up to ~10 evaluated in
fp32 on the device and on the host: a few ulps of the argument), mean_density
within RTOL, mean_count / local_step exact. The fused update's own stages (brick-sorted
query points, the EMA + packbits launch) are checked against the same
updates.
"""
import os

import numpy as np
import pytest
import torch

import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = [("b2", 2, 10.0), ("b1", 1, 0.5)]
RTOL = 2e-5


def _bits_match(got, want, grid, thresh):
    """Bitfields equal, except for cells whose density lies within RTOL of the
    threshold (the two fields may round to either side there)."""
    gb = np.unpackbits(got, bitorder="little")
    wb = np.unpackbits(want, bitorder="little")
    g = grid.reshape(-1)
    near = np.abs(g - thresh) <= RTOL * max(abs(thresh), 1e-30)
    return bool(np.all((gb == wb) | near))


def _fixture():
    return dict(np.load(os.path.join(GOLDEN, "density_reference.npz")))


def _draws(f, tag, u):
    """The update's draws in call order: int64 cells / picks, noise k / 2^16."""
    return [f[f"{tag}_u{u}_d{j}"].astype(np.int64) if kind == 0
            else f[f"{tag}_u{u}_d{j}"].astype(np.float32) * np.float32(2.0 ** -16)
            for j, kind in enumerate(f[f"{tag}_u{u}_kinds"])]


@pytest.mark.parametrize("tag,bound,thresh", CASES)
def test_fixture_consistent_with_oracle_packbits(tag, bound, thresh):
    """Each recorded bitfield is oracle.packbits(grid, min(mean_density,
    density_thresh)) of the recorded grid (renderer.py:588-589), and
    mean_density is the grid's clamped mean (:584); mean_count is the mean of
    the first min(16, local_step) step counts (:593-595)."""
    f = _fixture()
    for u in range(4):
        g = f[f"{tag}_u{u}_grid"]
        md = float(f[f"{tag}_u{u}_mean_density"])
        assert abs(md - float(np.clip(g, 0, None).astype(np.float64).mean())) <= 1e-6 * md
        bits = oracle.packbits(g, min(md, thresh))
        assert np.array_equal(bits, f[f"{tag}_u{u}_bitfield"])
    # the partial updates' occupied picks are cells of the previous grid's occupied list
    for u in (2, 3):
        prev = f[f"{tag}_u{u - 1}_grid"]
        C = prev.shape[0]
        for cas in range(C):
            picks = f[f"{tag}_u{u}_d{3 * cas + 1}"]
            occ = np.nonzero(prev[cas] > 0)[0]
            assert picks.max() < occ.size


class _Replay:
    """torch.rand / torch.randint served from the fixture's recorded draws, in
    order (the reference's rand_like / randint calls, renderer.py:533,551-567)."""

    def __init__(self, draws, dev):
        self.draws, self.dev, self.i = draws, dev, 0

    def _next(self, shape):
        v = self.draws[self.i]
        self.i += 1
        assert tuple(v.shape) == tuple(shape), (v.shape, shape)
        return torch.from_numpy(v).to(self.dev)

    def rand(self, *size, **kw):
        shape = size[0] if len(size) == 1 and isinstance(size[0], (tuple, list, torch.Size)) else size
        return self._next(tuple(shape)).float()

    def randint(self, low, high, size, **kw):
        return self._next(tuple(size)).long()


def _blob_model(cuda, bound, thresh):
    from nerf.renderer import NeRFRenderer

    class Blob(NeRFRenderer):
        def density(self, x):
            c = torch.tensor([0.15, -0.1, 0.05], device=x.device) * self.bound
            return {"sigma": 30.0 * torch.exp(-((x - c) ** 2).sum(-1) / (0.35 * self.bound * self.bound))}

    return Blob(bound=bound, cuda_ray=True, density_thresh=thresh, grid_size=16).to(cuda)


@pytest.mark.gpu
@pytest.mark.parametrize("tag,bound,thresh", CASES)
def test_reference_api_density_pipeline_matches_reference(cuda, monkeypatch, tag, bound, thresh):
    import nerf.renderer as rmod
    f = _fixture()
    m = _blob_model(cuda, bound, thresh)
    m.mark_untrained_grid(torch.from_numpy(f[f"{tag}_poses"]), tuple(float(v) for v in f[f"{tag}_intrinsics"]),
                          S=64)
    got = m.density_grid.cpu().numpy()
    assert np.array_equal(got == -1, f[f"{tag}_marked"] == -1)
    counts = np.arange(1, 17, dtype=np.int32) * 1000 + bound * 7
    for u in range(4):
        if u == 2:
            m.iter_density = 16
        m.step_counter[:, 0] = torch.from_numpy(counts + u).to(cuda)
        m.local_step = (5, 16, 30, 0)[u]
        rp = _Replay(_draws(f, tag, u), cuda)
        with monkeypatch.context() as mp:
            mp.setattr(rmod.torch, "rand", rp.rand)
            mp.setattr(rmod.torch, "randint", rp.randint)
            m.update_extra_state()
        assert rp.i == len(rp.draws)  # every recorded draw consumed, in order
        torch.cuda.synchronize()
        g, ref = m.density_grid.cpu().numpy(), f[f"{tag}_u{u}_grid"]
        assert np.array_equal(g < 0, ref < 0)
        np.testing.assert_allclose(g, ref, rtol=RTOL, atol=1e-30)
        md = float(f[f"{tag}_u{u}_mean_density"])
        assert abs(m.mean_density - md) <= RTOL * md
        assert _bits_match(m.density_bitfield.cpu().numpy(), f[f"{tag}_u{u}_bitfield"], ref, min(md, thresh)), u
        assert m.mean_count == int(f[f"{tag}_u{u}_mean_count"]) and m.local_step == 0


@pytest.mark.gpu
@pytest.mark.parametrize("tag,bound,thresh", CASES)
def test_fused_density_stages_match_reference(cuda, tag, bound, thresh):
    """The fused update's launches on the reference's draws: the query points
    in brick order (ngp_density_grid_points_sorted, partial updates) or draw
    order (full), the analytic density scatter-maxed into the scratch grid,
    then ngp_density_grid_ema_pack: grid, mean and bitfield as upstream's."""
    import _ngp_native as nat
    lib, P_ = nat.lib(), nat.ptr
    f = _fixture()
    H = int(f["H"])
    C = 1 + int(np.ceil(np.log2(bound)))
    H3 = H ** 3
    grid = torch.from_numpy(f[f"{tag}_marked"]).to(cuda).contiguous()
    bits = torch.zeros(C * H3 // 8, dtype=torch.uint8, device=cuda)
    tmp = torch.full((C, H3), -1.0, device=cuda)
    stats = torch.zeros(nat.DENSITY_STATS_LEN, dtype=torch.float64, device=cuda)
    s = nat.stream_of(grid)
    cen = torch.tensor([0.15, -0.1, 0.05], device=cuda) * bound
    for u in range(4):
        d = _draws(f, tag, u)
        partial = u >= 2
        if partial:  # per cascade: cells, picks into the occupied list, noise
            ppc = 2 * (H3 // 4)
            prev = grid.cpu().numpy()
            cs, ns = [], []
            for cas in range(C):
                cells, picks, noise = d[3 * cas:3 * cas + 3]
                occ = np.nonzero(prev[cas] > 0)[0].astype(np.int32)
                cs.append(np.concatenate([cells.astype(np.int32), oracle.morton3D_invert(occ[picks])]))
                ns.append(noise)
            coords = torch.from_numpy(np.concatenate(cs)).to(cuda).contiguous()
        else:
            ppc = H3
            ns = d
            coords = None
        noise = torch.from_numpy(np.concatenate(ns)).to(cuda).contiguous()
        P = C * ppc
        xyzs = torch.zeros(P, 3, device=cuda)
        idx = torch.zeros(P, dtype=torch.int32, device=cuda)
        if partial:
            ws = torch.zeros(int(lib.ngp_density_grid_sort_workspace_bytes(C, H)), dtype=torch.uint8, device=cuda)
            nat.check(lib.ngp_density_grid_points_sorted(P_(coords), P_(noise), P, ppc, C, H, float(bound), 0, P,
                                                         P_(ws), ws.numel(), P_(xyzs), P_(idx), s), "sorted")
        else:
            nat.check(lib.ngp_density_grid_points(None, P_(noise), P, ppc, C, H, float(bound), P_(xyzs), P_(idx), s),
                      "points")
        sig = 30.0 * torch.exp(-((xyzs - cen) ** 2).sum(-1) / (0.35 * bound * bound))
        tmp.view(-1).view(torch.int32).scatter_reduce_(0, idx.long(), sig.view(torch.int32), "amax")
        nat.check(lib.ngp_density_grid_ema_pack(P_(grid), P_(tmp), C, H, 0.95, float(thresh), P_(stats), P_(bits), s),
                  "ema_pack")
        torch.cuda.synchronize()
        ref = f[f"{tag}_u{u}_grid"]
        np.testing.assert_allclose(grid.cpu().numpy(), ref, rtol=RTOL, atol=1e-30)
        md = float(np.float32(stats[0].item() / grid.numel()))
        assert abs(md - float(f[f"{tag}_u{u}_mean_density"])) <= RTOL * md
        assert _bits_match(bits.cpu().numpy(), f[f"{tag}_u{u}_bitfield"], ref, min(md, thresh)), u
        assert float(tmp.max()) == -1.0  # the EMA launch resets the scratch grid

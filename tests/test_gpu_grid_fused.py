"""GPU: the fused train step's grid-encoder entry points against the oracle.

ngp_grid_encode_forward_fused reads world-space xyz and the fp32 table as half
(the reference's `(x + bound) / (2 * bound)` and `embeddings.half()` under
autocast, gridencoder/grid.py + nerf/renderer.py), or directly an fp16 copy:
bit-exact vs the oracle forward on the normalised inputs and the half table.

ngp_grid_encode_backward_fused adds into an fp16 grad table through the
binned path (per-bin LDS accumulation, segmented bins, in-wave merging of
equal corners) plus atomics for levels with more than 256 bins: compared to
the oracle's float64 scatter per level, relative norm error <= 2e-3 and
max abs error <= 4e-3 x max|ref| (fp16 table, one rounding per run / segment).
"""
import ctypes

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

LEGO_SCALE = float(np.exp2(np.log2(2048 / 16) / 15))


def _lib():
    import _ngp_native as nat
    return nat


def _world(B, bound, seed, concentrated=0.0, ordered=False):
    rng = np.random.default_rng(seed)
    if concentrated:  # everything inside a small cube: a few heavy bins
        x = (0.3 + concentrated * rng.random((B, 3))).astype(np.float32)
    else:
        x = rng.random((B, 3), dtype=np.float32)
    if ordered:  # rays: runs of samples along a line, as the marcher emits them
        n = B // 64
        o = rng.random((n, 1, 3)).astype(np.float32) * 0.6 + 0.2
        d = rng.standard_normal((n, 1, 3)).astype(np.float32)
        d /= np.linalg.norm(d, axis=-1, keepdims=True)
        t = (np.arange(64, dtype=np.float32) * 0.0017)[None, :, None]
        x = np.clip(o + t * d, 0.0, 1.0).reshape(-1, 3)[:B]
        if x.shape[0] < B:
            x = np.concatenate([x, rng.random((B - x.shape[0], 3), dtype=np.float32)])
    w = (x * np.float32(2 * bound) - np.float32(bound)).astype(np.float32)
    w[:2] = [[bound * 1.01, 0.0, 0.0], [0.0, -bound * 1.2, 0.0]]  # outside the box: skipped
    return w


def _normalise(w, bound):
    return ((w + np.float32(bound)) * np.float32(1.0 / (2.0 * bound))).astype(np.float32)


def _bwd(nat, dev, g16, w, offs, L, H, scale, bound, count=None, table=None, reps=1, layout=1, flag=None,
         zeroed=False, external=False):
    B = w.shape[0]
    S = float(np.float32(np.log2(scale)))
    offs_host = np.ascontiguousarray(offs, dtype=np.int32)
    hp = offs_host.ctypes.data_as(ctypes.c_void_p)
    ws_bytes = nat.lib().ngp_grid_encode_backward_fused_workspace_bytes(B, 3, 2, L, S, H, 0, hp)
    ws = torch.zeros(max(int(ws_bytes), 256), dtype=torch.uint8, device=dev)
    if table is None:
        table = torch.zeros(int(offs[-1]), 2, dtype=torch.float16, device=dev)
    gt, wt, ot = (torch.from_numpy(a).to(dev) for a in (g16, w, offs_host))
    if layout == 0:  # [L, B, C]
        gt = gt.view(B, L, 2).permute(1, 0, 2).contiguous()
    cnt = torch.tensor([count], dtype=torch.int32, device=dev) if count is not None else None
    # NGP_GRID_CURSORS_EXTERNAL (0x20): the caller clears the bin cursors, as
    # the fused step does; with a zeroed grad the hashed levels' bins then go
    # one per wave (gridencoder.hip wave_bin) instead of the workgroup image
    cbytes = int(nat.lib().ngp_grid_encode_backward_fused_counter_bytes(B, 3, 2, L, S, H, 0, hp))
    for _ in range(reps):
        nat.check(nat.lib().ngp_grid_encode_backward_fused(
            nat.ptr(gt), nat.ptr(wt), float(bound), nat.ptr(ot), nat.ptr(table), B,
            nat.ptr(cnt) if cnt is not None else None, 3, 2, L, S, H, 0, 0, 0, hp,
            nat.ptr(ws), ws.numel(), layout | (0x10 if zeroed else 0) | (0x20 if external else 0),
            nat.ptr(flag) if flag is not None else None, nat.stream_of(table)), "grid_backward_fused")
        if external:
            ws[:cbytes].zero_()
    torch.cuda.synchronize()
    # the workspace's counters are left zeroed for the next call
    assert int(ws[:256].sum()) == 0
    return table.float().cpu().numpy()


def _check_levels(got, ref, offs, what, rtol=2e-3, mtol=4e-3):
    for l in range(len(offs) - 1):
        a, r = got[offs[l]:offs[l + 1]], ref[offs[l]:offs[l + 1]]
        rn = np.linalg.norm(r)
        if rn == 0:
            assert np.abs(a).max() == 0, (what, l)
            continue
        rel = np.linalg.norm(a - r) / rn
        mx = np.abs(a - r).max() / np.abs(r).max()
        assert rel <= rtol and mx <= mtol, (what, l, rel, mx)


CASES = [
    # B, L, H, scale, log2T, layout
    (20000, 16, 16, LEGO_SCALE, 19, "uniform"),
    (60000, 16, 16, LEGO_SCALE, 19, "rays"),
    (120000, 8, 16, 1.5, 19, "concentrated"),   # heavy bins: several segments per bin
    (30000, 8, 16, 2.0, 22, "uniform"),          # 2^22-entry levels: 1024 bins of 2^12 (the large bin kernel, sparse flushes)
    (30000, 6, 16, 2.0, 23, "uniform"),          # 2^23-entry levels: 2048 bins, past kMaxBinsPerLevelBig: the atomic suffix
    (513, 4, 8, 2.0, 12, "uniform"),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"B{c[0]}L{c[1]}T{c[4]}{c[5]}")
def test_grid_backward_fused_vs_oracle(cuda, case):
    nat = _lib()
    B, L, H, scale, log2T, layout = case
    bound = 1.0 if layout != "rays" else 2.0
    offs = oracle.grid_offsets(3, L, 2, H, scale, log2T)
    w = _world(B, bound, seed=B + L, concentrated=0.25 * (layout == "concentrated"), ordered=layout == "rays")
    rng = np.random.default_rng(7)
    g16 = (rng.standard_normal((B, L * 2)) * 0.5).astype(np.float16)
    flag = torch.zeros(1, dtype=torch.int32, device=cuda)
    got = _bwd(nat, cuda, g16, w, offs, L, H, scale, bound, flag=flag, zeroed=True)  # fresh table
    assert int(flag.item()) == 0  # finite grads: GradScaler's check stays clear
    x = _normalise(w, bound)
    ref = oracle.grid_encode_backward(g16, x, offs, 2, scale, H)
    _check_levels(got, ref, offs, layout)


# wave bins take the hashed levels up to ~512 items per bin (rows <= 512 x
# bins per level / 8: 8192 rows on 2^19-entry levels); more rows run the
# image path over every bin (the dense regime), so both regimes are compared
WAVE_CASES = [(4000, 16, 16, LEGO_SCALE, 19, "uniform"), (8000, 16, 16, LEGO_SCALE, 19, "rays"),
              (6000, 12, 16, 1.5, 19, "spill"), (40000, 12, 16, 1.5, 19, "spill")]


@pytest.mark.parametrize("case", [c for c in CASES if c[4] <= 22] + WAVE_CASES,
                         ids=lambda c: f"B{c[0]}L{c[1]}T{c[4]}{c[5]}")
def test_grid_backward_wave_bins_equal_image_path(cuda, parity_report, case):
    """The hashed levels' bins summed one per wave (cursors cleared by the
    caller, grad zeroed: the fused step's configuration) against the same
    bins through the workgroup image (the cursors left to the kernel):
    bit-identical table grads, including bins that spilled past their
    capacity (the 0.03-wide cube) and 2^22-entry levels; and two wave-path
    calls give the same bits. (2^23-entry levels are past the binned prefix:
    their fp16 atomics add in arrival order, so that case is not compared.)"""
    nat = _lib()
    B, L, H, scale, log2T, layout = case
    bound = 1.0 if layout != "rays" else 2.0
    offs = oracle.grid_offsets(3, L, 2, H, scale, log2T)
    conc = {"concentrated": 0.25, "spill": 0.03 if B > 10000 else 0.01}.get(layout, 0.0)
    w = _world(B, bound, seed=B + L, concentrated=conc, ordered=layout == "rays")
    g16 = (np.random.default_rng(5).standard_normal((B, L * 2)) * 0.5).astype(np.float16)
    img = _bwd(nat, cuda, g16, w, offs, L, H, scale, bound, zeroed=True)
    wave = _bwd(nat, cuda, g16, w, offs, L, H, scale, bound, zeroed=True, external=True)
    again = _bwd(nat, cuda, g16, w, offs, L, H, scale, bound, zeroed=True, external=True)
    ne = img.view(np.uint32) != wave.view(np.uint32)
    assert not ne.any(), (int(ne.sum()), np.argwhere(ne.any(1))[:4].ravel().tolist())
    assert np.array_equal(wave.view(np.uint32), again.view(np.uint32))
    parity_report(f"grid backward wave bins {layout} B{B} L{L} T2^{log2T}: {int((wave != 0).any(1).sum())} "
                  f"entries, bit-identical to the workgroup image path")


def test_grid_backward_fused_bin_overflow(cuda):
    """Points in a 0.03-wide cube: on the hashed levels a few entries take all
    corners and bins overflow their capacity. The excess goes into the spill
    image as the same exact int64 counts as the binned items, so every entry
    is ONE fp16 rounding of the exact sum of the rounded run contributions:
    per entry within 2^-11 of the sum of |terms| (each run's half rounding)
    plus half an fp16 ulp of the result, and two launches on the same input
    give identical bits (no arrival-order dependence; the reference's atomics,
    gridencoder.cu:320-328, are order-dependent)."""
    nat = _lib()
    B, L, H, scale = 40000, 12, 16, 1.5
    offs = oracle.grid_offsets(3, L, 2, H, scale, 19)
    w = _world(B, 1.0, seed=4, concentrated=0.03)
    g16 = (np.random.default_rng(9).standard_normal((B, L * 2)) * 0.5).astype(np.float16)
    got = _bwd(nat, cuda, g16, w, offs, L, H, scale, 1.0, zeroed=True)
    again = _bwd(nat, cuda, g16, w, offs, L, H, scale, 1.0, zeroed=True)
    assert np.array_equal(got.view(np.uint32), again.view(np.uint32))  # deterministic bits
    x = _normalise(w, 1.0)
    ref = oracle.grid_encode_backward(g16, x, offs, 2, scale, H)
    _check_levels(got, ref, offs, "overflow")
    mag = oracle.grid_encode_backward(np.abs(g16.astype(np.float64)), x, offs, 2, scale, H)
    err = np.abs(got - ref)
    assert (err <= 2.0 ** -11 * (mag + np.abs(ref)) + 2.0 ** -24).all(), \
        float((err / np.maximum(mag, 1e-30)).max())


@pytest.mark.parametrize("layout", [1, 0])
def test_grid_backward_fused_count_clip_and_accumulate(cuda, layout):
    nat = _lib()
    B, L, H, scale = 40000, 16, 16, LEGO_SCALE
    offs = oracle.grid_offsets(3, L, 2, H, scale, 19)
    w = _world(B, 1.0, seed=11, ordered=True)
    g16 = (np.random.default_rng(3).standard_normal((B, L * 2)) * 0.5).astype(np.float16)
    n = 31000
    got = _bwd(nat, cuda, g16, w, offs, L, H, scale, 1.0, count=n, reps=2, layout=layout)  # two calls add up
    ref = 2.0 * oracle.grid_encode_backward(g16[:n], _normalise(w[:n], 1.0), offs, 2, scale, H)
    _check_levels(got, ref, offs, "clip+accumulate")


@pytest.mark.parametrize("table,layout", [("f32", 1), ("f16", 1), ("f16", 0)])
def test_grid_forward_fused_bit_exact(cuda, table, layout):
    nat = _lib()
    B, L, H, scale, bound = 9000, 16, 16, LEGO_SCALE, 2.0
    offs = oracle.grid_offsets(3, L, 2, H, scale, 19)
    rng = np.random.default_rng(5)
    emb = (rng.standard_normal((int(offs[-1]), 2)) * 0.1).astype(np.float32)
    w = _world(B, bound, seed=5)
    w[2] = [bound, bound, bound]  # on the far faces: inside
    n = 8500
    S = float(np.float32(np.log2(scale)))
    out = torch.full((B, L * 2), 7.0, dtype=torch.float16, device=cuda)
    wt, et, ot = (torch.from_numpy(a).to(cuda) for a in (w, emb, offs))
    if table == "f16":
        et = et.half()  # the fp16 copy the fused optimizer keeps
    cnt = torch.tensor([n], dtype=torch.int32, device=cuda)
    nat.check(nat.lib().ngp_grid_encode_forward_fused(nat.ptr(wt), bound, nat.ptr(et), nat.DTYPE_CODE[et.dtype],
                                                      nat.ptr(ot), nat.ptr(out), B, nat.ptr(cnt), 3, 2, L, S, H,
                                                      0, 0, 0, layout, nat.stream_of(out)), "grid_forward_fused")
    torch.cuda.synchronize()
    ref, _ = oracle.grid_encode_forward(_normalise(w[:n], bound), emb.astype(np.float16), offs, scale, H)
    got = out.cpu().numpy()
    if layout == 0:  # [L, B, 2] in the same buffer
        got = out.view(-1).view(L, B, 2).permute(1, 0, 2).reshape(B, L * 2).cpu().numpy()
    assert np.array_equal(got[:n].view(np.uint16), ref.view(np.uint16))  # outside rows: zeros in both
    assert np.all(got[n:] == 7.0)  # rows past the sample count untouched


@pytest.mark.parametrize("count", [None, 250001])
def test_grid_forward_large_batch_lends_chunks_bit_exact(cuda, count):
    """A density-query-sized batch (>= 2^18 points): the XCDs holding two hashed
    levels lend a share of their point chunks to the XCDs with a dense level
    (gridencoder.hip kFwdBorrowPct); every (point, level) is still encoded
    once, bit-exact vs the oracle, for the full batch and for a sample count
    that ends mid-chunk (the lent chunks are the last live ones)."""
    nat = _lib()
    B, L, H, scale, bound = 300000, 16, 16, LEGO_SCALE, 1.0
    offs = oracle.grid_offsets(3, L, 2, H, scale, 19)
    rng = np.random.default_rng(8)
    emb = (rng.standard_normal((int(offs[-1]), 2)) * 0.1).astype(np.float32)
    w = _world(B, bound, seed=8)
    n = B if count is None else count
    S = float(np.float32(np.log2(scale)))
    out = torch.full((B, L * 2), 7.0, dtype=torch.float16, device=cuda)
    wt, et, ot = (torch.from_numpy(a).to(cuda) for a in (w, emb, offs))
    et = et.half()
    cnt = torch.tensor([n], dtype=torch.int32, device=cuda) if count is not None else None
    nat.check(nat.lib().ngp_grid_encode_forward_fused(nat.ptr(wt), bound, nat.ptr(et), nat.DTYPE_CODE[et.dtype],
                                                      nat.ptr(ot), nat.ptr(out), B,
                                                      nat.ptr(cnt) if cnt is not None else None, 3, 2, L, S, H,
                                                      0, 0, 0, 1, nat.stream_of(out)), "grid_forward_fused")
    torch.cuda.synchronize()
    ref, _ = oracle.grid_encode_forward(_normalise(w[:n], bound), emb.astype(np.float16), offs, scale, H)
    got = out.cpu().numpy()
    assert np.array_equal(got[:n].view(np.uint16), ref.view(np.uint16))
    assert np.all(got[n:] == 7.0)


@pytest.mark.parametrize("log2T,zeroed,external", [(19, False, False), (19, True, False), (22, True, False),
                                                    (23, False, False), (19, True, True), (22, True, True)])
def test_grid_backward_fused_flags_nonfinite(cuda, log2T, zeroed, external):
    """The nonfinite flag is GradScaler's inf check made by the kernels that
    write the grads: an inf output grad, or finite terms whose fp16 sum
    overflows, must set it, on the binned levels (read-modify-write, fresh
    per-entry and per-item flushes) and (T = 2^23: levels past the binned
    prefix) the scanned ones; external: the hashed levels' wave bins."""
    nat = _lib()
    B, L, H, scale = 20000, 16, 16, LEGO_SCALE
    offs = oracle.grid_offsets(3, L, 2, H, scale, log2T)
    w = _world(B, 1.0, seed=5)
    g16 = (np.random.default_rng(2).standard_normal((B, L * 2)) * 0.5).astype(np.float16)
    for lvl in (0, L - 1):
        g = g16.copy()
        g[B // 2, 2 * lvl] = np.float16(np.inf)
        flag = torch.zeros(1, dtype=torch.int32, device=cuda)
        _bwd(nat, cuda, g, w, offs, L, H, scale, 1.0, flag=flag, zeroed=zeroed, external=external)
        assert int(flag.item()) == 1, ("inf grad", lvl)
    big = np.full((B, L * 2), 60000.0, np.float16)  # finite terms, their fp16 sums overflow
    flag = torch.zeros(1, dtype=torch.int32, device=cuda)
    _bwd(nat, cuda, big, w, offs, L, H, scale, 1.0, flag=flag, zeroed=zeroed, external=external)
    assert int(flag.item()) == 1, "sum overflow"

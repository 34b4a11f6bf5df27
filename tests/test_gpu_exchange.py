"""GPU: the touched-entry gradient exchange of the replicated data-parallel
step (csrc/exchange.hip, nerf/exchange.py; DESIGN.md §7 option B).

The reference averages gradients with DDP's all-reduce (nerf/utils.py:325-327)
and every rank runs the full Adam. Here every rank lists its nonzero fp16
channel pairs, the lists are all-gathered and every rank sums all of them in
int64 fixed point, so the averaged gradient is the exact mean of the ranks'
fp16 values rounded once to fp16, identical on every rank:

  * the two kernels against numpy's exact mean (float64 sum of fp16 values
    is exact; numpy's float64 -> float16 rounds once), with overlapping,
    cancelling, subnormal and large entries, ragged bins, a non-finite
    value, and a list over its capacity (every rank skips);
  * two ranks on the one visible GPU (gloo stages the lists through the host):
    the exchanged gradient is bit-identical to the exact mean of the two
    batches' gradients computed by single-process trainers, the parameters
    after the update equal the single-process Adam on that mean, the ranks
    stay bit-identical through eager and captured steps, and an overflow on
    one rank makes both skip the step and back the scale off.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _lib():
    import _ngp_native as nat
    return nat


def _sparse_grads(rng, n, world):
    gs = []
    for r in range(world):
        g = np.zeros(n, np.float16)
        idx = rng.choice(n, n // 6, replace=False)
        mag = 10.0 ** rng.integers(-8, 5, idx.size)  # subnormals (< 6.1e-5) up to 1e4
        g[idx] = (rng.standard_normal(idx.size) * mag).astype(np.float16)
        gs.append(g)
    # entries every rank touches, and pairs that cancel exactly
    common = rng.choice(n, 64, replace=False)
    for g in gs:
        g[common] = rng.standard_normal(common.size).astype(np.float16)
    if world > 1:
        gs[1][common[:16]] = -gs[0][common[:16]]
    if world > 2:
        gs[2][common[:16]] = 0
    gs[0][5] = np.float16(65504.0)  # the largest fp16 on every rank: the sum exceeds fp16, the mean does not
    for g in gs[1:]:
        g[5] = np.float16(65504.0)
    return gs


_BIN = 4096  # pairs per bin (kBinPairs)


def _list(nat, g, dev, cap=None, inf=None):
    """ngp_grad_exchange_list of one rank's gradient; returns (send, decoded)."""
    t = torch.from_numpy(g.copy()).to(dev)
    cap = g.size // 2 if cap is None else cap
    words = int(nat.lib().ngp_grad_exchange_words(g.size, cap))
    send = torch.full((words,), -1, dtype=torch.int64, device=dev)  # garbage the kernel must overwrite
    send[0] = 0  # but a zero header (a new buffer, or the last reduce's clear)
    nat.check(nat.lib().ngp_grad_exchange_list(nat.ptr(t), g.size, None if inf is None else nat.ptr(inf),
                                               nat.ptr(send), cap, nat.stream_of(t)), "list")
    torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy().view(np.uint16), g.view(np.uint16))  # the gradient is not changed
    return send


def _decode(send, n, cap):
    u = send.cpu().numpy().view(np.uint64)
    hdr = u[:2].copy().view(np.int32)
    nb = (n // 2 + _BIN - 1) // _BIN
    tab = u[2:2 + nb]
    return hdr, tab & np.uint64(0xffffffff), tab >> np.uint64(32), u[2 + nb:2 + nb + cap]


def _reduce(nat, sends, n, dev, cap, inf=None):
    world = len(sends)
    recv = torch.cat(sends)
    grad = torch.full((n,), 7.0, dtype=torch.float16, device=dev)  # every value is rewritten
    flag = torch.zeros(1, dtype=torch.int32, device=dev) if inf is None else inf
    stats = torch.zeros(2, dtype=torch.int32, device=dev)
    nat.check(nat.lib().ngp_grad_exchange_reduce(nat.ptr(recv), world, cap, nat.ptr(grad), n, nat.ptr(flag),
                                                 nat.ptr(stats), None, nat.stream_of(grad)), "reduce")
    torch.cuda.synchronize()
    return grad.cpu().numpy(), int(flag[0]), stats.cpu().tolist()


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_exchange_kernels_exact_mean(parity_report, world):
    nat = _lib()
    dev = torch.device("cuda:0")
    n = 8 * 6007  # 24,028 pairs: 6 bins, the last one ragged
    rng = np.random.default_rng(world)
    gs = _sparse_grads(rng, n, world)
    sends = []
    for g in gs:
        send = _list(nat, g, dev)
        hdr, start, cnt, items = _decode(send, n, n // 2)
        words = g.view(np.uint32)
        want = np.nonzero(words & 0x7fff7fff)[0]
        assert hdr[0] == want.size and hdr[1] == 0 and cnt.sum() == want.size
        for b in range(start.size):  # each bin's segment: exactly its nonzero pairs, once each
            seg = items[int(start[b]):int(start[b]) + int(cnt[b])]
            idx = (seg & np.uint64(0xffffffff)).astype(np.int64)
            wb = want[(want >= b * _BIN) & (want < (b + 1) * _BIN)]
            assert np.array_equal(np.sort(idx), wb)
            assert np.array_equal((seg >> np.uint64(32)).astype(np.uint32), words[idx])
        sends.append(send)
    out, inf, stats = _reduce(nat, sends, n, dev, n // 2)
    want = (np.sum([g.astype(np.float64) for g in gs], axis=0) / world).astype(np.float16)
    ne = out.view(np.uint16) != want.view(np.uint16)
    assert not ne.any(), (int(ne.sum()), np.argwhere(ne)[:4].ravel().tolist())
    peak = max(int(np.count_nonzero(g.view(np.uint32) & 0x7fff7fff)) for g in gs)
    assert inf == 0 and stats == [0, peak]
    parity_report(f"grad exchange kernels, world {world}: longest list {peak} items, mean bit-identical to "
                  f"numpy's exact fp64 mean rounded once to fp16")


def _tie_grads(rng, n, world):
    """Per-rank fp16 gradients whose exact mean is an fp16 rounding tie at
    every value (a mean formed with the inexact reciprocal of
    2^24 * world rounds twice and may leave a tie on the wrong side). Value j:
    tie m = x + ulp(x)/2 for a random normal x; ranks 1.. take random fp16
    values, rank 0 the remainder world * m - rest when that is an fp16 value
    (rejection sampling over candidates)."""
    out = np.zeros((world, n), dtype=np.float16)
    filled = np.zeros(n, dtype=bool)
    while not filled.all():
        k = int((~filled).sum())
        x = (rng.uniform(0.25, 64.0, 8 * k) * rng.choice([-1.0, 1.0], 8 * k)).astype(np.float16)
        xd = x.astype(np.float64)
        ulp = np.abs(np.nextafter(x, np.float16(np.inf) * np.sign(x)).astype(np.float64) - xd)
        m = xd + np.sign(xd) * ulp / 2
        rest = (rng.uniform(-4.0, 4.0, (world - 1, 8 * k)) * (rng.random((world - 1, 8 * k)) < 0.7)).astype(np.float16)
        r0 = world * m - rest.astype(np.float64).sum(0)
        ok = (np.abs(r0) < 60000) & (r0.astype(np.float16).astype(np.float64) == r0)
        idx = np.nonzero(~filled)[0][:int(ok.sum())]
        sel = np.nonzero(ok)[0][:idx.size]
        out[0, idx] = r0[sel].astype(np.float16)
        out[1:, idx] = rest[:, sel]
        filled[idx] = True
    return list(out)


@pytest.mark.parametrize("world", [3, 5, 6, 7])
def test_exchange_mean_rounds_ties_once(parity_report, world):
    nat = _lib()
    dev = torch.device("cuda:0")
    n = 8 * 1024
    gs = _tie_grads(np.random.default_rng(100 + world), n, world)
    exact = np.sum([g.astype(np.float64) for g in gs], axis=0) / world  # every value is an fp16 tie
    assert (exact.astype(np.float16).astype(np.float64) != exact).all()
    sends = [_list(nat, g, dev) for g in gs]
    out, inf, _ = _reduce(nat, sends, n, dev, n // 2)
    want = exact.astype(np.float16)  # numpy: one correctly rounded conversion (ties to even)
    ne = out.view(np.uint16) != want.view(np.uint16)
    assert not ne.any(), (int(ne.sum()), np.argwhere(ne)[:4].ravel().tolist())
    parity_report(f"grad exchange kernels, world {world}: {n} means that are fp16 ties, each rounded once "
                  f"(ties to even), bit-identical to numpy")


def test_exchange_nonfinite_raises_every_rank_flag():
    nat = _lib()
    dev = torch.device("cuda:0")
    n = 8 * 1000
    gs = _sparse_grads(np.random.default_rng(7), n, 2)
    gs[1][11] = np.float16(np.inf)
    gs[1][12] = np.float16(np.nan)
    sends = [_list(nat, g, dev) for g in gs]
    h0, h1 = _decode(sends[0], n, n // 2)[0], _decode(sends[1], n, n // 2)[0]
    assert h0[1] == 0 and h1[1] == 1
    # the non-finite pair (values 11, 12 = pair 5 and 6) is not listed
    assert h1[0] == int(np.count_nonzero(gs[1].view(np.uint32) & 0x7fff7fff)) - 2
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    out, inf, _ = _reduce(nat, sends, n, dev, n // 2, flag)
    assert inf == 1 and np.isfinite(out.astype(np.float32)).all()
    # a rank whose backward kernels raised its GradScaler flag reports it in its header
    local = torch.ones(1, dtype=torch.int32, device=dev)
    assert _decode(_list(nat, gs[0], dev, inf=local), n, n // 2)[0][1] == 1


def test_exchange_overflow_skips_on_every_rank():
    nat = _lib()
    dev = torch.device("cuda:0")
    n = 8 * 3000
    gs = _sparse_grads(np.random.default_rng(3), n, 2)
    cnt = [int(np.count_nonzero(g.view(np.uint32) & 0x7fff7fff)) for g in gs]
    cap = min(cnt) - 1  # both lists overflow; the items past cap are not written
    sends = [_list(nat, g, dev, cap=cap) for g in gs]
    assert [int(_decode(s_, n, cap)[0][0]) for s_ in sends] == cnt  # the header keeps the true count
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    out, inf, stats = _reduce(nat, sends, n, dev, cap, flag)
    assert inf == 2 and not out.any() and stats == [1, max(cnt)]  # skipped (no back-off bit), zero gradient
    ok = [_list(nat, g, dev, cap=max(cnt)) for g in gs]  # at capacity: no overflow
    out, inf, stats = _reduce(nat, ok, n, dev, max(cnt))
    assert inf == 0 and stats[0] == 0 and out.any()


def test_exchange_graph_replays_restart_the_list():
    """list -> (the all-gather: a copy at world 1) -> reduce captured in one
    graph and replayed: the reduce clears the rank's header, so every replay
    lists the same items and writes the same gradient."""
    nat = _lib()
    dev = torch.device("cuda:0")
    n = 8 * 6007
    g = _sparse_grads(np.random.default_rng(11), n, 1)[0]
    grad = torch.from_numpy(g).to(dev)
    cap = n // 2
    words = int(nat.lib().ngp_grad_exchange_words(n, cap))
    send = torch.zeros(words, dtype=torch.int64, device=dev)
    recv = torch.zeros(words, dtype=torch.int64, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    stats = torch.zeros(2, dtype=torch.int32, device=dev)
    lib, P = nat.lib(), nat.ptr

    def body():
        s_ = nat.stream_of(grad)
        nat.check(lib.ngp_grad_exchange_list(P(grad), n, None, P(send), cap, s_), "list")
        recv.copy_(send)
        nat.check(lib.ngp_grad_exchange_reduce(P(recv), 1, cap, P(grad), n, P(flag), P(stats), P(send), s_), "reduce")

    body()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        body()
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    cnt = int(np.count_nonzero(g.view(np.uint32) & 0x7fff7fff))
    assert int(recv[:1].cpu().numpy().view(np.int32)[0]) == cnt and int(send[0]) == 0
    assert stats.cpu().tolist() == [0, cnt] and int(flag[0]) == 0
    want = g.copy()
    want[want == 0] = 0  # a -0 is not listed: the reduce writes +0 there
    assert np.array_equal(grad.cpu().numpy().view(np.uint16), want.view(np.uint16))  # mean of one rank = itself


def test_exchange_empty_lists():
    nat = _lib()
    dev = torch.device("cuda:0")
    n = 64
    sends = [_list(nat, np.zeros(n, np.float16), dev) for _ in range(2)]
    assert all(_decode(s_, n, n // 2)[0][0] == 0 for s_ in sends)
    out, inf, stats = _reduce(nat, sends, n, dev, n // 2)
    assert not out.any() and inf == 0 and stats == [0, 0]


# ---- two ranks of the replicated step on one GPU (gloo) ------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _trainer(dev, distributed, seed=0):
    from nerf.fused import FusedTrainer
    from nerf.network_ff import NeRFNetwork
    from nerf.provider import SyntheticLego, lego_bitfield
    torch.manual_seed(0)
    model = NeRFNetwork(bound=1, cuda_ray=True).to(dev)
    with torch.no_grad():
        model.encoder.embeddings.normal_(0, 0.05)
    model.density_bitfield.copy_(torch.from_numpy(lego_bitfield()).to(dev))
    return FusedTrainer(model, SyntheticLego(dev, num_rays=1024), M=40000, seed=seed, distributed=distributed,
                        options=dict(sparse_exchange=True))


def _params(ft):
    return [p.detach().cpu().numpy().copy() for p in ft.params]


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "torch-ngp_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    try:
        if world == 1:
            # each rank's batch by a single-process trainer (the replicated step
            # seeds rank r's sampler with seed + 7919 r), then Adam on the exact mean
            grads = []
            for r in range(2):
                ft = _trainer(dev, False, seed=7919 * r)
                ft.step()
                torch.cuda.synchronize()
                grads.append(ft.flat_grad.cpu().numpy().copy())
            mean = ((grads[0].astype(np.float64) + grads[1].astype(np.float64)) / 2).astype(np.float16)
            ft.flat_grad.copy_(torch.from_numpy(mean))
            ft.flush()
            torch.cuda.synchronize()
            q.put(("ok", 0, dict(mean=mean, params=_params(ft), grads=grads)))
            return
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ft = _trainer(dev, True)
        assert ft.xchg and not ft.dp and ft.world == 2
        ft.step()  # body + exchange; the update stays pending
        torch.cuda.synchronize()
        out = dict(grad=ft.flat_grad.cpu().numpy().copy(), peak=int(ft._xchg.stats[1]))
        ft.flush()
        torch.cuda.synchronize()
        out["params1"] = _params(ft)
        for _ in range(2):
            ft.step()
        ft.capture(warmup=1)
        for _ in range(3):
            ft.step()
        ft.flush()
        torch.cuda.synchronize()
        out["params"], out["steps"] = _params(ft), ft.optimizer_steps
        # an overflow on rank 0 only: both ranks skip the update and back off
        if rank == 0:
            ft.state.view(torch.float32)[0] = 2.0 ** 40
        scale0, steps0 = ft.scale, ft.optimizer_steps
        ft.step()
        ft.flush()
        torch.cuda.synchronize()
        out["skipped"] = (ft.optimizer_steps == steps0, ft.scale == scale0 * 0.5,
                          all(np.array_equal(a, b) for a, b in zip(out["params"], _params(ft))))
        ft.state.view(torch.float32)[0] = 1024.0  # the same sane scale on both ranks again
        ft.step()  # and the next step trains again from clean gradients
        ft.flush()
        torch.cuda.synchronize()
        out["after"], out["steps_after"] = _params(ft), ft.optimizer_steps
        dist.barrier()
        dist.destroy_process_group()
        q.put(("ok", rank, out))
    except Exception as e:  # report the failure to the parent instead of hanging it
        import traceback
        q.put(("error", rank, repr(e) + traceback.format_exc()))


def _run(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
    for status, rank, o in out:
        assert status == "ok", (rank, o)
    assert all(p.exitcode == 0 for p in procs)
    return [o for _, _, o in sorted(out, key=lambda t: t[1])]


def test_replicated_two_ranks_exact_mean_and_in_sync(parity_report):
    r0, r1 = _run(2)
    ref, = _run(1)
    want = ref["mean"]
    assert np.abs(want.astype(np.float32)).max() > 0
    for o in (r0, r1):  # the exchanged gradient: the exact mean of both batches' gradients
        ne = o["grad"].view(np.uint16) != want.view(np.uint16)
        assert not ne.any(), (int(ne.sum()), np.argwhere(ne)[:4].ravel().tolist())
        for a, b in zip(o["params1"], ref["params"]):  # and Adam on it, as one process runs it
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    nz = [int(np.count_nonzero(g.view(np.uint32) & 0x7fff7fff)) for g in ref["grads"]]
    assert r0["peak"] == r1["peak"] == max(nz)  # the longest list: a rank's nonzero pairs
    for a, b in zip(r0["params"], r1["params"]):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert r0["steps"] == r1["steps"] >= 6
    assert all(r0["skipped"]) and all(r1["skipped"]), (r0["skipped"], r1["skipped"])
    assert r0["steps_after"] == r1["steps_after"] == r0["steps"] + 1
    for a, b in zip(r0["after"], r1["after"]):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) and np.isfinite(a).all()
    parity_report(f"replicated 2-rank step (gloo): exchanged grad bit-identical to the exact mean of the "
                  f"single-process grads (longest list {r0['peak']} items), params bit-identical across ranks, "
                  f"rank-0 overflow skipped on both ranks")

"""CPU, world_size 2 over gloo: the ray-sharded data-parallel path.

Each rank draws its own ray shard (seed + rank) and computes gradients on it;
nerf.train.average_gradients must leave every rank holding the gradient of
the mean loss over the union of the shards, and identical parameters after
an optimizer step (the same contract RCCL provides on the 8x MI355X node)."""
import os
import socket

import numpy as np

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(32, 64, bias=False), torch.nn.ReLU(),
                               torch.nn.Linear(64, 16, bias=False))


def _shard(rank, n=256):
    g = torch.Generator().manual_seed(1000 + rank)
    return torch.randn(n, 32, generator=g), torch.randn(n, 16, generator=g)


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "torch-ngp_amd")]
    from nerf.train import average_gradients
    from nerf.utils import get_rays
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = _model()
    for p in m.parameters():  # bench.py broadcasts initial parameters the same way
        dist.broadcast(p.data, 0)
    x, y = _shard(rank)
    loss = ((m(x) - y) ** 2).mean()
    loss.backward()
    average_gradients(list(m.parameters()))
    grads = [p.grad.clone() for p in m.parameters()]
    opt = torch.optim.Adam(m.parameters(), lr=1e-2, betas=(0.9, 0.99), eps=1e-15)
    opt.step()
    params = [p.detach().clone() for p in m.parameters()]
    # per-rank ray sampling: different pixels on different ranks
    torch.manual_seed(1234 + rank)
    pose = torch.eye(4)[None]
    rays = get_rays(pose, [1111.0, 1111.0, 400.0, 400.0], 800, 800, 64)
    q.put((rank, [g.numpy() for g in grads], [p.numpy() for p in params], rays["inds"].numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gradient_average_matches_full_batch():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, g, prm, inds = q.get(timeout=120)
        out[r] = (g, prm, inds)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference: mean loss over the union of both shards
    m = _model()
    xs, ys = zip(*[_shard(r) for r in range(world)])
    loss = ((m(torch.cat(xs)) - torch.cat(ys)) ** 2).mean()
    loss.backward()
    for r in range(world):
        for g, p in zip(out[r][0], m.parameters()):
            torch.testing.assert_close(torch.from_numpy(g), p.grad, rtol=1e-5, atol=1e-7)
    for a, b in zip(out[0][1], out[1][1]):
        assert (a == b).all()
    assert not (out[0][2] == out[1][2]).all()


# ---- the fused engine's ZeRO-1 sharding (nerf/zero1.py) over gloo ----------------
# The fused step's collectives on the flat buffers of its ShardPlan: guard
# poison at the head of every rank's chunk, averaging reduce-scatter into the
# owner's shard, the fused optimizer's arithmetic on the shard's sections only
# (GradScaler's inf check of the shard, unscale, torch.optim.Adam with
# betas (0.9, 0.99), eps 1e-15, LambdaLR 0.1 ** (epoch / iters);
# csrc/ngp_step.h adam_consts / adam_update / step_end_block, restated below
# in float32 with the kernels' operation order), all-gather of the updated
# values. The result must equal one process running torch.optim.Adam over the
# whole flat buffer with the mean gradient; a rank's poisoned gradient must
# reach every owner's shard, so every rank skips the step and backs the scale
# off together.
_SIZES = [2 * 40013, 7168, 11264]  # a small table + the NeRF sigma / colour MLPs


def _flat_grad(plan, rank):
    g = torch.Generator().manual_seed(77 + rank)
    flat = torch.zeros(plan.total, dtype=torch.float16)
    for v in plan.views(flat):
        v.copy_(torch.randn(v.numel(), generator=g).half())
    return flat


_LR, _B1, _B2, _EPS, _ITERS = 1e-2, 0.9, 0.99, 1e-15, 30000


class _ShardAdam:
    """The fused optimizer on one rank's shard (csrc/ngp_step.h): the state's
    GradScaler scale / growth tracker / Adam step / LR epoch, the shard's
    moments, the inf check over the averaged fp16 shard (NGP_SCALER_SCAN)."""

    def __init__(self, n, scale=65536.0):
        self.m, self.v = torch.zeros(n), torch.zeros(n)
        self.scale, self.tracker, self.step, self.epoch = scale, 0, 0, 0

    def update(self, p, g16, sections, lo):
        import math
        inf = not bool(torch.isfinite(g16.float()).all())
        f32 = torch.float32
        inv_scale = torch.tensor(1.0 / self.scale, dtype=torch.float64).to(f32)  # (float)(1.0 / (double)scale)
        step = self.step + 1
        lr = _LR * 0.1 ** min(self.epoch / _ITERS, 1.0)
        step_size = torch.tensor(lr / (1.0 - _B1 ** step), dtype=torch.float64).to(f32)
        inv_bc2 = 1.0 / torch.tensor(math.sqrt(1.0 - _B2 ** step), dtype=torch.float64).to(f32)
        b1, b2, eps = (torch.tensor(x, dtype=f32) for x in (_B1, _B2, _EPS))
        if not inf:
            for a, n, _ in sections:
                s = slice(lo + a, lo + a + n)
                gk = g16[a:a + n].float() * inv_scale
                m, v = self.m[a:a + n], self.v[a:a + n]
                m += (1.0 - b1) * (gk - m)
                v.mul_(b2).add_((1.0 - b2) * gk * gk)
                denom = torch.sqrt(v) * inv_bc2 + eps
                p[s] -= step_size * (m / denom)
        # GradScaler.update (growth_interval 2000 is not reached here), LR epoch, Adam step
        if inf:
            self.scale *= 0.5
            self.tracker = 0
        else:
            self.tracker += 1
            self.step += 1
        self.epoch += 1
        return inf


def _zero1_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "torch-ngp_amd")]
    from nerf.zero1 import ShardPlan
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    plan = ShardPlan(_SIZES, world, rank)
    params = torch.linspace(-1, 1, plan.total)
    opt = _ShardAdam(plan.chunk)
    shard = torch.empty(plan.chunk, dtype=torch.float16)
    fulls = []
    for it in range(3):  # three averaged updates of this rank's shard, gathered after each
        flat = _flat_grad(plan, rank + 10 * it)
        dist.reduce_scatter_tensor(shard, flat, op=dist.ReduceOp.AVG)
        assert not opt.update(params, shard, plan.sections(split_first=False), plan.lo)
        full = torch.empty(plan.total)
        dist.all_gather_into_tensor(full, params[plan.lo:plan.hi].contiguous())
        params = full.clone()
        fulls.append(full.numpy())
    # guard: rank 1's gradient overflowed; it poisons the head of every chunk
    bad = _flat_grad(plan, rank)
    if rank == 1:
        bad[torch.arange(world) * plan.chunk] = float("nan")
    dist.reduce_scatter_tensor(shard, bad, op=dist.ReduceOp.AVG)
    before = params.clone()
    skipped = opt.update(params, shard, plan.sections(split_first=False), plan.lo)
    q.put((rank, fulls, bool(torch.isnan(shard[0]).item()), plan.lo, plan.hi, plan.chunk, skipped,
           bool(torch.equal(before, params)), opt.scale, opt.step))
    dist.barrier()
    dist.destroy_process_group()


def test_zero1_shard_plan_layout():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "torch-ngp_amd")]
    from nerf.zero1 import ShardPlan
    sizes = [12239728, 7168, 11264]  # the Lego table, sigma and colour MLPs
    one = ShardPlan(sizes)
    assert one.starts == [0, 12239728, 12246896] and one.used == 12258160
    assert one.sections(True) == [(0, 12239728, False), (12239728, one.chunk - 12239728, True)]
    for world in (2, 4, 8):
        plans = [ShardPlan(sizes, world, r) for r in range(world)]
        p0 = plans[0]
        assert p0.chunk % 64 == 0 and p0.total >= p0.used and p0.total - p0.used < 64 * world
        # every value of every tensor is owned by exactly one rank
        for k, n in enumerate(sizes):
            spans = sorted(p.owned(k) for p in plans if p.owned(k)[1] > 0)
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def test_zero1_reduce_scatter_update_all_gather_two_ranks():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "torch-ngp_amd")]
    from nerf.zero1 import ShardPlan
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_zero1_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=300) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    plan = ShardPlan(_SIZES, 2, 0)
    # one process: torch.optim.Adam (+ LambdaLR) over the whole flat buffer with
    # the mean gradient (the fp16 average the reduction outputs), unscaled
    ref = torch.nn.Parameter(torch.linspace(-1, 1, plan.total))
    adam = torch.optim.Adam([ref], lr=_LR, betas=(_B1, _B2), eps=_EPS)
    sched = torch.optim.lr_scheduler.LambdaLR(adam, lambda it: 0.1 ** min(it / _ITERS, 1))
    refs = []
    for it in range(3):
        mean = ((_flat_grad(plan, 10 * it).float() + _flat_grad(plan, 1 + 10 * it).float()) / 2).half()
        ref.grad = mean.float() * (1.0 / 65536.0)  # GradScaler: the scaled fp16 grad x (1 / scale)
        adam.step()
        sched.step()
        refs.append(ref.detach().clone())
    for rank, fulls, poisoned, lo, hi, chunk, skipped, unchanged, scale, steps in out:
        assert (lo, hi) == (rank * chunk, (rank + 1) * chunk)
        for full, want in zip(fulls, refs):  # fused arithmetic vs torch's Adam: fp32 rounding of the same formula
            torch.testing.assert_close(torch.from_numpy(full), want, rtol=1e-6, atol=1e-7)
        assert poisoned  # the overflow on rank 1 reached rank 0's shard too
        assert skipped and unchanged and scale == 32768.0 and steps == 3  # every rank skipped and backed off
    assert np.array_equal(out[0][1][-1], out[1][1][-1])  # both ranks hold the same gathered parameters


# ---- the replicated step's touched-entry exchange (nerf/exchange.py) over gloo ----
# SparseExchange's host side (the fixed-size list buffers, their all-gather,
# the kernels' arguments) with its two kernels (csrc/exchange.hip) restated on
# the CPU: every rank must end with the exact mean of all ranks' fp16
# gradients rounded once to fp16, the same bits on every rank; a non-finite
# value on one rank raises every rank's GradScaler flag; a list longer than
# the capacity makes every rank skip (flag bit 1, zero gradient).
_BIN = 4096  # pairs per bin (csrc/exchange.hip kBinPairs)


def _exchange_grads(rank, n, step):
    rng = np.random.default_rng(100 * step + rank)
    g = np.zeros(n, np.float16)
    k = int(rng.integers(n // 20, n // 4))  # ragged: every rank lists a different number of pairs
    idx = rng.choice(n, k, replace=False)
    g[idx] = (rng.standard_normal(k) * 10.0 ** rng.integers(-8, 4, k)).astype(np.float16)
    g[:8] = np.float16(1.5 + rank)  # pairs every rank touches
    return g


def _exchange_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "torch-ngp_amd")]
    import nerf.exchange as xm
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class _Lib:  # the buffer-size arithmetic of csrc/exchange.hip
        @staticmethod
        def ngp_grad_exchange_bins(n):
            return (n // 2 + _BIN - 1) // _BIN

        @staticmethod
        def ngp_grad_exchange_words(n, cap):
            return 2 + _Lib.ngp_grad_exchange_bins(n) + cap

    xm.nat.lib = lambda: _Lib

    class CpuExchange(xm.SparseExchange):
        """The kernels restated in numpy; a bin's items in index order, the
        bins' segments placed in a rank-dependent order (the device reserves
        them with atomics)."""

        def list(self):
            w = self.grad.view(torch.int32).numpy().view(np.uint32)
            bad = ((w & 0x7c00) == 0x7c00) | ((w & 0x7c000000) == 0x7c000000)
            ok = ((w & 0x7fff7fff) != 0) & ~bad
            send = self.send.numpy().view(np.uint64)
            assert send[0] == 0  # cleared by the last reduce (or a new buffer)
            send[:] = 0
            hdr = send[:2].view(np.int32)
            hdr[1] = int(bad.any() or int(self.inf_flag[0]) != 0)
            nb, pos = self.n_bins, 0
            for b in np.random.default_rng(rank).permutation(nb):
                idx = np.nonzero(ok[b * _BIN:(b + 1) * _BIN])[0] + b * _BIN
                send[2 + b] = (np.uint64(idx.size) << np.uint64(32)) | np.uint64(pos)
                for j, p in enumerate(idx):
                    if pos + j < self.cap:
                        send[2 + nb + pos + j] = (np.uint64(w[p]) << np.uint64(32)) | np.uint64(p)
                pos += idx.size
            hdr[0] = pos

        def reduce(self):
            recv = self.recv.numpy().view(np.uint64).reshape(self.world, self.words)
            hdr = recv[:, :2].copy().view(np.int32).reshape(self.world, 4)
            self.send[0] = 0  # the next list starts from a zero header
            over = bool((hdr[:, 0] > self.cap).any())
            if (hdr[:, 1] & 1).any() or over:
                self.inf_flag[0] |= (1 if (hdr[:, 1] & 1).any() else 0) | (2 if over else 0)
            self.stats[0] += int(over)
            self.stats[1] = max(int(self.stats[1]), int(hdr[:, 0].max()))
            acc = np.zeros(self.n, np.int64)
            if not over:
                nb = self.n_bins
                for r in range(self.world):
                    for b in range(nb):
                        t = recv[r, 2 + b]
                        start, cnt = int(t & np.uint64(0xffffffff)), int(t >> np.uint64(32))
                        it = recv[r, 2 + nb + start:2 + nb + start + cnt]
                        pair = (it & np.uint64(0xffffffff)).astype(np.int64)
                        h = (it >> np.uint64(32)).astype(np.uint32).view(np.float16).reshape(-1, 2)
                        for c in range(2):
                            np.add.at(acc, 2 * pair + c, (h[:, c].astype(np.float64) * 2.0 ** 24).astype(np.int64))
            self.grad.copy_(torch.from_numpy((acc.astype(np.float64) * 2.0 ** -24 / self.world).astype(np.float16)))

    n = 8 * 4096 + 64  # 5 bins, the last one ragged
    flat = torch.zeros(n, dtype=torch.float16)
    inf = torch.zeros(1, dtype=torch.int32)
    xc = CpuExchange(flat, inf, world, nccl=False, cap=n // 2)
    outs = []
    for step in range(2):
        flat.copy_(torch.from_numpy(_exchange_grads(rank, n, step)))
        xc()
        outs.append((flat.numpy().copy(), int(inf[0]), int(xc.stats[1])))
    # rank 1 overflows: every rank's flag goes up, nothing non-finite reaches the mean
    g = _exchange_grads(rank, n, 2)
    if rank == 1:
        g[100] = np.float16(np.inf)
    flat.copy_(torch.from_numpy(g))
    xc()
    outs.append((flat.numpy().copy(), int(inf[0]), int(xc.stats[1])))
    # a list over the capacity: every rank skips (bit 1), zero gradient, counted
    inf.zero_()
    xc.resize(16)
    flat.copy_(torch.from_numpy(_exchange_grads(rank, n, 0)))
    xc()
    outs.append((flat.numpy().copy(), int(inf[0]), xc.overflows))
    q.put((rank, outs))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sparse_exchange_exact_mean_on_every_rank(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = 8 * 4096 + 64
    peak = 0
    for step in range(3):
        gs = [_exchange_grads(r, n, step) for r in range(world)]
        if step == 2:
            gs[1][100] = 0  # the non-finite value is dropped from the sum
        want = (np.sum([g.astype(np.float64) for g in gs], axis=0) / world).astype(np.float16)
        peak = max([peak] + [int(np.count_nonzero(g.view(np.uint32) & 0x7fff7fff)) for g in gs])
        for r in range(world):
            got, inf, seen = out[r][step]
            assert np.array_equal(got.view(np.uint16), want.view(np.uint16)), (step, r)
            assert inf == (1 if step == 2 else 0) and seen == peak
    for r in range(world):
        got, inf, overflows = out[r][3]
        assert inf == 2 and overflows == 1 and not got.any()

"""CPU, world_size 2 over gloo: the ray-sharded data-parallel path.

Each rank draws its own ray shard (seed + rank) and computes gradients on it;
nerf.train.average_gradients must leave every rank holding the gradient of
the mean loss over the union of the shards, and identical parameters after
an optimizer step (the same contract RCCL provides on the 8x MI355X node)."""
import os
import socket

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
# owner's shard, an update of the shard's optimizer sections only, all-gather
# of the updated values. The result must equal one process updating the whole
# flat buffer with the mean gradient; a rank's poisoned gradient must reach
# every owner's shard.
_SIZES = [2 * 40013, 7168, 11264]  # a small table + the NeRF sigma / colour MLPs


def _flat_grad(plan, rank):
    g = torch.Generator().manual_seed(77 + rank)
    flat = torch.zeros(plan.total, dtype=torch.float16)
    for v in plan.views(flat):
        v.copy_(torch.randn(v.numel(), generator=g).half())
    return flat


def _update(p, g, sections, lo):
    """A stand-in elementwise optimizer over [lo + a, lo + a + n) sections."""
    for a, n, _ in sections:
        s = slice(lo + a, lo + a + n)
        p[s] -= 0.1 * g[a:a + n].float() + 0.01 * p[s]


def _zero1_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "torch-ngp_amd")]
    from nerf.zero1 import ShardPlan
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    plan = ShardPlan(_SIZES, world, rank)
    params = torch.linspace(-1, 1, plan.total)
    flat = _flat_grad(plan, rank)
    shard = torch.empty(plan.chunk, dtype=torch.float16)
    dist.reduce_scatter_tensor(shard, flat, op=dist.ReduceOp.AVG)
    _update(params, shard, plan.sections(split_first=False), plan.lo)
    full = torch.empty(plan.total)
    dist.all_gather_into_tensor(full, params[plan.lo:plan.hi].contiguous())
    # guard: rank 1's gradient overflowed; it poisons the head of every chunk
    bad = _flat_grad(plan, rank)
    if rank == 1:
        bad[torch.arange(world) * plan.chunk] = float("nan")
    dist.reduce_scatter_tensor(shard, bad, op=dist.ReduceOp.AVG)
    q.put((rank, full.numpy(), bool(torch.isnan(shard[0]).item()), plan.lo, plan.hi, plan.chunk))
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
    # one process: the mean gradient (fp16 average, as the reduction's output) over the whole buffer
    mean = ((_flat_grad(plan, 0).float() + _flat_grad(plan, 1).float()) / 2).half()
    ref = torch.linspace(-1, 1, plan.total)
    _update(ref, mean, [(0, plan.total, True)], 0)
    for rank, full, poisoned, lo, hi, chunk in out:
        assert (lo, hi) == (rank * chunk, (rank + 1) * chunk)
        assert torch.allclose(torch.from_numpy(full), ref, rtol=0, atol=2e-3)
        assert poisoned  # the overflow on rank 1 reached rank 0's shard too

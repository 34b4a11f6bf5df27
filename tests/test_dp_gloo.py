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

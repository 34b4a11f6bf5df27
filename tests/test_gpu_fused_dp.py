"""GPU, world_size 2: the fused engine's data-parallel path.

Both ranks run on the one visible GPU (gloo backend, which stages device
tensors through the host; RCCL needs one GPU per rank). Each rank draws its
own rays; the flat fp16 gradient is averaged by a reduce-scatter, each rank's
optimizer updates its shard and the fp16 forward copy is all-gathered
(ZeRO-1): after a few steps, captured included, and flush(), both ranks must
hold bit-identical parameters, and they must differ from a single-rank run.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "torch-ngp_amd")]
    import torch.distributed as dist
    from nerf.fused import FusedTrainer
    from nerf.network_ff import NeRFNetwork
    from nerf.provider import SyntheticLego, lego_bitfield
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = NeRFNetwork(bound=1, cuda_ray=True).to(dev)
    with torch.no_grad():
        model.encoder.embeddings.normal_(0, 0.05)
    model.density_bitfield.copy_(torch.from_numpy(lego_bitfield()).to(dev))
    ft = FusedTrainer(model, SyntheticLego(dev, num_rays=1024), M=40000, distributed=world > 1)
    if world > 1:  # the data-parallel defaults this test covers: draw-ahead, the tail in
        # the grid forward's launch, the live-row backwards (gloo: the three-graph form)
        assert ft.dp and ft._draw_ahead and ft._dp_tail and ft._live and not ft._nccl
    for _ in range(3):
        ft.step()
    ft.capture(warmup=1)
    for _ in range(3):
        ft.step()
    ft.flush()
    torch.cuda.synchronize()
    params = [p.detach().cpu().numpy() for p in ft.params]
    steps = ft.optimizer_steps
    # GradScaler under the sharded optimizer: an overflow on ONE rank must make
    # every rank skip the step and back the scale off (its backward's kernels
    # raise the rank's flag, ngp_grad_guard spreads it to every shard)
    if rank == 0:
        ft.state.view(torch.float32)[0] = 2.0 ** 40  # this rank's fp16 grads overflow
    scale0 = ft.scale
    ft._sample()
    ft._march()
    ft._network()
    ft._reduce()
    ft._optimizer()
    ft._gather_half(wait=True)
    torch.cuda.synchronize()
    skipped = (ft.optimizer_steps == steps, ft.scale == scale0 * 0.5,
               all(np.array_equal(a, p.detach().cpu().numpy()) for a, p in zip(params, ft.params)))
    q.put((rank, params, steps, skipped))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _equiv_worker(rank, world, port, q):
    """world 2: ONE data-parallel step from the same initial parameters; returns
    this rank's averaged gradient shard and the parameters after flush().
    world 1: the same step's gradients of each rank's batch, computed one
    rank-seed at a time by single-process trainers."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "torch-ngp_amd")]
    import torch.distributed as dist
    from nerf.fused import FusedTrainer
    from nerf.network_ff import NeRFNetwork
    from nerf.provider import SyntheticLego, lego_bitfield
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)

    def trainer(distributed, seed=0):
        torch.manual_seed(0)
        model = NeRFNetwork(bound=1, cuda_ray=True).to(dev)
        with torch.no_grad():
            model.encoder.embeddings.normal_(0, 0.05)
        model.density_bitfield.copy_(torch.from_numpy(lego_bitfield()).to(dev))
        opts = dict(exact_reduce=True) if distributed and os.environ.get("NGP_TEST_EXACT_REDUCE") else None
        return FusedTrainer(model, SyntheticLego(dev, num_rays=1024), M=40000, seed=seed, distributed=distributed,
                            options=opts)

    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ft = trainer(True)
        ft.step()  # sample -> march -> network -> reduce-scatter (the update stays pending)
        torch.cuda.synchronize()
        shard = ft.grad_shard.cpu().numpy()
        ft.flush()
        torch.cuda.synchronize()
        q.put((rank, ft.lo, shard, [p.detach().cpu().numpy() for p in ft.params], ft.total, ft._exact_reduce))
        dist.barrier()
        dist.destroy_process_group()
        return
    grads = []
    for r in range(2):  # the data-parallel sampler seeds rank r with seed + 7919 r
        ft = trainer(False, seed=7919 * r)
        ft._sample()
        ft._forward_backward()
        torch.cuda.synchronize()
        grads.append(ft.flat_grad.clone())
    # the gradient of the mean loss over both batches, then the optimizer on it
    mean = ((grads[0].float() + grads[1].float()).half() / 2)
    exact = ((grads[0].float() + grads[1].float()) / 2).half()  # DDP's arithmetic: fp32 sum, / world, one rounding
    ft.flat_grad.copy_(mean)
    ft._optimizer()
    torch.cuda.synchronize()
    q.put((0, 0, mean.cpu().numpy(), [p.detach().cpu().numpy() for p in ft.params], ft.total, exact.cpu().numpy()))


def _run(world, target=_worker):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=600) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return out


def test_fused_data_parallel_two_ranks_stay_in_sync():
    two = _run(2)
    (_, p0, s0, k0), (_, p1, s1, k1) = two
    assert s0 == s1 >= 6
    for a, b in zip(p0, p1):
        assert np.array_equal(a, b)
    assert all(k0) and all(k1), (k0, k1)  # both ranks skipped the step with rank 0's inf
    (_, ps, _, _), = _run(1)
    assert any(not np.array_equal(a, b) for a, b in zip(p0, ps))  # the other rank's rays mattered


def test_zero1_step_equals_single_process_step_on_both_batches():
    """ZeRO-1 equivalence: the averaged gradient the two ranks' reduce-scatter
    leaves in their shards is the mean of the two batches' gradients computed
    by single-process trainers, and the parameters after the sharded update
    (flush: Adam per shard + all-gather) equal a single-process Adam step on
    that mean."""
    two = sorted(_run(2, _equiv_worker), key=lambda t: t[0])
    (_, _, want, p_ref, total, _), = _run(1, _equiv_worker)
    got = np.zeros(total, np.float16)
    for _, lo, shard, _, _, _ in two:
        got[lo:lo + shard.size] = shard
    g, w = got.astype(np.float64), want.astype(np.float64)
    assert np.abs(w).max() > 0
    assert np.linalg.norm(g - w) <= 1e-3 * np.linalg.norm(w)
    assert (got.view(np.uint16) == want.view(np.uint16)).mean() >= 0.999
    for p in (two[0][3], two[1][3]):  # both ranks hold the full, identical parameters
        for a, b in zip(p, p_ref):
            assert np.abs(a - b).max() <= 2.5e-2  # Adam's first step is lr * sign(g)
            assert (a == b).mean() >= 0.999


def test_zero1_exact_reduce_is_the_fp32_mean(parity_report, monkeypatch):
    """options exact_reduce: the reduce-scatter runs in
    fp32 (SUM, / world) and rounds each averaged value to fp16 once -- the
    arithmetic of the reference's DDP all-reduce of fp32 gradients
    (nerf/utils.py:325-327). The two ranks' shards equal fp16((g0 + g1) / 2)
    from single-process trainers' gradients bit for bit."""
    monkeypatch.setenv("NGP_TEST_EXACT_REDUCE", "1")
    two = sorted(_run(2, _equiv_worker), key=lambda t: t[0])
    assert all(t[5] for t in two)
    (_, _, _, _, total, exact), = _run(1, _equiv_worker)
    got = np.zeros(total, np.float16)
    for _, lo, shard, _, _, _ in two:
        got[lo:lo + shard.size] = shard
    assert np.abs(exact.astype(np.float32)).max() > 0
    ne = got.view(np.uint16) != exact.view(np.uint16)
    assert not ne.any(), (int(ne.sum()), np.argwhere(ne)[:4].ravel().tolist())
    parity_report(f"ZeRO-1 exact_reduce, 2 ranks: {total} averaged gradient values bit-identical to "
                  f"fp16(fp32 sum / 2) of the single-process gradients")


def _density_worker(rank, world, port, q):
    """update_density on every rank: same draws, sharded queries, MAX
    all-reduce of the scratch grid."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "torch-ngp_amd")]
    import torch.distributed as dist
    from nerf.fused import FusedTrainer
    from nerf.network_ff import NeRFNetwork
    from nerf.provider import SyntheticLego, lego_bitfield
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = NeRFNetwork(bound=1, cuda_ray=True).to(dev)
    with torch.no_grad():
        model.encoder.embeddings.normal_(0, 0.3)
    model.density_bitfield.copy_(torch.from_numpy(lego_bitfield()).to(dev))
    ft = FusedTrainer(model, SyntheticLego(dev, num_rays=256), M=20000, distributed=world > 1)
    for it in range(3):
        if it == 2:
            model.iter_density = 16
        ft.update_density()
    torch.cuda.synchronize()
    q.put((rank, model.density_grid.cpu().numpy(), model.density_bitfield.cpu().numpy()))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def test_update_density_is_rank_consistent():
    two = sorted(_run(2, _density_worker), key=lambda t: t[0])
    (_, g1, b1), = _run(1, _density_worker)
    for _, g, b in two:
        assert np.array_equal(b, b1)
        np.testing.assert_allclose(g, g1, rtol=0, atol=0)

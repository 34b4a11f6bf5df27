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


def _run(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
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

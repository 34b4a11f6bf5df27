"""GPU, RCCL: the fused engine's data-parallel step over a one-rank `nccl`
(= RCCL on ROCm) process group, in a spawned child process.

FusedTrainer(distributed=True) takes the ZeRO-1 path at any world size: three
hipGraphs, ngp_grad_guard, `reduce_scatter_tensor(op=AVG)` of the flat fp16
gradient on RCCL's stream, the sharded Adam, the async
`all_gather_into_tensor` of the fp16 forward copy overlapped with the next
batch's sample + march, flush()'s all-gather of the fp32 masters, and the
density update's MAX all-reduce. With one rank every collective is an
identity, so the run must equal the single-process (non data-parallel) step
bit for bit: parameters, Adam moments, GradScaler state, density grid and
bitfield (reference hook: nerf/utils.py:325-327, the DDP wrap this replaces).
This is the code path the driver's 8-GPU bench runs; here it executes RCCL on
the one GPU of the box. The replicated step (options sparse_exchange: the
world-1 step on every rank, the gradients averaged by the touched-entry
exchange of nerf/exchange.py) must equal it too: at world 1 the exchange's
exact fixed-point mean of one rank's list is that rank's gradient.
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


def _trainer(dev, distributed, mode="whole_step_graph"):
    from nerf.fused import FusedTrainer
    from nerf.network_ff import NeRFNetwork
    from nerf.provider import SyntheticLego, lego_bitfield
    torch.manual_seed(0)
    model = NeRFNetwork(bound=1, cuda_ray=True).to(dev)
    with torch.no_grad():
        model.encoder.embeddings.normal_(0, 0.05)
    model.density_bitfield.copy_(torch.from_numpy(lego_bitfield()).to(dev))
    opts = dict(sparse_exchange=True) if mode == "sparse_exchange" else dict(dp_graph=mode != "three_graphs")
    if mode == "exact_reduce":
        opts["exact_reduce"] = True
    return FusedTrainer(model, SyntheticLego(dev, num_rays=1024), M=40000, distributed=distributed, options=opts)


def _snap(ft):
    ft.flush()
    torch.cuda.synchronize()
    return [p.detach().cpu().numpy().copy() for p in ft.params]


def _run_steps(ft):
    phases = {}
    ft.step()
    phases["step1"] = _snap(ft)
    for _ in range(2):  # eager
        ft.step()
    phases["eager3"] = _snap(ft)
    ft.capture(warmup=1)
    for _ in range(4):  # graph replays (+ the collectives between them)
        ft.step()
    phases["graphs"] = _snap(ft)
    ft.update_density()  # flushes, then the density update (MAX all-reduce in dp)
    for _ in range(2):
        ft.step()
    ft.flush()
    torch.cuda.synchronize()
    m1, m2 = ft._moments()
    return dict(phases=phases, params=[p.detach().cpu().numpy() for p in ft.params],
                m=m1[:ft._starts[-1] + ft.params[-1].numel()].cpu().numpy(),
                v=m2[:ft._starts[-1] + ft.params[-1].numel()].cpu().numpy(),
                steps=ft.optimizer_steps, scale=ft.scale, loss=ft.last_loss,
                grid=ft.model.density_grid.cpu().numpy(), bits=ft.model.density_bitfield.cpu().numpy(),
                mean_density=ft.mean_density, dp=ft.dp, xchg=ft.xchg, nccl=ft._nccl,
                whole=getattr(ft, "_dp_whole", None) is not None)


def _worker(port, q, mode):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "torch-ngp_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    try:
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        backend = dist.get_backend()
        # the whole step, collectives included, in one graph (the default), or three graphs
        dp = _run_steps(_trainer(dev, True, mode))
        single = _run_steps(_trainer(dev, False))
        dist.barrier()
        dist.destroy_process_group()
        q.put(("ok", backend, dp, single))
    except Exception as e:  # report the failure to the parent instead of hanging it
        import traceback
        q.put(("error", repr(e), traceback.format_exc(), None))


@pytest.mark.parametrize("mode", ["three_graphs", "whole_step_graph", "sparse_exchange", "exact_reduce"])
def test_rccl_world1_data_parallel_step_equals_single_process(parity_report, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q, mode))
    p.start()
    status, backend, dp, single = q.get(timeout=300)
    p.join(timeout=60)
    assert status == "ok", (backend, dp)
    assert p.exitcode == 0
    assert backend == "nccl" and dp["nccl"] and not single["dp"] and not single["xchg"]
    if mode == "sparse_exchange":
        assert dp["xchg"] and not dp["dp"]
    else:
        assert dp["dp"] and not dp["xchg"]
        assert dp["whole"] == (mode != "three_graphs")  # the graph phase replayed the whole-step graph
    assert dp["steps"] == single["steps"] >= 8 and dp["scale"] == single["scale"]
    assert np.isfinite(dp["loss"]) and dp["loss"] == single["loss"]
    for ph in dp["phases"]:  # first phase where the runs part, and by how much
        for k, (a, b) in enumerate(zip(dp["phases"][ph], single["phases"][ph])):
            ne = a.view(np.uint32) != b.view(np.uint32)
            assert not ne.any(), (ph, ["table", "sigma", "color"][k], int(ne.sum()),
                                  float(np.abs(a - b).max()), np.argwhere(ne)[:4].tolist())
    ng = dp["grid"].view(np.uint32) != single["grid"].view(np.uint32)
    assert not ng.any(), ("density grid", int(ng.sum()), float(np.abs(dp["grid"] - single["grid"]).max()))
    assert np.array_equal(dp["bits"], single["bits"]) and dp["mean_density"] == single["mean_density"]
    for k, (a, b) in enumerate(zip(dp["params"], single["params"])):
        ne = a.view(np.uint32) != b.view(np.uint32)
        assert not ne.any(), ("final", ["table", "sigma", "color"][k], int(ne.sum()), float(np.abs(a - b).max()),
                              np.argwhere(ne)[:4].tolist())
    assert np.array_equal(dp["m"].view(np.uint32), single["m"].view(np.uint32))
    assert np.array_equal(dp["v"].view(np.uint32), single["v"].view(np.uint32))
    parity_report(f"RCCL world 1 data-parallel step ({mode}): "
                  f"{dp['steps']} optimizer steps, params / moments / density grid bit-identical to the "
                  f"single-process step, loss {dp['loss']:.6f}")

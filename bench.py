"""Train-step rays/s of the instant-ngp hot path on synthetic 800x800 Lego.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    (N > 1: launched by torch.distributed.run, one rank per GPU, RCCL)

One step = sample 4096 rays of a random training pose -> near/far ->
march_rays_train -> hash-grid encode -> sigma FFMLP -> trunc_exp -> SH ->
colour FFMLP -> composite -> MSE -> full backward -> Adam.
--engine fused (default): nerf/fused.py, the step as 11 fused launches in
one hipGraph; --engine autograd: nerf/train.py, the same step through the
reference-API autograd Functions (torch glue ops between them).
The roofline's grid backward is timed by the kernels themselves on the chip's
100 MHz constant clock over the timed region's own graph replays (bin launch
start -> accumulate end, NGP_GRID_TIMING; ROCm refuses event nodes inside
captured graphs); the other per-launch device times come from HIP events
between the launches of eager steps run right after the timed region, with
the sample counts of those same steps.
The density bitfield is the analytic Lego-like fixture (density-grid update
excluded from the timed step as SURVEY §8(d) defines it; its cost is reported
separately as `density_update_ms`). Rank 0 prints ONE JSON line.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "torch-ngp_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "train-step rays/sec (fwd+bwd) on 800×800 Lego; 1/2/4/8 MI355X"
PUBLISHED_V100_RAYS_PER_S = 97 * 4096  # readme.md:211 via BASELINE.md (V100, torch -O)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
FP16_MFMA_PEAK_TFLOPS = 2500.0  # dense fp16 MFMA (spec)


# name -> (description, H, W, log2_hashmap_size, occupancy, bound, dt_gamma)
WORKLOADS = {
    "lego": ("lego_800x800_train_step (synthetic analytic Lego, bound 1, 1 cascade, 128^3 bitfield fixture, "
             "hashgrid L16 C2 T2^19, FFMLP 64-wide)", 800, 800, 19, "boxes", 1, 0.0),
    "lego_dense": ("lego_800x800_dense_occupancy_train_step (synthetic Lego, bound 1, ball r=0.7 occupancy, "
                   "hashgrid L16 C2 T2^19, FFMLP 64-wide)", 800, 800, 19, "ball", 1, 0.0),
    "truck": ("truck_1920x1080_train_step (Config 5 single-GPU leg: synthetic scene at 1920x1080, bound 1, "
              "hashgrid L16 C2 T2^22 = 39.6M entries, FFMLP 64-wide)", 1080, 1920, 22, "boxes", 1, 0.0),
    "fox": ("fox_shaped_800x800_train_step (Config 3 shapes on the synthetic scene: bound 2, 2 cascades, "
            "dt_gamma 1/128, desired_resolution 4096, hashgrid L16 C2 T2^19, FFMLP 64-wide)", 800, 800, 19,
            "boxes", 2, 1.0 / 128),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--num_rays", type=int, default=4096)
    ap.add_argument("--no-graph", dest="graph", action="store_false")
    ap.add_argument("--kernel-steps", type=int, default=10,
                    help="eager instrumented steps for kernel timing (only without --ring / hipGraphs)")
    ap.add_argument("--ring", type=int, default=0,
                    help="copies of the step graph with event-record nodes, replayed in turn in the timed "
                         "region; per-launch times are read from the last min(steps, ring) of them. ROCm 7 "
                         "refuses event nodes in captured graphs ('External events are disallowed in rocm'), "
                         "so the default 0 times the launches with events between eager steps run right after "
                         "the timed region, with those steps' own sample counts")
    ap.add_argument("--graph-steps", type=int, default=10,
                    help="fused engine, world 1: training steps captured back to back in one hipGraph (the "
                         "timed region replays it K / S times, every step complete); 1: one step per graph")
    ap.add_argument("--settle-steps", type=int, default=1000,
                    help="untimed steps after the warmup that bring the GPU to its sustained clock")
    ap.add_argument("--cpu-budget", type=float, default=20.0, help="seconds of CPU baseline work")
    ap.add_argument("--no-cpu", dest="cpu", action="store_false")
    ap.add_argument("--engine", choices=["fused", "autograd"], default="fused")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="lego",
                    help="lego: the headline (Config 2, Lego 800x800, box occupancy, ~19 samples/ray); "
                         "lego_dense: same with a ball occupancy (~80 samples/ray); "
                         "truck: Config 5 single-GPU leg (1920x1080, log2T 22); "
                         "fox: Config 3 shapes (bound 2, 2 cascades, dt_gamma 1/128)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="collective backend for N > 1: nccl (= RCCL, the measured path) or gloo "
                         "(host-staged; a rehearsal of the data-parallel step with every rank on the "
                         "visible GPUs, e.g. 2 ranks on a 1-GPU box)")
    return ap.parse_args()


class KernelTimer:
    """HIP-event timing of one _backend entry (one kernel launch per call) on
    the stream it is launched on (torch's current stream)."""

    def __init__(self, namespace, attr):
        self.ns, self.attr = namespace, attr
        self.fn = getattr(namespace, attr)
        self.pairs = []
        self.active = False

    def __enter__(self):
        def wrapped(*a, **k):
            if not self.active:
                return self.fn(*a, **k)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            r = self.fn(*a, **k)
            e.record()
            self.pairs.append((s, e))
            return r
        setattr(self.ns, self.attr, wrapped)
        return self

    def __exit__(self, *exc):
        setattr(self.ns, self.attr, self.fn)

    def mean_ms(self):
        torch.cuda.synchronize()
        ts = [s.elapsed_time(e) for s, e in self.pairs]
        return float(np.mean(ts)) if ts else float("nan")


def launch_cmd(gpus, argv, port):
    """The torch.distributed.run command line that starts `gpus` ranks of this
    script (one per GPU, rendezvous on 127.0.0.1) with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` without a launcher: start the N ranks as a child
        # torch.distributed.run (this process has made no GPU call) and exit
        # with its status; rank 0 of the children prints the JSON line
        import subprocess
        sys.exit(subprocess.call(launch_cmd(args.gpus, sys.argv[1:], _free_port())))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if world > 1 and args.backend == "gloo":
        local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        dist.init_process_group("gloo")
    elif world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)
    # what the collective layer itself reports (the ranks RCCL / gloo joined)
    comm = {"backend": dist.get_backend() if world > 1 else None,
            "world_size": dist.get_world_size() if world > 1 else 1}
    assert comm["world_size"] == args.gpus
    torch.manual_seed(1234 + rank)
    np.random.seed(rank)

    from nerf.network_ff import NeRFNetwork
    from nerf.provider import SyntheticLego, lego_bitfield, sphere_bitfield

    desc, img_h, img_w, log2T, occ, bound, dt_gamma = WORKLOADS[args.workload]
    model = NeRFNetwork(bound=bound, cuda_ray=True, density_thresh=10, log2_hashmap_size=log2T).to(dev)
    if world > 1:  # identical initial parameters on every rank
        for p in model.parameters():
            dist.broadcast(p.data, 0)
    bits = (lego_bitfield(cascade=model.cascade, bound=float(bound)) if occ == "boxes"
            else sphere_bitfield(cascade=model.cascade, bound=float(bound)))
    bits = torch.from_numpy(bits).to(dev)
    model.density_bitfield.copy_(bits)
    data = SyntheticLego(dev, H=img_h, W=img_w, num_rays=args.num_rays)
    args.dt_gamma = dt_gamma
    if args.engine == "fused":
        result = run_fused(args, model, data, bits, world, dev)
    else:
        result = run_autograd(args, model, data, bits, world, dev)
    result["config"]["collective"] = comm
    result["config"]["workload"] = desc
    result["config"]["image_hw"] = [img_h, img_w]
    spr = result["config"]["samples_per_step"] / args.num_rays
    result["samples_per_ray"] = round(spr, 2)
    result["samples_per_s"] = round(result["value"] * spr, 1)

    if rank == 0 and world == 1 and args.cpu:
        result["cpu_baseline"] = cpu_baseline(model, data, args)

    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_autograd(args, model, data, bits, world, dev):
    """The step through the reference-API autograd Functions (nerf/train.py)."""
    import gridencoder.backend as gb
    import ffmlp.backend as fb
    import raymarching.backend as rb
    from nerf.train import Trainer

    trainer = Trainer(model, data, lr=1e-2, iters=30000, fp16=True, update_density=False,
                      distributed=world > 1, dt_gamma=args.dt_gamma)

    # warm-up: first step sizes the sample buffer with a D2H sync (mean_count = 0
    # path of raymarching.py); afterwards mean_count is fixed from the measured
    # counts, exactly what update_extra_state does upstream every 16 steps.
    counts = []
    n_first = max(2, min(args.warmup, 8))
    for _ in range(n_first):
        trainer.train_step()
        counts.append(int(model.step_counter[(model.local_step - 1) % 16, 0].item()))
    mean_count = int(np.mean(counts) * 1.25)
    if world > 1:
        t = torch.tensor([mean_count], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        mean_count = int(t.item())
    model.mean_count = mean_count
    for _ in range(max(0, args.warmup - n_first)):
        trainer.train_step()
    used_graph = False
    if args.graph:
        try:
            trainer.capture()
            for _ in range(3):
                trainer.step()
            used_graph = True
        except Exception as e:  # eager steps are the same kernels; record why
            print(f"[bench] graph capture failed, running eager: {e!r}", file=sys.stderr)
            trainer.graph = None
            trainer.static = None
    torch.cuda.synchronize()

    # ---------------- timed region ----------------
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = trainer.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    rays_total = args.num_rays * world * args.steps
    value = rays_total / elapsed
    samples = model.step_counter[:, 0].float()
    samples_per_step = int(samples[samples > 0].mean().item()) if (samples > 0).any() else 0

    # -------- per-kernel HIP-event timing (eager steps, same shapes) --------
    trainer_graph, trainer_static = trainer.graph, trainer.static
    trainer.graph, trainer.static = None, None
    timers = {
        "grid_encode_backward": KernelTimer(gb._backend, "grid_encode_backward_bm"),
        "grid_encode_forward": KernelTimer(gb._backend, "grid_encode_forward_bm"),
        "ffmlp_backward": KernelTimer(fb._backend, "ffmlp_backward"),
        "ffmlp_forward": KernelTimer(fb._backend, "ffmlp_forward"),
        "march_rays_train": KernelTimer(rb._backend, "march_rays_train"),
        "composite_rays_train_forward": KernelTimer(rb._backend, "composite_rays_train_forward"),
        "composite_rays_train_backward": KernelTimer(rb._backend, "composite_rays_train_backward"),
    }
    for tm in timers.values():
        tm.__enter__()
    for tm in timers.values():
        tm.active = True
    for _ in range(args.kernel_steps):
        trainer.train_step()
    kernel_ms = {k: tm.mean_ms() for k, tm in timers.items()}
    for tm in timers.values():
        tm.__exit__()
    trainer.graph, trainer.static = trainer_graph, trainer_static
    M_k = samples_per_step
    # algorithmic bytes; fp16 table, D=3, L=16, C=2
    grid_fwd_bytes = 588 * M_k
    grid_bwd_bytes = 1100 * M_k
    per_call_calls = {"grid_encode_forward": 1}
    dominant = max(("grid_encode_backward", "grid_encode_forward"), key=lambda k: kernel_ms[k])
    dom_bytes = grid_bwd_bytes if dominant == "grid_encode_backward" else grid_fwd_bytes
    achieved = dom_bytes / (kernel_ms[dominant] * 1e-3) / 1e9
    ffmlp_flops = 110592 * M_k
    mlp_ms = kernel_ms["ffmlp_forward"] * 2 + kernel_ms["ffmlp_backward"] * 2
    del per_call_calls

    # density-grid update cost (reported, not in the timed step)
    density = density_update_times(model, bits)

    result = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "rays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / PUBLISHED_V100_RAYS_PER_S, 3),
        "dtype": "fp16",
        "data": "synthetic",
        "config": {
            "num_rays_per_gpu": args.num_rays,
            "global_batch_rays": args.num_rays * world,
            "samples_per_step": samples_per_step,
            "mean_count_M": mean_count,
            "parallelism": f"dp{world}",
            "hipgraph": used_graph,
            "baseline_ref": "V100 97 it/s x 4096 rays (readme.md:211)",
        },
        "roofline": {
            "kernel": dominant,
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": pmc_traffic(dominant, args.workload)[0],
            "traffic_source": pmc_traffic(dominant, args.workload)[1],
            "algorithmic_bytes_per_launch": int(dom_bytes),
            "avg_launch_ms": round(kernel_ms[dominant], 5),
        },
        "kernels_ms": {k: round(v, 5) for k, v in kernel_ms.items()},
        "ffmlp_mfma": {"flops_per_step": ffmlp_flops, "ms": round(mlp_ms, 5),
                        "tflops": round(ffmlp_flops / (mlp_ms * 1e-3) / 1e12, 2) if mlp_ms > 0 else None,
                        "peak_tflops": FP16_MFMA_PEAK_TFLOPS},
        "density_update_ms": density,
        "loss": float(loss.float().item()),
    }

    result["config"]["engine"] = "autograd"
    return result


def run_fused(args, model, data, bits, world, dev):
    from nerf.fused import FusedTrainer

    # sample-buffer size: measured counts x 1.25 (mean_count, update_extra_state)
    probe = FusedTrainer(model, data, M=args.num_rays * 64, distributed=world > 1, dt_gamma=args.dt_gamma)
    counts = []
    for _ in range(4):
        probe.step()
        counts.append(probe.sample_count())
    mean_count = int(np.mean(counts) * 1.25)
    if world > 1:
        t = torch.tensor([mean_count], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        mean_count = int(t.item())
    probe.flush()  # data parallel: every rank's shard of the masters gathered back
    del probe
    torch.cuda.empty_cache()
    ft = FusedTrainer(model, data, M=mean_count, distributed=world > 1, dt_gamma=args.dt_gamma)
    for _ in range(max(1, args.warmup)):
        ft.step()
    used_graph = False
    timing = "eager"
    if args.graph:
        try:
            ft.capture(multi=args.graph_steps if world == 1 else 1)
            ft.run(3 * max(1, args.graph_steps))
            used_graph = True
        except Exception as e:  # eager launches are the same kernels; record why
            print(f"[bench] graph capture failed, running eager: {e!r}", file=sys.stderr)
            ft.graph = None
    if used_graph and args.ring > 0 and not ft.dp:
        try:  # the timed region replays graphs that carry event-record nodes
            ft.capture(warmup=1, ring=min(args.ring, 16))
            timing = "graph_events"
        except Exception as e:
            print(f"[bench] timing-ring capture failed, per-launch times from eager steps: {e!r}",
                  file=sys.stderr)
    torch.cuda.synchronize()
    # clock settle: the GPU raises its clocks only under sustained load. A
    # 20-step run right after 5 warmup steps measured 15.0M rays/s against
    # 17.3M for 200 steps on the same box (profiles/r02zl_settle.txt), so a
    # fixed number of untimed steps (same on every rank: they hold
    # collectives) runs before the timed region.
    for i in range(0, args.settle_steps, 64):
        ft.run(min(64, args.settle_steps - i))
        torch.cuda.synchronize()
    torch.cuda.synchronize()

    # ---------------- timed region ----------------
    if world > 1:
        dist.barrier()
    ft.grid_timing_reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ft.run(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    grid_clock = ft.grid_timing(last=args.steps)  # the timed region's grid backwards (<= 256 of them)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = args.num_rays * world * args.steps / elapsed
    samples = model.step_counter[:, 0].float()
    samples_per_step = int(samples[samples > 0].mean().item()) if (samples > 0).any() else 0
    loss = ft.last_loss

    # ---------------- per-kernel device time (roofline) ----------------
    # timing "graph_events": the event nodes of the last min(steps, ring) graph
    # replays of the timed region, with those steps' own sample counts;
    # "eager": eager steps after the timed region, events between launches
    if timing == "graph_events":
        kernel_ms, per_replay, counts = ft.ring_times(last=args.steps)
    else:
        ft.flush()
        kernel_ms, per_replay, counts = ft.timed_steps(args.kernel_steps, with_counts=True)
    counts = [min(int(c), ft.M) for c in counts]
    rows = float(np.mean(counts))  # mean samples per step of the timed launches
    # SURVEY §8(d) per-sample bytes; achieved = sum of bytes / sum of times
    per_sample = {"grid_encode_backward": 1100, "grid_encode_forward": 588}
    dominant = max(per_sample, key=lambda k: kernel_ms[k])
    dom_bytes = per_sample[dominant] * rows
    achieved = per_sample[dominant] * sum(counts) / (sum(per_replay[dominant]) * 1e-3) / 1e9
    roof_timing = {"timing": timing, "launches_timed": len(counts), "samples_per_timed_launch": counts,
                   "launch_ms_per_timed_step": [round(v, 5) for v in per_replay[dominant]],
                   "avg_launch_ms": round(kernel_ms[dominant], 5)}
    if dominant == "grid_encode_backward" and grid_clock and grid_clock[0] == args.steps:
        # the grid backward's own clock over the timed region's graph replays:
        # bin launch start -> accumulate end on the 100 MHz constant clock,
        # the samples of exactly those launches (NGP_GRID_TIMING)
        _, ms, samp = grid_clock
        calls = len(ms)
        dom_bytes = per_sample[dominant] * sum(samp) / calls
        achieved = per_sample[dominant] * sum(samp) / (sum(ms) * 1e-3) / 1e9
        roof_timing = {"timing": "device_clock_timed_region", "launches_timed": calls,
                       "samples_timed": sum(samp), "avg_launch_ms": round(sum(ms) / calls, 5),
                       "launch_ms_min_median_max": [round(float(v), 5) for v in
                                                    (min(ms), np.median(ms), max(ms))],
                       "eager_events": {"avg_launch_ms": round(kernel_ms[dominant], 5),
                                        "frac": round(per_sample[dominant] * sum(counts)
                                                      / (sum(per_replay[dominant]) * 1e-3) / 1e9
                                                      / HBM_PEAK_GBS, 4)}}
    mlp_ms = sum(v for k, v in kernel_ms.items() if k.startswith("ffmlp"))
    ffmlp_flops = 110592 * rows
    step_bytes = whole_step_bytes(rows, args.num_rays, sum(p.numel() for p in model.parameters()),
                                  int(model.encoder.embeddings.numel()))

    density = density_update_times(model, bits, ft)

    return {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "rays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / PUBLISHED_V100_RAYS_PER_S, 3),
        "dtype": "fp16",
        "data": "synthetic",
        "config": {
            "num_rays_per_gpu": args.num_rays,
            "global_batch_rays": args.num_rays * world,
            "samples_per_step": samples_per_step,
            "mean_count_M": mean_count,
            "parallelism": f"dp{world}",
            "hipgraph": used_graph,
            "graph_steps": ft._multi if used_graph and ft.graph_multi is not None else 1,
            "settle_steps": args.settle_steps,
            "engine": "fused",
            "dt_gamma": args.dt_gamma,
            "cascade": int(model.cascade),
            "bound": float(model.bound),
            "baseline_ref": "V100 97 it/s x 4096 rays (readme.md:211)",
        },
        "roofline": {
            "kernel": dominant,
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": pmc_traffic(dominant, args.workload)[0],
            "traffic_source": pmc_traffic(dominant, args.workload)[1],
            "algorithmic_bytes_per_launch": int(dom_bytes),
            **roof_timing,
        },
        "kernels_ms": {k: round(v, 5) for k, v in kernel_ms.items()},
        "ffmlp_mfma": {"flops_per_step": int(ffmlp_flops), "ms": round(mlp_ms, 5),
                        "tflops": round(ffmlp_flops / (mlp_ms * 1e-3) / 1e12, 2) if mlp_ms > 0 else None,
                        "peak_tflops": FP16_MFMA_PEAK_TFLOPS},
        # SURVEY §8(d)'s secondary figure: the step's algorithmic bytes over the
        # whole step time (per rank) against the HBM peak
        "step_roofline": {"algorithmic_bytes": int(step_bytes),
                          "frac": round(step_bytes / (ms_per_step * 1e-3) / (HBM_PEAK_GBS * 1e9), 4)},
        "density_update_ms": density,
        # beside the headline (which SURVEY §8(d) defines without it): the step
        # with upstream's density-grid cadence amortized in, one partial
        # device-draw update (FusedTrainer.update_density) per 16 steps
        "with_density_update": amortized_density(ms_per_step, density, args.num_rays * world),
        "loss": loss,
    }


def amortized_density(ms_per_step, density, rays_per_step):
    """ms/step and rays/s with one partial density update per 16 steps
    (nerf/utils.py update_extra_interval = 16), or None if not measured."""
    upd = (density or {}).get("fused_partial")
    if not upd or not ms_per_step:
        return None
    ms = ms_per_step + upd / 16.0
    return {"ms_per_step": round(ms, 4), "rays_per_s": round(rays_per_step / (ms * 1e-3), 1),
            "update": "fused_partial / 16"}


def density_update_times(model, bits, ft=None, reps=3):
    """Wall time (ms, best of `reps`, synchronised) of one density-grid update
    (excluded from the step; upstream runs it every 16 steps):
    the reference-API update_extra_state (torch draws, device query / EMA /
    packbits) and, with a fused trainer, its device-draw update_density; full
    updates (the first 16) and partial ones. The bitfield fixture is restored
    afterwards."""
    def best(fn, it0):
        ts = []
        for _ in range(reps + 1):
            model.iter_density = it0
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e3)
        return round(min(ts[1:]), 3)

    def ref_update():
        with torch.autocast("cuda", dtype=torch.float16):
            model.update_extra_state()

    grid0 = model.density_grid.clone()
    out = {}
    for name, it0 in (("full", 0), ("partial", 16)):
        model.density_grid.copy_(grid0)
        out[f"update_extra_state_{name}"] = best(ref_update, it0)
        if ft is not None:
            model.density_grid.copy_(grid0)
            out[f"fused_{name}"] = best(ft.update_density, it0)
    model.density_grid.copy_(grid0)
    model.iter_density = 0
    model.density_bitfield.copy_(bits)
    if ft is not None:
        ft.refresh_occupancy()
    return out


_PMC_KERNELS = {"grid_encode_backward": ("k_grid_bwd_bin", "k_grid_bin_accum"),
                "grid_encode_forward": ("k_grid_fwd_pair",)}


def whole_step_bytes(samples, rays, n_params, n_table):
    """Algorithmic HBM bytes of one step per SURVEY §8(d): grid forward 588 B and
    backward 1,100 B per sample (+ the fp16 table grad's zero fill, 2 B per table
    value), march 48 B/ray + 32 B/sample, composite forward 32 B/ray + 24
    B/sample and backward 52 B/ray + 40 B/sample, SH 76 B/direction, dense Adam
    28 B/parameter."""
    return (588 * samples + 1100 * samples + 2 * n_table + 48 * rays + 32 * samples + 32 * rays + 24 * samples
            + 52 * rays + 40 * samples + 76 * samples + 28 * n_params)


def pmc_traffic(kernel, workload="lego"):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    of the SAME workload (profiles/r*_step_kernels.json with its "workload"
    key; summaries without one are the default Lego bench), written by
    tools/prof.sh + tools/prof_summary.py from separate --pmc FETCH_SIZE /
    WRITE_SIZE passes over this bench. FETCH_SIZE doubled per
    MI355X_MICROARCH.md's HBM section (gfx950 tallies wide streaming reads at
    half); WRITE_SIZE as read. None when no summary of this workload exists."""
    import glob
    def order(f):  # rNN then the tag: r01z < r01ab < r02a
        tag = os.path.basename(f).split("_")[0]
        return (int(tag[1:3]) if tag[1:3].isdigit() else 0, len(tag), tag)
    files = []
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_step_kernels*.json")), key=order):
        try:
            doc = json.load(open(f))
        except (OSError, ValueError):
            continue
        if doc.get("workload", "lego") == workload and doc.get("pmc_per_launch"):
            files.append((f, doc))
    if not files:
        return None, None
    pmc = files[-1][1]["pmc_per_launch"]
    files = [files[-1][0]]
    fetch = write = 0
    found = False
    for pre in _PMC_KERNELS.get(kernel, ()):
        for k, v in pmc.items():
            if k.startswith(pre) and "#" not in k:
                fetch += v.get("fetch_bytes", 0)
                write += v.get("write_bytes", 0)
                found = True
    if not found:
        return None, None
    return int(2 * fetch + write), {"file": os.path.relpath(files[-1], ROOT), "fetch_size_raw": int(fetch),
                                    "write_size": int(write)}


def host_threads():
    """Host threads this process may use: the CPUs it is pinned to, capped by
    OMP_NUM_THREADS when set (os.cpu_count() counts the whole machine, which on
    a shared GPU box is many times this process's share)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp))) if omp and omp.isdigit() else n


def cpu_baseline(model, data, args):
    """BASELINE.json configs[0] on the host: the pure-PyTorch Config 1 train
    step (oracle/torch_nerf.py: run() uniform sampling with 512 steps, torch
    hash grid + SH, nn.Linear MLPs, Adam; synthetic Lego 200x200, 4096 rays) on
    all of this process's host threads, kind "pytorch". Beside it (`port`):
    the oracle's C/numpy restatement of the Config-2 step (the cuda_ray
    pipeline) on one thread, for a same-shape ratio."""
    from oracle import torch_nerf
    threads = host_threads()
    rps, steps, secs, losses = torch_nerf.time_train_steps(threads, budget_s=args.cpu_budget, warmup=1,
                                                           max_steps=5, num_rays=args.num_rays)
    out = {"value": round(rps, 2), "unit": "rays/s", "cores": threads, "kind": "pytorch",
           "sample": f"{steps} timed Config-1 train steps x {args.num_rays} rays x 512 samples (synthetic Lego "
                     f"200x200, fp32, after 1 warm-up) in {secs:.1f}s on {threads} threads "
                     f"(torch.set_num_threads), oracle/torch_nerf.py"}
    out["port"] = port_baseline(model, data, args)
    return out


def port_baseline(model, data, args):
    """The oracle's CPU restatement of the Config-2 train step (kind 'port'),
    single-threaded, on a bounded sample of 4096-ray batches."""
    try:
        from threadpoolctl import threadpool_limits
    except ImportError:  # pragma: no cover
        threadpool_limits = None
    import oracle
    from oracle.pipeline import CPUNeRF, time_cpu_baseline

    emb = model.encoder.embeddings.detach().float().cpu().numpy()
    cpu = CPUNeRF(emb, model.encoder.offsets.cpu().numpy(), model.encoder.per_level_scale,
                  model.sigma_net.weights.detach().float().cpu().numpy(),
                  model.color_net.weights.detach().float().cpu().numpy(),
                  model.density_bitfield.cpu().numpy())
    oracle.build()
    batches = []
    for _ in range(8):
        b = data.sample()
        ro = b["rays_o"][0].cpu().numpy().astype(np.float32)
        rd = b["rays_d"][0].cpu().numpy().astype(np.float32)
        rgba = b["images"][0].cpu().numpy().astype(np.float32)
        bg = np.random.rand(ro.shape[0], 3).astype(np.float32)
        noises = np.random.rand(ro.shape[0]).astype(np.float32)
        batches.append((ro, rd, rgba, bg, noises))
    ctx = threadpool_limits(1) if threadpool_limits else None
    if ctx:
        ctx.__enter__()
    try:
        rps, steps, rays, secs, m = time_cpu_baseline(cpu, batches, args.cpu_budget / 2)
    finally:
        if ctx:
            ctx.__exit__(None, None, None)
    return {"value": round(rps, 2), "unit": "rays/s", "cores": 1, "kind": "port",
            "sample": f"{steps} train steps x {args.num_rays} rays (the benched workload, mean {int(m)} "
                      f"samples/step) in {secs:.1f}s, oracle/pipeline.py, 1 thread"}


if __name__ == "__main__":
    main()

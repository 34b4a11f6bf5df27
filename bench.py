"""Train-step rays/s of the instant-ngp hot path on synthetic 800x800 Lego.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    (N > 1: launched by torch.distributed.run, one rank per GPU, RCCL)

One step = sample 4096 rays of a random training pose -> near/far ->
march_rays_train -> hash-grid encode -> sigma FFMLP -> trunc_exp -> SH ->
colour FFMLP -> composite -> MSE -> full backward -> Adam.
--engine fused (default): nerf/fused.py, the step as 8 fused launches in
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
    "fox": ("fox_shaped_800x800_train_step (Config 3 shapes: bound 2, 2 cascades, dt_gamma 1/128, "
            "desired_resolution 4096, a Fox-shaped ellipsoid occupancy, hashgrid L16 C2 T2^19, FFMLP 64-wide)",
            800, 800, 19, "fox", 2, 1.0 / 128),
}
LEGS = ("lego_dense", "truck", "fox")


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
    ap.add_argument("--no-legs", dest="legs", action="store_false",
                    help="skip the other workloads (lego_dense, truck, fox) run after the headline at N=1")
    ap.add_argument("--leg-steps", type=int, default=50)
    ap.add_argument("--leg-settle", type=int, default=300)
    ap.add_argument("--no-render", dest="render", action="store_false",
                    help="skip the test-render speed (one full image per iteration) at N=1")
    ap.add_argument("--no-dp-path", dest="dp_path", action="store_false",
                    help="skip the data-parallel engine path measured on a one-rank RCCL group at N=1")
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
    ap.add_argument("--exchange", choices=["zero1", "sparse"], default="zero1",
                    help="data-parallel gradient exchange for N > 1: zero1 (reduce-scatter + sharded Adam + "
                         "all-gather, whole step in one graph) or sparse (every rank runs the world-1 step and "
                         "the full Adam; touched-entry lists all-gathered, DESIGN.md section 7)")
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
    # stdout carries exactly the one JSON line: whatever the libraries print on
    # file descriptor 1 (RCCL's version banner at communicator init) goes to
    # stderr, the JSON line to the saved descriptor
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
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
            "world_size": dist.get_world_size() if world > 1 else 1,
            "exchange": args.exchange if world > 1 else None}
    assert comm["world_size"] == args.gpus
    torch.manual_seed(1234 + rank)
    np.random.seed(rank)

    model, data, bits, desc, img_h, img_w, dt_gamma = make_workload(args.workload, dev, world, args.num_rays)
    args.dt_gamma = dt_gamma
    ft = None
    if args.engine == "fused":
        result, ft = run_fused(args, model, data, bits, world, dev)
    else:
        result = run_autograd(args, model, data, bits, world, dev)
    result["config"]["collective"] = comm
    result["config"]["workload"] = desc
    result["config"]["image_hw"] = [img_h, img_w]
    spr = result["config"]["samples_per_step"] / args.num_rays
    result["samples_per_ray"] = round(spr, 2)
    result["samples_per_s"] = round(result["value"] * spr, 1)
    if args.engine == "fused" and ft.live_fraction() is not None:
        # the backwards walk only these rows (the rest carry a zero gradient)
        result["live_rows_frac"] = round(ft.live_fraction(), 4)
    if world == 1 and args.engine == "fused":
        result["touched"] = touched_pairs(ft)
        ft.flush()
        if args.render:
            result["render"] = render_probe(args, model, data, dev)
        if args.dp_path:
            result["dp_path"] = dp_path_probe(args, model, data, dev, result)
        if args.legs:
            del ft
            torch.cuda.empty_cache()
            result["legs"] = {w: run_leg(args, w, dev) for w in LEGS if w != args.workload}

    if rank == 0 and world == 1 and args.cpu:
        result["cpu_baseline"] = cpu_baseline(model, data, args)

    if rank == 0:
        sys.stdout.flush()
        line = (json.dumps(result) + "\n").encode()
        while line:
            line = line[os.write(json_fd, line):]
    if world > 1:
        dist.destroy_process_group()


def make_workload(name, dev, world, num_rays):
    """Model (random init, identical on every rank), its benched occupancy
    bitfield and the synthetic dataset of a WORKLOADS entry."""
    from nerf.network_ff import NeRFNetwork
    from nerf.provider import SyntheticLego, fox_bitfield, lego_bitfield, sphere_bitfield
    desc, img_h, img_w, log2T, occ, bound, dt_gamma = WORKLOADS[name]
    model = NeRFNetwork(bound=bound, cuda_ray=True, density_thresh=10, log2_hashmap_size=log2T).to(dev)
    if world > 1:  # identical initial parameters on every rank
        for p in model.parameters():
            dist.broadcast(p.data, 0)
    occupancy = {"boxes": lego_bitfield, "ball": sphere_bitfield, "fox": fox_bitfield}[occ]
    bits = torch.from_numpy(occupancy(cascade=model.cascade, bound=float(bound))).to(dev)
    model.density_bitfield.copy_(bits)
    data = SyntheticLego(dev, H=img_h, W=img_w, num_rays=num_rays)
    return model, data, bits, desc, img_h, img_w, dt_gamma


def run_leg(args, name, dev):
    """One more workload in the same invocation (N=1): the same timed region
    (warmup, capture, clock settle, exactly leg_steps complete steps), with its
    samples / ray, rays/s and the grid backward on its own clock beside the
    same workload's committed PMC traffic."""
    model, data, bits, desc, img_h, img_w, dt_gamma = make_workload(name, dev, 1, args.num_rays)
    ft, mean_count = make_trainer(args, model, data, 1, dev, dt_gamma)
    elapsed, used_graph, grid_clock = timed_run(args, ft, 1, dev, args.leg_steps, 5, args.leg_settle,
                                                args.graph_steps)
    counts = ft._recent_counts(min(16, args.leg_steps)).float().mean().item()
    rays_s = args.num_rays * args.leg_steps / elapsed
    out = {"workload": desc, "rays_per_s": round(rays_s, 1), "ms_per_step": round(elapsed / args.leg_steps * 1e3, 4),
           "steps": args.leg_steps, "samples_per_ray": round(counts / args.num_rays, 2),
           "samples_per_s": round(rays_s * counts / args.num_rays, 1), "mean_count_M": mean_count,
           "hipgraph": used_graph,
           "grid_encode_backward": grid_roofline(grid_clock, args.leg_steps, name,
                                                 counts if getattr(ft, "_live", False) else None)}
    if ft.live_fraction() is not None:
        out["live_rows_frac"] = round(ft.live_fraction(), 4)
    out["touched"] = touched_pairs(ft)
    del ft, model
    torch.cuda.empty_cache()
    return out


def touched_pairs(ft, steps=4):
    """Nonzero fp16 channel pairs of a step's flat gradient (table + MLPs):
    what one rank lists per step in the replicated step's touched-entry
    exchange (8 bytes each), against the dense buffer."""
    n = []
    for _ in range(steps):
        ft.step()  # the step's gradient stays in flat_grad until the next step's Adam
        torch.cuda.synchronize()
        n.append(int(((ft.flat_grad.view(torch.int32) & 0x7fff7fff) != 0).sum()))
    pairs = float(np.mean(n))
    return {"pairs_per_step": round(pairs, 1), "list_bytes": int(8 * pairs), "flat_pairs": int(ft.total // 2),
            "dense_fp16_bytes": int(2 * ft.total), "frac": round(pairs / (ft.total // 2), 4)}


def render_probe(args, model, data, dev, images=5, pose=7):
    """Test-render speed (the reference publishes 7.8 it/s
    test speed on a V100, readme.md:211): one full HxW image per iteration of
    the model as the bench run trained it, eval mode, through the
    device-driven loop (nerf/fused_render.py: march / network / composite with
    the alive-ray list kept on the device, K iterations per hipGraph replay,
    one host read of the loop state per replay), wall time per image
    synchronised; beside it the reference-API loop (NeRFRenderer.run_cuda,
    one host sync per iteration) on the same rays."""
    from nerf.fused_render import FusedRenderer
    from nerf.utils import get_rays
    model.eval()
    try:
        rays = get_rays(data.poses[pose:pose + 1], data.intrinsics, data.H, data.W, -1)
        ro, rd = rays["rays_o"], rays["rays_d"]
        N = data.H * data.W
        r = FusedRenderer(model, N, dt_gamma=args.dt_gamma)
        r.load_weights()
        r.capture()

        def timed(fn, reps):
            ts = []
            for _ in range(reps + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                out = fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            return float(np.mean(ts[1:])), out

        secs, out = timed(lambda: r.render(ro, rd, bg_color=1), images)
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
            ref_secs, ref = timed(lambda: model.render(ro, rd, staged=True, bg_color=1, perturb=False,
                                                       dt_gamma=args.dt_gamma, max_steps=1024), 2)
        diff = (out["image"].reshape(-1, 3) - ref["image"].reshape(-1, 3).float()).abs().max(-1).values
        res = {"metric": "test render (one full image per iteration, inference march / network / composite loop)",
               "image_hw": [data.H, data.W], "images_timed": images, "ms_per_image": round(secs * 1e3, 3),
               "it_per_s": round(1.0 / secs, 2), "rays_per_s": round(N / secs, 1),
               "device_iterations": r.iterations, "iterations_per_graph": r.K,
               "reference_api_loop": {"ms_per_image": round(ref_secs * 1e3, 3), "it_per_s": round(1.0 / ref_secs, 2)},
               "image_vs_reference_api": {"pixels_within_1e-3": round(float((diff <= 1e-3).float().mean()), 6),
                                          "max_abs": float(diff.max())},
               "weights_sum_mean": round(float(out["weights_sum"].mean()), 4),
               "baseline_ref": "V100 7.8 it/s test speed (readme.md:211)",
               "vs_published": round(1.0 / secs / 7.8, 2)}
        del r
        torch.cuda.empty_cache()
        return res
    finally:
        model.train()


def dp_path_probe(args, model, data, dev, headline):
    """The data-parallel engine path (FusedTrainer(distributed=True), ZeRO-1:
    three graphs, grad guard, reduce-scatter, sharded Adam, async all-gather)
    on a one-rank RCCL (`nccl`) group on this GPU: its per-rank step time and
    per-phase times (eager, serial phases with events between them; at world
    1 the collectives are RCCL's local copies), the bytes each rank's
    collectives move per step at 8 ranks, and what the 1 -> 8 scaling target
    leaves for exposed collective time. Reference: the DDP all-reduce it
    replaces, nerf/utils.py:325-327."""
    import socket
    if dist.is_initialized():
        return None
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        m2, d2, bits2, _, _, _, dtg = make_workload(args.workload, dev, 1, args.num_rays)
        # the engine's data-parallel step as the N > 1 bench runs it: the whole
        # step (collectives included) captured in one graph, graph_steps per replay
        ft, _ = make_trainer(args, m2, d2, 1, dev, dtg, distributed=True)
        assert ft.dp and ft._nccl
        steps = max(20, args.steps)
        elapsed, used_graph, _ = timed_run(args, ft, 1, dev, steps, 5, 300, args.graph_steps)
        ms = elapsed / steps * 1e3
        whole_captured = bool(used_graph and ft._dp_whole is not None)
        graph_steps = ft._multi
        phases = ft.timed_steps(args.kernel_steps)
        # the three-graph form (dp_graph=False: collectives between the graphs), for comparison
        m3, d3, _, _, _, _, _ = make_workload(args.workload, dev, 1, args.num_rays)
        ft3, _ = make_trainer(args, m3, d3, 1, dev, dtg, distributed=True, options=dict(dp_graph=False))
        e3, g3, _ = timed_run(args, ft3, 1, dev, steps, 5, 300, 1)
        three = {"ms_per_step": round(e3 / steps * 1e3, 4), "graphs": bool(g3)}
        del ft3, m3
        # the replicated step (sparse_exchange, DESIGN.md section 7 option B): the
        # world-1 step graph with the touched-entry exchange captured after its
        # backward (list kernel, one fixed-size all-gather, reduce kernel; no
        # host read-back)
        m4, d4, _, _, _, _, _ = make_workload(args.workload, dev, 1, args.num_rays)
        ft4, _ = make_trainer(args, m4, d4, 1, dev, dtg, distributed=True, options=dict(sparse_exchange=True))
        assert ft4.xchg
        e4, g4, _ = timed_run(args, ft4, 1, dev, steps, 5, 300, 1)
        xc = ft4._xchg
        timed_longest = int(xc.stats[1])  # the timed steps' longest list (statistics restarted by the fit)
        mean_list = touched_pairs(ft4)["pairs_per_step"]
        fit_peak = getattr(ft4, "xchg_fit_peak", None)
        sparse = {"ms_per_step": round(e4 / steps * 1e3, 4), "graphs": bool(g4),
                  "whole_step_graph": ft4.graph is not None, "list_cap": xc.cap,
                  "fit": "2 x the longest list of the trailing settle block (statistics restarted before it)",
                  "fit_window_longest_list": fit_peak, "longest_list": timed_longest,
                  "mean_list": mean_list,
                  "longest_over_mean": round(timed_longest / mean_list, 3) if mean_list else None,
                  "cap_over_longest": round(xc.cap / max(timed_longest, 1), 3),
                  "list_bytes_per_rank": xc.bytes_per_step()[0],
                  "pairs_total": int(xc.pairs), "overflows": xc.overflows,
                  "per_rank_bytes_8_ranks": {"send": xc.bytes_per_step()[0], "receive": 7 * xc.bytes_per_step()[0],
                                             "zero1_reduce_scatter_plus_all_gather":
                                                 int(2 * 2 * ft4.total * 7 / 8)}}
        del ft4, m4
        # ZeRO-1 with the gradient reduced in fp32 (options exact_reduce: DDP's
        # arithmetic, twice the reduce-scatter's bytes)
        m5, d5, _, _, _, _, _ = make_workload(args.workload, dev, 1, args.num_rays)
        ft5, _ = make_trainer(args, m5, d5, 1, dev, dtg, distributed=True, options=dict(exact_reduce=True))
        e5, g5, _ = timed_run(args, ft5, 1, dev, steps, 5, 300, args.graph_steps)
        exact = {"ms_per_step": round(e5 / steps * 1e3, 4), "graphs": bool(g5),
                 "whole_step_graph": ft5._dp_whole is not None,
                 "per_rank_bytes_8_ranks": {"reduce_scatter_fp32": int(4 * ft5.total * 7 / 8),
                                            "all_gather_fp16": int(2 * ft5.total * 7 / 8)}}
        del ft5, m5
        grad_bytes = 2 * ft.total  # the flat fp16 gradient = the fp16 forward copy
        truck_bytes = 2 * _flat_total(22)
        W = 8
        headline_ms = headline["ms_per_step"]
        budget = W * headline_ms / 6.0  # per-rank step time that still gives 6x at 8 ranks
        out = {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "graphs": used_graph,
               "whole_step_graph": whole_captured, "graph_steps": graph_steps,
               "ms_per_step": round(ms, 4), "rays_per_s": round(args.num_rays / (ms * 1e-3), 1),
               "three_graphs": three, "sparse_exchange": sparse, "exact_reduce": exact,
               "phases_ms": {k: round(v, 5) for k, v in phases.items()},
               "flat_grad_bytes": int(grad_bytes),
               "per_rank_bytes_8_ranks": {
                   "config4_lego": {"reduce_scatter": int(grad_bytes * (W - 1) / W),
                                    "all_gather": int(grad_bytes * (W - 1) / W)},
                   "config5_truck": {"flat_grad_bytes": int(truck_bytes),
                                     "reduce_scatter": int(truck_bytes * (W - 1) / W),
                                     "all_gather": int(truck_bytes * (W - 1) / W)}},
               "scaling_budget_8_ranks": {"per_rank_ms_for_6x": round(budget, 4),
                                          "compute_ms_world1_dp_path": round(ms, 4),
                                          "exposed_collective_ms_allowed": round(budget - ms, 4)}}
        # the same step at 8 ranks without its collectives: world 1's collectives are
        # RCCL's local copies (dropped) and its Adam sweeps 8 shards (7/8 dropped)
        ph = out["phases_ms"]
        coll = ph.get("reduce_scatter", 0.0) + ph.get("all_gather", 0.0)
        est = ms - coll - ph.get("optimizer", 0.0) * (W - 1) / W
        out["scaling_budget_8_ranks"].update(
            compute_ms_8_ranks_est=round(est, 4), exposed_collective_ms_allowed_8_ranks=round(budget - est, 4),
            estimate="graph ms/step - world-1 reduce_scatter/all_gather phases - 7/8 of the optimizer phase")
        del ft, m2
        torch.cuda.empty_cache()
        return out
    finally:
        dist.destroy_process_group()


def _flat_total(log2T):
    """Length of the flat parameter buffer (table + both MLPs, 8-aligned
    each) for a bound-1 model with a 2^log2T-entry hash table."""
    from gridencoder import GridEncoder
    enc = GridEncoder(input_dim=3, num_levels=16, level_dim=2, base_resolution=16, log2_hashmap_size=log2T,
                      desired_resolution=2048)
    n_tab = int(enc.offsets[-1]) * 2
    r8 = lambda n: (n + 7) // 8 * 8  # noqa: E731
    return r8(n_tab) + r8(64 * (32 + 64 + 16)) + r8(64 * (32 + 64 + 64 + 16))


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


def adam_bytes(ft, groups=None):
    """Algorithmic HBM bytes of one Adam sweep of this rank (SURVEY §8(d) and
    DESIGN.md §4): per parameter p, m, v read + write (24 B) and the fp16 grad
    read + clear (4 B); + 2 B for an fp16 forward copy where one is written (the
    MLPs; the table too when it is kept, data parallel). groups (world 1, from
    FusedTrainer.adam_groups): the sweep stores nothing for a table group it
    leaves unchanged (moments and gradient zero: 16 B / parameter, the reads)
    and does not clear a gradient group that is zero (26 B), so those bytes
    are not counted."""
    n_tab = int(ft.params[0].numel())
    n_mlp = int(sum(p.numel() for p in ft.params[1:]))
    if ft.dp:
        return int(30 * ft.chunk)
    if groups is None or not ft.table32:
        return int((28 if ft.table32 else 30) * n_tab + 30 * n_mlp)
    idle, zero_g, total = groups
    rest = n_tab - 4 * (idle + zero_g)
    return int(16 * 4 * idle + 26 * 4 * zero_g + 28 * rest + 30 * n_mlp)


def launch_bytes(ft, samples, rays, live=None, groups=None):
    """SURVEY §8(d) per-unit bytes of each launch of the world-1 step body
    (timed_body_steps names): None for the MFMA-bound MLP launches. The grid
    backward's 1,100 B are per LIVE sample when the backwards walk only the
    rows with a nonzero gradient (options live_rows; `live` = their count)."""
    march = 48 * rays + 32 * samples
    out = {"march_rays_train+adam": adam_bytes(ft, groups) + march, "march_rays_train": march,
           "step_head": None, "grid_encode_forward": 588 * samples, "grid_encode_backward": 1100 * (samples if live is None else live),
           "composite_loss": (32 + 52) * rays + (24 + 40) * samples, "ffmlp_forward": None, "ffmlp_backward": None}
    return out


def make_trainer(args, model, data, world, dev, dt_gamma, grid_timing=True, distributed=None, options=None):
    """A FusedTrainer with its sample buffer sized as upstream sizes it
    (mean_count = measured counts x 1.25, update_extra_state)."""
    from nerf.fused import FusedTrainer
    dp = world > 1 if distributed is None else distributed
    probe = FusedTrainer(model, data, M=args.num_rays * 64, distributed=dp, dt_gamma=dt_gamma, options=options)
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
    ft = FusedTrainer(model, data, M=mean_count, distributed=dp, dt_gamma=dt_gamma, grid_timing=grid_timing,
                      options=options)
    return ft, mean_count


def timed_run(args, ft, world, dev, steps, warmup, settle, graph_steps):
    """Warm up, capture, settle the clocks, then time exactly `steps` complete
    steps between barriers + synchronize (max over ranks). Returns (elapsed s,
    used_graph, the grid backward's own clock over the timed steps)."""
    for _ in range(max(1, warmup)):
        ft.step()
    used_graph = False
    if args.graph:
        try:
            ft.capture(multi=graph_steps if (not ft.dp or ft._dp_graph) else 1)
            ft.run(3 * max(1, graph_steps))
            used_graph = True
        except Exception as e:  # eager launches are the same kernels; record why
            print(f"[bench] graph capture failed, running eager: {e!r}", file=sys.stderr)
            ft.graph = None
    torch.cuda.synchronize()
    # clock settle: the GPU raises its clocks only under sustained load. A
    # 20-step run right after 5 warmup steps measured 15.0M rays/s against
    # 17.3M for 200 steps on the same box (profiles/r02zl_settle.txt), so a
    # fixed number of untimed steps (same on every rank: they hold
    # collectives) runs before the timed region.
    for i in range(0, settle, 64):
        if ft.xchg and i > 0 and i + 64 >= settle:
            # the lists are fitted on a trailing window: the statistics restart
            # before the last settle block, so the early-training peak (12x
            # the steady longest list in round 5) does not size them
            ft._xchg.reset_stats()
        ft.run(min(64, settle - i))
        torch.cuda.synchronize()
    if ft.xchg:
        # the replicated step's touched-entry lists sized for the steady regime
        # (2 x the longest list of the trailing settle block; graphs captured again)
        ft.xchg_fit_peak = int(ft._xchg.stats[1])
        ft.fit_exchange(2.0)
        ft.run(max(2, graph_steps))
    torch.cuda.synchronize()
    # ---------------- timed region ----------------
    if world > 1:
        dist.barrier()
    ft.grid_timing_reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ft.run(steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # a bounded cross-workgroup wait of the in-launch emit that ran out would
    # have made some step's sample offsets wrong: such a run is not a result
    err = ft.device_errors()
    if err:
        raise RuntimeError(f"march emit wait timed out during the run (error word {err:#x})")
    if ft.exchange_overflows:  # a skipped update is work not done: not a result either
        raise RuntimeError(f"{ft.exchange_overflows} steps skipped on a gradient-exchange list overflow")
    grid_clock = ft.grid_timing(last=steps)  # the timed region's grid backwards (<= 256 of them)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, used_graph, grid_clock


def grid_roofline(grid_clock, steps, workload, all_samples=None):
    """The grid backward (bin + accumulate) on its own clock over the timed
    region's graph replays: 1,100 B per sample x the samples of
    exactly those launches / their summed spans (NGP_GRID_TIMING). north_star's
    grid_encode target is read against this figure."""
    if not grid_clock or grid_clock[0] != steps:
        return None
    _, ms, samp = grid_clock
    calls = len(ms)
    achieved = 1100 * sum(samp) / (sum(ms) * 1e-3) / 1e9
    traffic, src = pmc_traffic("grid_encode_backward", workload)
    out = {"kernel": "grid_encode_backward", "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": src,
           "algorithmic_bytes_per_launch": int(1100 * sum(samp) / calls), "timing": "device_clock_timed_region",
           "launches_timed": calls, "samples_timed": int(sum(samp)), "avg_launch_ms": round(sum(ms) / calls, 5),
           "launch_ms_min_median_max": [round(float(v), 5) for v in (min(ms), np.median(ms), max(ms))]}
    if all_samples:
        # the backward walks only the live rows (options live_rows): samples_timed
        # counts those, the bytes above are theirs. Beside it, the reference's
        # work (its backward reads every sample's gradient) over the same time:
        # an equivalent rate, not bytes this kernel moved
        eq = 1100 * all_samples * calls / (sum(ms) * 1e-3) / 1e9
        out["rows"] = "live (a nonzero gradient)"
        out["all_samples_per_launch"] = int(all_samples)
        out["reference_equivalent_frac"] = round(eq / HBM_PEAK_GBS, 4)
    return out


def launch_roofline(ft, kernel_ms, per_step, counts, rays, workload, live=None, groups=None):
    """The step's longest launch (over all launches of the body, timed with
    HIP events between the launches of eager body steps on the launch stream,
    the sample counts of those same steps): its algorithmic bytes (SURVEY
    §8(d)) over its mean duration. World 1 that is the march launch carrying
    the previous step's Adam; `adam_bytes_frac` is Adam's share of its bytes."""
    S = float(np.mean(counts))
    nbytes = launch_bytes(ft, S, rays, live, groups)
    dom = max(kernel_ms, key=lambda k: kernel_ms[k])
    out = {"kernel": dom, "timing": "eager_body_events", "launches_timed": len(per_step[dom]),
           "avg_launch_ms": round(kernel_ms[dom], 5),
           "share_of_launch_time": round(kernel_ms[dom] / sum(kernel_ms.values()), 4)}
    if nbytes.get(dom) is None:  # an MLP launch: MFMA-bound
        # forward 36,864 FLOP / sample, backward twice that per live sample
        flops = 36864 * S if "forward" in dom else 73728 * (S if live is None else live)
        ach = flops / (kernel_ms[dom] * 1e-3) / 1e12
        out.update(bound="mfma", achieved=round(ach, 2), peak=FP16_MFMA_PEAK_TFLOPS, unit="TFLOP/s",
                   frac=round(ach / FP16_MFMA_PEAK_TFLOPS, 4), traffic=None)
        return out
    b = nbytes[dom]
    ach = b / (kernel_ms[dom] * 1e-3) / 1e9
    traffic, src = pmc_traffic(dom, workload)
    out.update(bound="hbm", achieved=round(ach, 1), peak=HBM_PEAK_GBS, unit="GB/s", frac=round(ach / HBM_PEAK_GBS, 4),
               traffic=traffic, traffic_source=src, algorithmic_bytes_per_launch=int(b))
    if dom == "march_rays_train+adam":
        ab = b - (48 * rays + 32 * S)
        out["adam_bytes"] = int(ab)
        out["adam_bytes_frac"] = round(ab / b, 4)
        if groups is not None:  # the table's 4-parameter groups Adam leaves / does not clear
            out["adam_table_groups"] = {"unchanged": groups[0], "grad_zero": groups[1], "total": groups[2]}
    out["per_launch_ms"] = {k: round(v, 5) for k, v in kernel_ms.items()}
    out["per_launch_frac"] = {k: round(nbytes[k] / (v * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                              for k, v in kernel_ms.items() if nbytes.get(k)}
    return out


def run_fused(args, model, data, bits, world, dev):
    opts = dict(sparse_exchange=True) if args.exchange == "sparse" else None
    ft, mean_count = make_trainer(args, model, data, world, dev, args.dt_gamma, options=opts)
    elapsed, used_graph, grid_clock = timed_run(args, ft, world, dev, args.steps, args.warmup, args.settle_steps,
                                                args.graph_steps)
    ms_per_step = elapsed / args.steps * 1e3
    value = args.num_rays * world * args.steps / elapsed
    samples = model.step_counter[:, 0].float()
    samples_per_step = int(samples[samples > 0].mean().item()) if (samples > 0).any() else 0
    loss = ft.last_loss

    # ---------------- per-launch device time (roofline) ----------------
    groups = None
    if world == 1:
        kernel_ms, per_step, counts = ft.timed_body_steps(args.kernel_steps)
        groups = ft.adam_groups()  # the pending update's (the last timed body step's gradient)
    else:
        ft.flush()
        kernel_ms, per_step, counts = ft.timed_steps(args.kernel_steps, with_counts=True)
    counts = [min(int(c), ft.M) for c in counts]
    rows = float(np.mean(counts))
    # the rows the backwards walk (options live_rows: those with a nonzero gradient)
    lc = getattr(ft, "body_live_counts", None) if world == 1 else None
    live = float(np.mean(lc)) if lc else None
    grid = grid_roofline(grid_clock, args.steps, args.workload,
                         samples_per_step if getattr(ft, "_live", False) else None)
    if world == 1:
        roofline = launch_roofline(ft, kernel_ms, per_step, counts, args.num_rays, args.workload, live, groups)
    else:  # the data-parallel step's phases include collectives: the grid backward names the roofline
        roofline = grid
    mlp_ms = sum(v for k, v in kernel_ms.items() if k.startswith("ffmlp"))
    ffmlp_flops = 36864 * rows + 73728 * (rows if live is None else live)
    step_bytes = whole_step_bytes(rows, args.num_rays, sum(p.numel() for p in model.parameters()),
                                  int(model.encoder.embeddings.numel()), live)

    density = density_update_times(model, bits, ft)
    cadence = density_cadence(ft, bits, args) if world == 1 else None

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
        "roofline": roofline,
        # north_star's grid_encode target, on the grid backward's own clock
        "roofline_grid_encode": grid,
        "kernels_ms": {k: round(v, 5) for k, v in kernel_ms.items()},
        "kernel_samples": counts,
        "kernel_live_rows": lc or None,
        "ffmlp_mfma": {"flops_per_step": int(ffmlp_flops), "ms": round(mlp_ms, 5),
                        "tflops": round(ffmlp_flops / (mlp_ms * 1e-3) / 1e12, 2) if mlp_ms > 0 else None,
                        "peak_tflops": FP16_MFMA_PEAK_TFLOPS},
        # SURVEY §8(d)'s secondary figure: the step's algorithmic bytes over the
        # whole step time (per rank) against the HBM peak
        "step_roofline": {"algorithmic_bytes": int(step_bytes),
                          "frac": round(step_bytes / (ms_per_step * 1e-3) / (HBM_PEAK_GBS * 1e9), 4)},
        "density_update_ms": density,
        # beside the headline (which SURVEY §8(d) defines without it): upstream's
        # density-grid cadence timed end to end, one partial update per 16 steps
        "with_density_update": cadence,
        "loss": loss,
    }, ft


def density_cadence(ft, bits, args, cycles=6, every=16):
    """The training loop at upstream's density cadence (update_extra_interval
    = 16, nerf/utils.py), timed end to end: `cycles` x [update_density()
    (partial, device draws; it flushes the pending Adam first), restore the
    benched bitfield fixture (a device copy + the occupancy image rebuild, so
    the steps march the same workload as the headline), run(16) (the first
    step after the flush from its own graph, then the multi-step graph)],
    after one untimed cycle."""
    model = ft.model
    grid0 = model.density_grid.clone()
    it0 = model.iter_density
    model.iter_density = 16  # partial updates, as upstream after the first 16
    ft.run(every)
    # one untimed cycle first: the first call of a code path pays one-time host
    # costs (buffer allocation, first launches: ~100 ms in tools/cadence_probe2.py)
    ft.update_density()
    model.density_bitfield.copy_(bits)
    ft.refresh_occupancy()
    ft.run(every)
    torch.cuda.synchronize()
    eager0 = ft.eager_steps
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(cycles + 1)]
    host = []
    t0 = time.perf_counter()
    for c in range(cycles):
        evs[c].record()
        ft.update_density()
        model.density_bitfield.copy_(bits)
        ft.refresh_occupancy()
        ft.run(every)
        host.append(time.perf_counter())
    evs[cycles].record()
    torch.cuda.synchronize()
    secs = time.perf_counter() - t0
    gpu_cycle = [evs[c].elapsed_time(evs[c + 1]) for c in range(cycles)]
    host_cycle = [(b - a) * 1e3 for a, b in zip([t0] + host[:-1], host)]
    eager = ft.eager_steps - eager0
    # the same cycles again, synchronised after each part (where the time goes)
    parts = {"update_density": 0.0, "restore": 0.0, "run": 0.0}

    def part(name, fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        parts[name] += (time.perf_counter() - t) * 1e3 / cycles

    for _ in range(cycles):
        part("update_density", ft.update_density)
        part("restore", lambda: (model.density_bitfield.copy_(bits), ft.refresh_occupancy()))
        part("run", lambda: ft.run(every))
    model.density_grid.copy_(grid0)
    model.iter_density = it0
    model.density_bitfield.copy_(bits)
    ft.refresh_occupancy()
    ms = secs * 1e3 / (cycles * every)
    return {"ms_per_step": round(ms, 4), "rays_per_s": round(args.num_rays / (ms * 1e-3), 1),
            "timing": f"{cycles} x [partial update_density + bitfield fixture restore + run({every})], wall",
            "eager_steps": int(eager), "parts_ms_per_cycle_synced": {k: round(v, 4) for k, v in parts.items()},
            "cycle_ms_gpu_events": [round(v, 3) for v in gpu_cycle],
            "cycle_ms_host_enqueue": [round(v, 3) for v in host_cycle]}


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
                # the step's forward carries the tail (k_grid_fwd_tail); k_grid_fwd_pair
                # also counts the density update's 2M-point queries
                "grid_encode_forward": ("k_grid_fwd_tail",),
                "march_rays_train+adam": ("void k_march_train<4u>", "k_march_emit")}


def whole_step_bytes(samples, rays, n_params, n_table, live=None):
    """Algorithmic HBM bytes of one step per SURVEY §8(d): grid forward 588 B and
    backward 1,100 B per sample (+ the fp16 table grad's zero fill, 2 B per table
    value), march 48 B/ray + 32 B/sample, composite forward 32 B/ray + 24
    B/sample and backward 52 B/ray + 40 B/sample, SH 76 B/direction, dense Adam
    28 B/parameter. The backward's bytes are per live sample when the
    backwards walk only those (`live`, options live_rows)."""
    return (588 * samples + 1100 * (samples if live is None else live) + 2 * n_table + 48 * rays + 32 * samples + 32 * rays + 24 * samples
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

"""Fused instant-ngp train step: one training iteration of the reference
(nerf/utils.py Trainer.train_step :453-497 + optimizer/scaler/scheduler
:194-217, 574-609) as ~22 kernel launches through the C ABI, no autograd.

The autograd path (nerf.train.Trainer + the gridencoder/raymarching/
shencoder/ffmlp Functions) is the reference's op-level API and stays the
parity anchor; this engine computes the same iteration with the elementwise
glue fused into the hot-path kernels (DESIGN.md "fused step"):

    lego_rays -> march_rays_train -> grid_encode(fused) -> sigma FFMLP
    -> glue(trunc_exp, SH, cat) -> color FFMLP -> composite+loss+backward
    -> color FFMLP backward -> glue backward -> sigma FFMLP backward
    -> grid_encode backward(fused) -> GradScaler check + Adam + update

Static shapes: N rays per step, M = the sample buffer (mean_count); rows past
the marcher's sample count are skipped on the device, so a fixed M costs
nothing beyond its memory. Every launch goes to the current stream, so the
whole step captures into one hipGraph (`capture`).

Step order: `step()` runs [optimizer of the PREVIOUS step's gradients ->
sample -> march -> network], so one graph holds a whole step. Data parallel
(world > 1, ZeRO-1): [optimizer of this rank's shard] -> all-gather of the
fp16 forward copy, overlapped with [sample -> march] -> [network] -> guard +
averaging reduce-scatter of the gradient, captured as one graph over RCCL
(the all-gather on RCCL's stream beside sample + march); with gloo or
options dp_graph=False the collectives sit between three graphs. The arithmetic is the reference's, in the
reference's order; only the last step's update stays pending until
`flush()` (the read-outs below flush first). Running that optimizer on a side
stream beside sample + march was measured and lost: Adam and the marcher's
scan/emit are both memory-bound and slowed each other more than they
overlapped (profiles/r01u_overlap_trace.txt).
"""
import ctypes
import sys

import numpy as np
import torch
import torch.distributed as dist

import _ngp_native as nat

from .provider import LEGO_BOXES, LEGO_COLORS
from .exchange import SparseExchange
from .zero1 import ShardPlan

_F16 = nat.DTYPE_CODE[torch.float16]
_F32 = nat.DTYPE_CODE[torch.float32]
_RELU, _NONE = 0, 6
_DEFER, _GEO, _PAIR = 1, 2, 4  # NGP_FFMLP_DEFER_REDUCE, NGP_FFMLP_NERF_GEO, NGP_FFMLP_PAIR_MAJOR
_SCAN, _PRECHECKED = 1, 2  # NGP_SCALER_SCAN, NGP_SCALER_PRECHECKED
_ZEROED, _EXTERNAL = 0x10, 0x20  # NGP_GRID_GRAD_ZEROED, NGP_GRID_CURSORS_EXTERNAL (grad layout 0: [L,M,2])
_TIMING = 0x40  # NGP_GRID_TIMING
_SHADOW_ALL = 2  # NGP_ADAM_SHADOW_ALL (zero_grads bit 1)


def _vp_array(ptrs):
    return (ctypes.c_void_p * len(ptrs))(*ptrs)


# The step's structure. Every option defaults to the measured-fastest form
# (DESIGN.md section 1); the alternatives remain because a configuration needs
# them (the data-parallel step, shapes the one-launch kernels do not cover) or
# as the reference forms the equivalence tests compare against, selected per
# trainer with `options=`:
#   table16       world 1: keep an fp16 copy of the table for the grid forward
#                 (default: the forward reads the fp32 table, rounding on load)
#   split_head    world 1: the step head (Adam + batch) as its own launch
#   split_reduce  the MLP dW slab reduce in its own launch
#   split_fwd     the sigma and colour MLP forwards as two launches
#   split_bwd     the two MLP backwards as two launches
#   march_adam    world 1: the pending Adam rides in the march launch
#   tail_in_fwd   the bookkeeping + MLP packs ride in the grid forward's launch
#   emit_inline   the march launch emits its samples itself (no emit launch)
#   draw_ahead    the next batch is drawn in the grid backward's bin launch
#   live_rows     the backwards walk the rows with a nonzero gradient only
#   dp_graph      data parallel over RCCL: the whole step is one graph
#   density_sort  partial density updates draw their cells as order statistics, in
#                 Morton order (False: the counter-RNG draws in draw order)
#   sparse_exchange  data parallel: every rank runs the world-1 step with the
#                 full Adam, the gradients meet in a touched-entry exchange
#                 (nerf/exchange.py) instead of the ZeRO-1 collectives
#   exact_reduce  ZeRO-1: reduce-scatter the gradient in fp32 (SUM, then / world
#                 and one fp16 rounding into the shard), the arithmetic of the
#                 reference's DDP all-reduce of fp32 grads (nerf/utils.py:325-327),
#                 at twice the reduce-scatter's link bytes; default: an fp16 AVG
#                 reduce-scatter, which rounds at every ring hop
DEFAULT_OPTIONS = dict(table16=False, split_head=False, split_reduce=False, split_fwd=False, split_bwd=False,
                       march_adam=True, tail_in_fwd=True, emit_inline=True, draw_ahead=True, live_rows=True,
                       dp_graph=True, density_sort=True, sparse_exchange=False, exact_reduce=False,
                       density_run_max=False)


class FusedTrainer:
    def __init__(self, model, dataset, M, lr=1e-2, iters=30000, max_steps=1024, T_thresh=1e-4,
                 dt_gamma=0.0, seed=0, betas=(0.9, 0.99), eps=1e-15, init_scale=65536.0,
                 growth_interval=2000, distributed=False, grid_timing=False, options=None):
        """distributed: ray-sharded data parallelism over the initialised
        torch.distributed group: each rank draws its own rays; the flat fp16
        gradient is averaged with one RCCL reduce-scatter, each rank's Adam
        updates its 1/world shard and the fp16 forward copy is all-gathered
        (ZeRO-1; see `_reduce`).
        grid_timing: the binned grid backward times itself on the chip's
        constant clock (`grid_timing()`, the bench's roofline clock); off by
        default, since it adds ring stores to the backward's launches.
        options: DEFAULT_OPTIONS overrides (the step's structure)."""
        opts = dict(DEFAULT_OPTIONS)
        for k, v in (options or {}).items():
            if k not in opts:
                raise ValueError(f"FusedTrainer: unknown option {k!r} (known: {sorted(opts)})")
            opts[k] = bool(v)
        self.options = opts
        assert model.cuda_ray, "the fused step marches the density bitfield (cuda_ray=True)"
        enc = model.encoder
        assert enc.level_dim == 2 and enc.num_levels * enc.level_dim == 32 and enc.input_dim == 3
        assert model.sigma_net.input_dim == 32 and model.color_net.input_dim == 32
        self.model, self.data = model, dataset
        dev = model.density_bitfield.device
        self.dev = dev
        self.N = N = int(dataset.num_rays)
        self.M = M = int(M)
        self.max_steps, self.T_thresh, self.dt_gamma = int(max_steps), float(T_thresh), float(dt_gamma)
        self.lr, self.iters, self.betas, self.eps = float(lr), int(iters), betas, float(eps)
        self.growth_interval, self.seed = int(growth_interval), int(seed)
        self.density_seed = int(seed)  # the density-grid draws are the same on every rank
        # dp: the data-parallel (ZeRO-1) step with its collectives, also at
        # world size 1 (a one-rank group runs the same RCCL calls);
        # sparse_exchange: the world-1 step on every rank + the exchange (xchg)
        self._dist = bool(distributed and dist.is_initialized())
        self.xchg = self._dist and opts["sparse_exchange"]
        self.dp = self._dist and not self.xchg
        self.world = dist.get_world_size() if self._dist else 1
        if self.world > 1:
            self.seed += 7919 * dist.get_rank()
        self.enc = enc
        self.S = float(np.log2(enc.per_level_scale))
        self.sig_net, self.col_net = model.sigma_net, model.color_net

        def z(*shape, dtype=torch.float32):
            return torch.zeros(*shape, dtype=dtype, device=dev)

        # per-ray and per-sample buffers
        self.rays_o, self.rays_d = z(N, 3), z(N, 3)
        self.rgba, self.bg = z(N, 4), z(N, 3)
        self.nears, self.fars, self.noises = z(N), z(N), z(N)
        self.loss_ray = z(N)
        self.counter = z(2, dtype=torch.int32)
        self.rays = z(N, 3, dtype=torch.int32)
        self.xyzs, self.dirs, self.deltas = z(M, 3), z(M, 3), z(M, 2)
        ws = nat.lib().ngp_march_rays_train_workspace_bytes(N, self.max_steps, model.cascade, model.grid_size)
        self.march_ws = z(ws, dtype=torch.uint8)
        self.refresh_occupancy()
        h = torch.float16
        # enc_out / g_enc are [L=16][M][2] (the grid's level-major layout; the
        # sigma network reads / writes them pair-major): every grid kernel then
        # moves whole lines per level
        self.enc_out, self.h_sigma = z(M, 32, dtype=h), z(M, 16, dtype=h)
        self.sigma, self.color_in, self.color_out = z(M), z(M, 32, dtype=h), z(M, 16, dtype=h)
        self.g_color_out, self.g_h = z(M, 16, dtype=h), z(M, 16, dtype=h)
        self.g_enc = z(M, 32, dtype=h)
        # parameters: fp32 masters, fp16 grads and fp16 forward copies, each one
        # flat buffer with the same 8-aligned layout (tensor k at starts[k]):
        # the optimizer is one elementwise sweep over [lo, hi) of it, and a
        # data-parallel step moves the gradient and the forward copy with one
        # collective each
        self.params = [enc.embeddings, self.sig_net.weights, self.col_net.weights]
        sizes = [p.numel() for p in self.params]
        self.rank = dist.get_rank() if self._dist else 0
        # ZeRO-1 layout (nerf/zero1.py): 8-aligned tensors, a 64-aligned chunk
        # per rank (sparse_exchange: every rank owns everything)
        self.plan = plan = ShardPlan(sizes, 1, 0) if self.xchg else ShardPlan(sizes, self.world, self.rank)
        starts = plan.starts + [plan.used]
        self.chunk = chunk = plan.chunk
        self.total = total = plan.total
        self.lo, self.hi = plan.lo, plan.hi
        self.flat_param = z(total)
        self.flat_grad = z(total, dtype=h)
        self.flat_half = z(total, dtype=h)
        with torch.no_grad():
            for a, p in zip(starts[:-1], self.params):  # re-home the model's parameters
                view = self.flat_param[int(a):int(a) + p.numel()].view(p.shape)
                view.copy_(p.detach())
                p.data = view
                self.flat_half[int(a):int(a) + p.numel()].copy_(view.reshape(-1))
        self._starts = [int(a) for a in starts[:-1]]
        self.grads = [self.flat_grad[int(a):int(a) + n].view(p.shape)
                      for a, n, p in zip(starts[:-1], sizes, self.params)]
        self.w_half = [self.flat_half[int(a):int(a) + n].view(p.shape)
                       for a, n, p in zip(starts[:-1], sizes, self.params)]
        # Adam moments of this rank's shard only (ZeRO-1); world 1: everything
        self.exp_avg, self.exp_avg_sq = z(chunk), z(chunk)
        # the averaged gradient shard (reduce-scatter output); world 1: the flat grad itself
        self.grad_shard = z(chunk, dtype=h) if self.dp else self.flat_grad
        # exact_reduce: the fp32 image of the flat gradient and of this rank's shard sum
        self._exact_reduce = self.dp and opts["exact_reduce"]
        self._grad32 = z(self.total) if self._exact_reduce else None
        self._shard32 = z(chunk) if self._exact_reduce else None
        self._offsets_host = (ctypes.c_int32 * enc.offsets.numel())(*enc.offsets.cpu().tolist())
        gb = nat.lib().ngp_grid_encode_backward_fused_workspace_bytes(
            M, enc.input_dim, enc.level_dim, enc.num_levels, self.S, enc.base_resolution,
            int(enc.align_corners), self._offsets_host)
        self.grid_ws = z(max(int(gb), 256), dtype=torch.uint8)  # zero-filled: bin cursors start at 0
        # the step head clears the bin cursors for the grid backward (NGP_GRID_CURSORS_EXTERNAL)
        self._grid_counter_bytes = int(nat.lib().ngp_grid_encode_backward_fused_counter_bytes(
            M, enc.input_dim, enc.level_dim, enc.num_levels, self.S, enc.base_resolution,
            int(enc.align_corners), self._offsets_host))
        self._grid_flags = _ZEROED | (_EXTERNAL if self._grid_counter_bytes else 0)
        # the binned grid backward can time itself (grid_timing; plain stores
        # into a ring in the workspace: per call its start, samples and the
        # accumulate workgroups' ends)
        self._grid_timing_at = int(nat.lib().ngp_grid_encode_backward_fused_timing_offset(
            M, enc.input_dim, enc.level_dim, enc.num_levels, self.S, enc.base_resolution,
            int(enc.align_corners), self._offsets_host))
        if not grid_timing:
            self._grid_timing_at = 0
        if self._grid_timing_at:
            self._grid_flags |= _TIMING
            self.grid_timing_reset()
        self.mlp_ws = []
        for net in (self.sig_net, self.col_net):
            b = nat.lib().ngp_ffmlp_backward_workspace_bytes(M, net.input_dim, net.padded_output_dim,
                                                             net.hidden_dim, net.num_layers)
            self.mlp_ws.append(z(b, dtype=torch.uint8))
        # weight-fragment images of both networks, packed once per step
        nets = (self.sig_net, self.col_net)
        self.mlp_img = [z(int(nat.lib().ngp_ffmlp_image_bytes(n.input_dim, n.hidden_dim, n.num_layers)),
                          dtype=torch.uint8) for n in nets]
        self._pk = dict(
            w=_vp_array([nat.ptr(t) for t in self.w_half[1:]]),
            ins=(ctypes.c_uint32 * 2)(*[n.input_dim for n in nets]),
            hid=(ctypes.c_uint32 * 2)(*[n.hidden_dim for n in nets]),
            nl=(ctypes.c_uint32 * 2)(*[n.num_layers for n in nets]),
            img=_vp_array([nat.ptr(t) for t in self.mlp_img]),
            ws=_vp_array([nat.ptr(t) for t in self.mlp_ws]),
            B=(ctypes.c_uint32 * 2)(M, M),
            gw=_vp_array([nat.ptr(g) for g in self.grads[1:]]))
        self.state = z(nat.lib().ngp_fused_state_bytes(), dtype=torch.uint8)
        nat.check(nat.lib().ngp_fused_state_init(nat.ptr(self.state), float(init_scale),
                                                 nat.stream_of(self.state)), "fused_state_init")
        # host-side constants of the synthetic scene
        boxes = [v for (lo, hi), rgb in zip(LEGO_BOXES, LEGO_COLORS) for v in (*lo, *hi, *rgb)]
        self._boxes = (ctypes.c_float * len(boxes))(*boxes)
        self._nboxes = len(LEGO_BOXES)
        self._intr = (ctypes.c_float * 4)(*[float(v) for v in dataset.intrinsics])
        self._aabb = (ctypes.c_float * 6)(*model.aabb_train.detach().cpu().tolist())
        # World 1: the grid forward reads the fp32 table and rounds each value to
        # half as it loads it (the same values autocast's cast gives), so Adam
        # does not write an fp16 copy of the table (2 of its 28 B / parameter).
        # Data parallel: the fp16 copy is what the all-gather moves.
        self.table32 = not self.dp and not opts["table16"]
        self._merge_head = not self.dp and not opts["split_head"]
        # the MLP dW reduce in the grid backward's bin launch (split_reduce: its own launch)
        self._split_reduce = opts["split_reduce"]
        # one launch for the sigma + colour forwards where ngp_nerf_forward covers
        # the shapes (split_fwd keeps two launches)
        sn_, cn_ = self.sig_net, self.col_net
        self._one_fwd = (not opts["split_fwd"] and sn_.hidden_dim == 64
                         and cn_.hidden_dim == 64 and sn_.input_dim == 32 and cn_.input_dim == 32
                         and 2 <= sn_.num_layers <= 3 and 2 <= cn_.num_layers <= 4)
        # ... and for both backwards (ngp_nerf_backward; split_bwd: two launches)
        self._one_bwd = (not opts["split_bwd"] and sn_.hidden_dim == 64
                         and cn_.hidden_dim == 64 and sn_.input_dim == 32 and cn_.input_dim == 32
                         and 2 <= sn_.num_layers <= 3 and 2 <= cn_.num_layers <= 3)
        sec = plan.sections(self.table32)  # the table, then the two MLPs
        self._opt = dict(
            params=_vp_array([nat.ptr(self.flat_param) + 4 * (self.lo + a) for a, _, _ in sec]),
            grads=_vp_array([nat.ptr(self.grad_shard) + 2 * a for a, _, _ in sec]),
            m=_vp_array([nat.ptr(self.exp_avg) + 4 * a for a, _, _ in sec]),
            v=_vp_array([nat.ptr(self.exp_avg_sq) + 4 * a for a, _, _ in sec]),
            half=_vp_array([nat.ptr(self.flat_half) + 2 * (self.lo + a) if hv else None for a, _, hv in sec]),
            sizes=(ctypes.c_uint64 * len(sec))(*[n for _, n, _ in sec]),
            n=len(sec))
        self._nccl = self._dist and dist.get_backend() == "nccl"
        # GradScaler's inf check is made by the kernels that write the grads
        # (grid backward, MLP dW reduce) into this flag: the optimizer's found-inf
        # flag (world 1) or the data-parallel guard's per-rank flag
        self._inf_flag = nat.lib().ngp_fused_inf_flag(nat.ptr(self.state), int(self.dp))
        # sparse_exchange: the averaged gradient of every rank's batch replaces
        # this rank's after each backward (the optimizer reads the flag above)
        self._xchg = SparseExchange(self.flat_grad, self._inf_flag, self.world, self._nccl) if self.xchg else None
        # World 1: the pending Adam rides in the march launch (its workgroups'
        # Adam waves stream the parameters while the march waves probe the
        # occupancy image); the step head then only draws the batch.
        # march_adam=False: Adam in the head launch, before the march.
        self._march_adam = self._merge_head and opts["march_adam"]
        if self._march_adam:
            o, job = self._opt, nat.AdamJob()
            job.n_tensors = o["n"]
            for q in range(o["n"]):
                job.params[q], job.grads[q], job.exp_avg[q] = o["params"][q], o["grads"][q], o["m"][q]
                job.exp_avg_sq[q], job.half_params[q], job.sizes[q] = o["v"][q], o["half"][q], o["sizes"][q]
            job.lr, job.beta1, job.beta2, job.eps = self.lr, self.betas[0], self.betas[1], self.eps
            job.iters, job.zero_grads, job.grad_mult = self.iters, 1, 1.0
            self._job = job
        # ... and (with the Adam sweep whole in the march launch) the march
        # launch emits its samples itself and leaves the bookkeeping + MLP packs
        # row to the grid forward's launch: no emit launch (tail_in_fwd=False:
        # the tail row in the emit launch; emit_inline=False: the emit launch)
        self._tail_in_fwd = self._march_adam and opts["tail_in_fwd"]
        if self._tail_in_fwd:
            self._job.flags |= nat.ADAM_JOB_TAIL_LATER
        if self._march_adam and not opts["emit_inline"]:
            self._job.flags |= nat.ADAM_JOB_EMIT_LAUNCH
        # ... and the next batch is drawn while this step's grid backward runs
        # (a column of the bin launch; the batch buffers are dead once the
        # composite has read its targets), so the step starts with the march:
        # no head launch. The march + Adam launch clears the bin cursors.
        # draw_ahead=False: the head launch draws the batch.
        # Data parallel too (round 5): the bin launch draws the next batch, the
        # step clears the bin cursors itself, and the deferred bookkeeping and the
        # MLP packs ride in the grid forward's launch (_dp_tail): no head launch
        # and no pack launch per step.
        self._draw_ahead = (self._march_adam or self.dp) and not self._split_reduce and opts["draw_ahead"]
        self._dp_tail = self.dp and opts["tail_in_fwd"]
        self._ahead = False  # the batch buffers hold the next step's batch
        self._pre_ahead = None  # data parallel: the batch state the "pre" graph was captured in
        if self._draw_ahead and self._march_adam:
            self._job.clear, self._job.clear_bytes = nat.ptr(self.grid_ws), self._grid_counter_bytes
        if self._draw_ahead:
            m_, d_, bj = self.model, self.data, nat.BatchJob()
            bj.poses, bj.n_poses, bj.intrinsics4 = nat.ptr(d_.poses), d_.poses.shape[0], ctypes.addressof(self._intr)
            bj.H, bj.W, bj.N = d_.H, d_.W, self.N
            bj.boxes, bj.nboxes, bj.aabb6 = ctypes.addressof(self._boxes), self._nboxes, ctypes.addressof(self._aabb)
            bj.min_near, bj.seed, bj.state = float(m_.min_near), self.seed, nat.ptr(self.state)
            bj.rays_o, bj.rays_d, bj.rgba, bj.bg = (nat.ptr(self.rays_o), nat.ptr(self.rays_d), nat.ptr(self.rgba),
                                                    nat.ptr(self.bg))
            bj.nears, bj.fars, bj.noises = nat.ptr(self.nears), nat.ptr(self.fars), nat.ptr(self.noises)
            bj.counter, bj.step_counter = nat.ptr(self.counter), nat.ptr(m_.step_counter)
            self._batch_job = bj
        # the backwards over the live rows only (live_rows, default on): rows whose
        # gradient the composite left zero in every component (behind a ray's
        # early termination, or underflowed to zero in fp16) are skipped by the
        # MLP and grid backwards, as instant-ngp compacts its samples before
        # the backward; needs the one-launch MLP backward and the draw-ahead
        # bin launch (where the list is consumed)
        self._live = opts["live_rows"] and self._one_bwd and self._draw_ahead and not self._split_reduce
        if self._live:
            i32 = torch.int32
            self._live_bufs = dict(ray_rows=z(M, dtype=i32), cnt=z(N, dtype=i32), rows=z(M, dtype=i32),
                                   total=z(4, dtype=i32))
        self.graph = None
        self.graph_multi, self._multi = None, 1  # capture(multi=S): S step bodies in one graph
        # data parallel over RCCL: the whole step is captured, collectives included
        # (dp_graph=False: three graphs with the collectives between them)
        self._dp_graph = self.dp and opts["dp_graph"]
        self._dp_whole = None
        self._fresh = None  # world 1: graph of the first step after a flush (capture)
        self.eager_steps = 0  # world 1: steps run as eager launches (not graph replays)
        self._ring, self._ring_i = [], 0  # timing graphs (capture(ring=R))
        self._events, self._capturing = None, False
        self._dens = None  # density-grid update buffers (update_density)
        # partial updates draw their random cells in Morton order (density_sort=False: the
        # counter-RNG draws in draw order, as ngp_density_grid_draw makes them)
        self._dens_sorted = opts["density_sort"]
        self._pending = False  # gradients of the last forward/backward not yet applied

    def sync_half(self):
        """Refresh the fp16 forward copies after the fp32 parameters were
        changed outside the fused optimizer (loading, manual edits)."""
        with torch.no_grad():
            for h, p in zip(self.w_half, self.params):
                h.copy_(p)

    def refresh_occupancy(self):
        """Rebuild the marcher's occupancy image after density_bitfield changed
        (model.update_extra_state); the captured step reuses it."""
        m = self.model
        nat.check(nat.lib().ngp_march_occupancy_build(
            nat.ptr(m.density_bitfield), m.cascade, m.grid_size, self.N, self.max_steps,
            nat.ptr(self.march_ws), self.march_ws.numel(), nat.stream_of(self.march_ws)),
            "march_occupancy_build")

    # ------------------------------------------------------ density grid
    def update_density(self, decay=0.95):
        """The density-grid update (update_extra_state, renderer.py:498-598)
        with device-side draws: no host sync, so it can run inside a training
        loop at the upstream cadence (every 16 steps). Full updates while
        iter_density < 16, then partial ones (uniform + occupied cells), as
        upstream. Data parallel: every rank draws the same cells (the draw
        seed does not depend on the rank), queries its 1/world of them, and a
        MAX all-reduce of the scratch grid gives every rank the same grid and
        bitfield. mean_density stays on the device (`mean_density`)."""
        m, lib, P_ = self.model, nat.lib(), nat.ptr
        H, C = m.grid_size, m.cascade
        H3 = H ** 3
        dev, s = self.dev, nat.stream_of(self.rays_o)
        d = self._dens
        if d is None:
            wsb = int(lib.ngp_density_grid_draw_workspace_bytes(C, H))
            d = self._dens = dict(
                coords=torch.zeros(C * H3 // 2, 3, dtype=torch.int32, device=dev),
                noise=torch.zeros(C * H3, 3, device=dev),
                xyzs=torch.zeros(C * H3, 3, device=dev),
                idx=torch.zeros(C * H3, dtype=torch.int32, device=dev),
                enc=torch.zeros(self.enc.num_levels, C * H3 // self.world + 1, 2, dtype=torch.float16, device=dev),
                tmp=torch.full((C, H3), -1.0, device=dev),
                stats=torch.zeros(nat.DENSITY_STATS_LEN, dtype=torch.float64, device=dev),
                ws=torch.zeros(max(wsb, 256), dtype=torch.uint8, device=dev),
                ostat_ws=torch.zeros(max(int(lib.ngp_density_grid_ostat_workspace_bytes(C, H)), 256),
                                     dtype=torch.uint8, device=dev),
                table=torch.zeros_like(self.params[0], dtype=torch.float16) if self.table32 else None,
                mean_count=torch.zeros(1, dtype=torch.int64, device=dev),
                sigma=torch.zeros(C * H3 // 2 // self.world + 1, device=dev))
        # the pending optimizer update first (the query reads the parameters);
        # its sweep writes the query's fp16 table copy as well
        fresh_table = d["table"] is not None and self._pending and not self.dp
        # world 1: the update's bookkeeping rides in the query's grid-forward
        # launch below (one block, beside the MLP fragment packs), not in a
        # launch of its own after the sweep
        self.flush(table_half=d["table"] if fresh_table else None, defer_end=not self.dp)
        partial = int(m.iter_density >= 16)
        ppc = 2 * (H3 // 4) if partial else H3
        P = C * ppc
        lo, hi = self.rank * P // self.world, (self.rank + 1) * P // self.world
        lo0, e, n = lo, self.enc, hi - lo
        sorted_ = bool(partial and self._dens_sorted and H & (H - 1) == 0)
        if sorted_:
            # this rank's slice of the draws, generated in Morton order (the
            # same i.i.d. draws as order statistics), at the head of xyzs / idx
            nat.check(lib.ngp_density_grid_draw_sorted(P_(m.density_grid), C, H, self.density_seed, m.iter_density,
                                                       float(m.bound), lo, hi, P_(d["ws"]), d["ws"].numel(),
                                                       P_(d["ostat_ws"]), d["ostat_ws"].numel(), P_(d["xyzs"]),
                                                       P_(d["idx"]), s), "density_grid_draw_sorted")
            lo = 0
        else:
            nat.check(lib.ngp_density_grid_draw(P_(m.density_grid), C, H, partial, self.density_seed,
                                                m.iter_density, P_(d["coords"]), P_(d["noise"]), P_(d["ws"]),
                                                d["ws"].numel(), s), "density_grid_draw")
            nat.check(lib.ngp_density_grid_points(P_(d["coords"]) if partial else None, P_(d["noise"]), P, ppc, C,
                                                  H, float(m.bound), P_(d["xyzs"]), P_(d["idx"]), s),
                      "density_grid_points")
        if d["table"] is not None and not fresh_table:  # world 1 keeps no fp16 table copy: make one for the query
            d["table"].copy_(self.params[0].detach())
        table = d["table"] if d["table"] is not None else self.w_half[0]
        # the encodings are [L][n][2] (pair-major, row stride n) at the buffer's
        # head; the same launch packs the fragment images of the weights the
        # flush left (the next step packs them again from the same weights)
        # and, world 1, runs the flush's deferred bookkeeping (end_pending)
        sn, pk = self.sig_net, self._pk
        nat.check(lib.ngp_grid_encode_forward_fused_tail(
            P_(d["xyzs"]) + 12 * lo, float(m.bound), P_(table), _F16, P_(e.offsets), P_(d["enc"]), n, None,
            e.input_dim, e.level_dim, e.num_levels, self.S, e.base_resolution, e.gridtype_id, int(e.align_corners),
            e.interp_id, None if self.dp else P_(self.state), 2.0, 0.5, self.growth_interval, _PRECHECKED,
            P_(self.loss_ray), self.N, 2, pk["w"], pk["ins"], pk["hid"], pk["nl"], pk["img"], s),
            "grid_encode_forward_fused_tail")
        dens = (P_(d["enc"]), P_(self.mlp_img[0]), n, sn.hidden_dim, sn.num_layers, float(m.density_scale))
        if sorted_ and self.options["density_run_max"]:
            # densities per point, then each run of one cell's draws -> its max (no global atomics)
            nat.check(lib.ngp_nerf_density_forward_rows(*dens, P_(d["sigma"]), s), "nerf_density_forward_rows")
            nat.check(lib.ngp_density_grid_run_max(P_(d["sigma"]), P_(d["idx"]), C, H, lo0, hi, P_(d["tmp"]), s),
                      "density_grid_run_max")
        elif sorted_:
            # an integer atomic max per point from the MLP's epilogue (the draws at
            # lo = 0): the epilogue's atomics cost the query ~4 us, the run-max
            # launch 14 (partial update 0.428 -> 0.415 ms wall, r07zd)
            nat.check(lib.ngp_nerf_density_forward(P_(d["enc"]), P_(self.w_half[1]), P_(self.mlp_img[0]), n,
                                                   sn.input_dim, sn.hidden_dim, sn.num_layers, float(m.density_scale),
                                                   P_(d["idx"]), P_(d["tmp"]), s), "nerf_density_forward")
        elif not partial and H & (H - 1) == 0:
            # the full update's point p is cell p (Morton order): densities straight into tmp_grid
            nat.check(lib.ngp_nerf_density_forward_rows(*dens, P_(d["tmp"]) + 4 * lo, s), "nerf_density_forward_rows")
        else:
            nat.check(lib.ngp_nerf_density_forward(P_(d["enc"]), P_(self.w_half[1]), P_(self.mlp_img[0]), n,
                                                   sn.input_dim, sn.hidden_dim, sn.num_layers, float(m.density_scale),
                                                   P_(d["idx"]) + 4 * lo, P_(d["tmp"]), s), "nerf_density_forward")
        if self._dist:
            if self._nccl:
                dist.all_reduce(d["tmp"], op=dist.ReduceOp.MAX)
            else:
                host = d["tmp"].cpu()
                dist.all_reduce(host, op=dist.ReduceOp.MAX)
                d["tmp"].copy_(host)
        nat.check(lib.ngp_density_grid_ema_pack(P_(m.density_grid), P_(d["tmp"]), C, H, float(decay),
                                                float(m.density_thresh), P_(d["stats"]), P_(m.density_bitfield), s),
                  "density_grid_ema_pack")
        m.iter_density += 1
        self.refresh_occupancy()
        # the reference's bookkeeping after an update (renderer.py:584, 593-596),
        # kept on the device (no host sync) and resolved on read: mean_density
        # from the update's stats, mean_count from the last min(16, local_step)
        # batches' sample counts, then local_step = 0
        self._mean_density_pending = True
        total = min(16, int(m.local_step))
        if total > 0:
            self._mean_count_pending = self._recent_count_mean(total)
        m.local_step = 0

    def _recent_count_mean(self, total):
        """int(mean) of the sample counts of the last `total` batches, as a
        device scalar (no host sync): one launch (ngp_density_mean_count)
        instead of the gather's small torch ops."""
        out = self._dens["mean_count"]
        nat.check(nat.lib().ngp_density_mean_count(
            nat.ptr(self.model.step_counter), nat.ptr(self.state) + 4 * self._S_DRAW, nat.ptr(self.counter), total,
            int(self._ahead), nat.ptr(out), nat.stream_of(out)), "density_mean_count")
        return out

    @property
    def mean_density(self):
        """model.mean_density, after the last update_density's value
        (torch.mean(...).item(), :584) has been read back from the device."""
        if getattr(self, "_mean_density_pending", False):
            self.model.mean_density = float(np.float32(self._dens["stats"][0].item() / self.model.density_grid.numel()))
            self._mean_density_pending = False
        return float(self.model.mean_density)

    @property
    def mean_count(self):
        """model.mean_count, after the last update_density's value (:593-595)."""
        mc = getattr(self, "_mean_count_pending", None)
        if mc is not None:
            self.model.mean_count = int(mc.item())
            self._mean_count_pending = None
        return int(self.model.mean_count)

    # ------------------------------------------------------------------ step
    def _tick(self, name):
        """Event after each launch while `timed_steps` instruments eager steps
        or `capture(ring=...)` records a timing graph (inside a capture the
        event is an event-record node of the graph: `external`)."""
        if self._events is not None:
            ev = torch.cuda.Event(enable_timing=True, external=self._capturing)
            ev.record()
            self._events.append((name, ev))

    _TIMING_RING, _TIMING_MAX_WG, _TIMING_HEADS = 256, 1024, 64  # include/ngp_hip.h NGP_GRID_TIMING_*

    def _grid_timing_words(self):
        a = self._grid_timing_at
        n = self._TIMING_HEADS + 4 * self._TIMING_RING + self._TIMING_RING * self._TIMING_MAX_WG
        return self.grid_ws[a:a + 4 * n].view(torch.int32)

    def grid_timing_reset(self):
        """Restart the grid backward's self-timing ring (calls := 0)."""
        if self._grid_timing_at:
            self._grid_timing_words()[0] = 0

    def grid_timing(self, last=None):
        """Device time of the grid backward's last calls since
        grid_timing_reset() (at most 256, `last` if given): the MLP backward
        launch's end (or the bin launch's start) -> the accumulate's last
        workgroup end, measured by the kernels on the
        chip's 100 MHz constant clock, so graph replays are timed as they run
        (no events in the graphs). Returns (calls, ms per call, samples per
        call), oldest first, or None when the backward is unbinned."""
        if not self._grid_timing_at:
            return None
        torch.cuda.synchronize()
        w = self._grid_timing_words().cpu().numpy().view(np.uint32)
        R, W, H = self._TIMING_RING, self._TIMING_MAX_WG, self._TIMING_HEADS
        calls = int(w[0])
        n = min(calls, R, last or R)
        ms, samples = [], []
        for c in range(calls - n, calls):
            start, samp, nwg = (int(v) for v in w[H + 4 * (c % R):H + 4 * (c % R) + 3])
            row = w[H + 4 * R + (c % R) * W:][:W].astype(np.int64)
            ends = row[:min(nwg, W)]
            # the span starts where the previous launch (the MLP backward,
            # ngp_nerf_backward: its workgroups' ends fill the row from the
            # top) ended, when those ends are this call's (within 100 us before
            # the bin launch's first block): the bin launch's dispatch ramp
            # then counts, as in the trace's kernel times
            prev = row[max(min(nwg, W), W - W // 4):]
            d = (start - prev) & 0xffffffff
            fresh = prev[(d > 0) & (d < 10_000)]
            if fresh.size:
                start = int(fresh[((start - fresh) & 0xffffffff).argmin()])
            ms.append(float(((ends - start) & 0xffffffff).max()) * 1e-5)
            samples.append(samp)
        return calls, ms, samples

    def _recent_counts(self, n):
        """Sample counts of the last n batches (oldest first) as a device
        tensor: the newest is still in `counter`, batch `it` was recorded in
        step_counter slot it % 16 when batch it + 1 was drawn (n <= 16)."""
        assert 1 <= n <= 16
        draw = self.state.view(torch.int32)[self._S_DRAW].long()
        if self._ahead:  # the next batch is drawn: the newest count went to step_counter too
            k = torch.arange(n - 1, -1, -1, device=self.dev)
            return self.model.step_counter[(draw - 2 - k) & 15, 0].long()
        k = torch.arange(n - 1, 0, -1, device=self.dev)
        old = self.model.step_counter[(draw - 1 - k) & 15, 0].long()
        return torch.cat([old, self.counter[:1].long()])

    def ring_times(self, last=None):
        """Per-phase device time of the last replays of the timing ring
        (`capture(ring=R)`; the events are nodes of the replayed graphs, so
        these are the steps of the timed region themselves), with the sample
        count of each of those steps. Returns (per-phase mean ms, per-replay
        ms of each phase, per-replay sample counts), oldest replay first."""
        n = min(self._ring_i, len(self._ring), last or len(self._ring))
        assert n > 0, "no ring replays yet"
        torch.cuda.synchronize()
        order = [(self._ring_i - n + j) % len(self._ring) for j in range(n)]
        per = {}
        for r in order:
            ev = self._ring[r][1]
            for (_, a), (name, b) in zip(ev[:-1], ev[1:]):
                per.setdefault(name, []).append(a.elapsed_time(b))
        counts = self._recent_counts(n).cpu().tolist()
        return {k: float(np.mean(v)) for k, v in per.items()}, per, counts

    def timed_steps(self, k, with_counts=False):
        """Device time per phase (ms, mean over k eager steps), measured with
        events on the launch stream between consecutive launches: each phase's
        kernels run in the cache state of a real step (the previous step's
        optimizer has streamed the parameters through), unlike back-to-back
        repeats of one kernel. A spin kernel ahead of each step lets the host
        queue every launch first, so no phase includes host launch gaps. The
        phases run serially here (the all-gather is waited for right away).
        with_counts: also the per-step times of each phase and the steps'
        sample counts (mean, per-step, counts)."""
        self.flush()
        acc, per, counts = {}, {}, []
        for i in range(k):
            torch.cuda.synchronize()
            torch.cuda._sleep(4_000_000)  # keep the GPU busy while the host queues the step
            self._events = []
            self._tick("start")
            self._sample()
            self._march()
            self._network()
            self._reduce()
            self._optimizer(defer=i < k - 1)
            self._gather_half(wait=True)
            self.model.local_step += 1
            torch.cuda.synchronize()
            ev, self._events = self._events, None
            counts.append(self.sample_count())
            for (_, a), (name, b) in zip(ev[:-1], ev[1:]):
                acc[name] = acc.get(name, 0.0) + a.elapsed_time(b)
                per.setdefault(name, []).append(a.elapsed_time(b))
        mean = {n: v / k for n, v in acc.items()}
        return (mean, per, counts) if with_counts else mean

    def timed_body_steps(self, k):
        """Per-launch device time of the world-1 step body exactly as the
        graphs run it (Adam inside the march launch, the next batch drawn in
        the bin launch, ...): k eager steps, events between consecutive
        launches on the launch stream, a spin kernel ahead of each step so the
        host has queued every launch before the first runs. Returns (per-launch
        mean ms, per-step ms of each launch, per-step sample counts)."""
        assert not self.dp
        if not self._pending:
            self.step()
        per, counts = {}, []
        self.body_live_counts = []  # the live rows of those steps (live_rows)
        for _ in range(k):
            torch.cuda.synchronize()
            torch.cuda._sleep(4_000_000)
            self._events = []
            self._tick("start")
            self._body(True)
            self.model.local_step += 1
            torch.cuda.synchronize()
            ev, self._events = self._events, None
            counts.append(self.sample_count())
            if self._live:
                self.body_live_counts.append(int(self._live_bufs["total"][0]))
            for (_, a), (name, b) in zip(ev[:-1], ev[1:]):
                per.setdefault(name, []).append(a.elapsed_time(b))
        return {n: float(np.mean(v)) for n, v in per.items()}, per, counts

    def _body(self, pending):
        """One step's launches (world 1): [optimizer(previous grads)] ->
        sample -> march -> network forward/backward. With an update pending,
        Adam and the batch draw share one launch and the deferred scaler
        bookkeeping + MLP packs ride in the march's emit launch (12 launches
        instead of 13; options split_head keeps them apart). By default
        (march_adam) Adam runs inside the march launch instead, beside the
        march waves, and the head launch only draws the batch."""
        if pending and self._march_adam:
            if not self._ahead:
                self._sample(nets=0)  # the MLP packs need Adam's fp16 weights: emit tail
            self._march(tail=True, adam=True)
        elif pending and self._merge_head:
            self._optimizer_head()
            self._march(tail=True)
        else:
            if pending:
                self._optimizer(defer=True)
            if self._ahead:  # the batch is drawn: the head's other parts (packs, cursor clear)
                lib, pk = nat.lib(), self._pk
                nat.check(lib.ngp_ffmlp_pack(2, pk["w"], pk["ins"], pk["hid"], pk["nl"], pk["img"],
                                             nat.stream_of(self.rays_o)), "ffmlp_pack")
                if self._grid_counter_bytes:
                    self.grid_ws[:self._grid_counter_bytes].zero_()
            else:
                self._sample()
            self._march()
        self._network(draw=self._draw_ahead, adam_split=pending and self._march_adam)

    def _xbody(self, pending, graph=False):
        """The world-1 body, and with sparse_exchange the gradient exchange
        after it (RCCL: in the same graph; gloo stages through the host, so a
        graph holds the body only and step() runs the exchange after it)."""
        self._body(pending)
        if self._xchg is not None and (self._nccl or not graph):
            self._xchg()
            self._tick("grad_exchange")

    def _optimizer_head(self):
        lib, P, s = nat.lib(), nat.ptr, nat.stream_of(self.rays_o)
        o, m, d = self._opt, self.model, self.data
        args = (o["n"], o["params"], o["grads"], o["m"], o["v"], o["half"], o["sizes"], self.lr, self.betas[0],
                self.betas[1], self.eps, self.iters, 1, 1.0, _PRECHECKED, P(self.state),
                P(d.poses), d.poses.shape[0], self._intr, d.H, d.W, self.N, self._boxes, self._nboxes, self._aabb,
                float(m.min_near), self.seed, P(self.rays_o), P(self.rays_d), P(self.rgba), P(self.bg),
                P(self.nears), P(self.fars), P(self.noises), P(self.counter), P(m.step_counter),
                P(self.grid_ws) if self._grid_counter_bytes else None, self._grid_counter_bytes)
        nat.check(lib.ngp_fused_optimizer_update_head(*args, s), "fused_optimizer_update_head")
        self._tick("optimizer")

    # ---- data parallel (world > 1): ZeRO-1 --------------------------------
    # The flat fp16 gradient is guarded (ngp_grad_guard) and averaged with one
    # reduce-scatter; each rank's optimizer updates its shard of the fp32
    # masters, the moments and the fp16 forward copy; the forward copy is
    # all-gathered on the collective stream while the next batch is sampled
    # and marched (neither reads a parameter). Per step each rank moves the
    # gradient once and the forward copy once (what one all-reduce moves) and
    # sweeps 1/world of the Adam state.
    def _guard(self):
        """GradScaler under sharding: the backward's kernels set the per-rank
        inf flag (no scan, n = 0); a flagged rank poisons every rank's chunk.
        The last launch of the network phase (inside its graph)."""
        nat.check(nat.lib().ngp_grad_guard(nat.ptr(self.flat_grad), 0, self.chunk, self.world,
                                           nat.ptr(self.state), nat.stream_of(self.flat_grad)), "grad_guard")

    def _reduce(self):
        """Averaging reduce-scatter of the (guarded) flat fp16 gradient into
        this rank's shard. The gradient is cleared for the next backward by the
        optimizer launch that consumes the shard (`_optimizer`)."""
        if not self.dp:
            return
        if self._exact_reduce:
            # DDP's arithmetic: fp32 sum over the ranks, / world, then the one
            # fp16 rounding the shard's storage needs (a NaN from the guard
            # still reaches every owner)
            self._grad32.copy_(self.flat_grad)
            if self._nccl:
                dist.reduce_scatter_tensor(self._shard32, self._grad32, op=dist.ReduceOp.SUM)
            else:
                out = torch.empty(self.chunk, dtype=torch.float32)
                dist.reduce_scatter_tensor(out, self._grad32.cpu(), op=dist.ReduceOp.SUM)
                self._shard32.copy_(out)
            torch.div(self._shard32, float(self.world), out=self._shard32)
            self.grad_shard.copy_(self._shard32)
        elif self._nccl:
            dist.reduce_scatter_tensor(self.grad_shard, self.flat_grad, op=dist.ReduceOp.AVG)
        else:  # gloo (tests): host-staged
            out = torch.empty(self.chunk, dtype=self.flat_grad.dtype)
            dist.reduce_scatter_tensor(out, self.flat_grad.cpu(), op=dist.ReduceOp.AVG)
            self.grad_shard.copy_(out)
        self._tick("reduce_scatter")

    def _gather_half(self, wait):
        """All-gather of the fp16 forward copy; returns the pending work."""
        if not self.dp:
            return None
        shard = self.flat_half[self.lo:self.hi]
        work = None
        if self._nccl:
            work = dist.all_gather_into_tensor(self.flat_half, shard, async_op=True)
        else:
            full = torch.empty(self.total, dtype=self.flat_half.dtype)
            dist.all_gather_into_tensor(full, shard.cpu())
            self.flat_half.copy_(full)
        if wait and work is not None:
            work.wait()
            work = None
        self._tick("all_gather")
        return work

    def _gather_masters(self):
        if not self.dp:
            return
        shard = self.flat_param[self.lo:self.hi]
        if self._nccl:
            dist.all_gather_into_tensor(self.flat_param, shard)
        else:
            full = torch.empty(self.total, dtype=self.flat_param.dtype)
            dist.all_gather_into_tensor(full, shard.cpu())
            self.flat_param.copy_(full)

    def _sample(self, nets=None):
        """The step head: batch of N rays (rays, RGBA target, background, march
        noise, near/far), the pending bookkeeping of a deferred optimizer
        update, and both networks' MLP fragment images, in one launch."""
        lib, P, s = nat.lib(), nat.ptr, nat.stream_of(self.rays_o)
        m, d, pk = self.model, self.data, self._pk
        self._ahead = False  # this draw replaces a batch drawn ahead (and resets the counter)
        # data parallel: the fp16 weights are still being all-gathered while
        # the batch is drawn, so the networks are packed in _network instead
        if nets is None:
            nets = 0 if self.dp else 2
        nat.check(lib.ngp_fused_step_head(P(d.poses), d.poses.shape[0], self._intr, d.H, d.W, self.N,
                                          self._boxes, self._nboxes, self._aabb, float(m.min_near), self.seed,
                                          P(self.state), P(self.rays_o), P(self.rays_d), P(self.rgba), P(self.bg),
                                          P(self.nears), P(self.fars), P(self.noises), P(self.counter),
                                          P(m.step_counter), 2.0, 0.5, self.growth_interval, 1, P(self.loss_ray),
                                          nets, pk["w"], pk["ins"], pk["hid"], pk["nl"], pk["img"],
                                          P(self.grid_ws) if self._grid_counter_bytes else None,
                                          self._grid_counter_bytes, s),
                  "fused_step_head")
        self._tick("step_head")

    def _forward_backward(self):
        """march -> network -> composite + MSE -> full backward into the fp16 grads
        (on the batch in the buffers; `_sample()` draws one)."""
        self._march()
        self._network()

    def _march(self, tail=False, adam=False):
        lib, P, s = nat.lib(), nat.ptr, nat.stream_of(self.rays_o)
        m, M, N, cnt = self.model, self.M, self.N, P(self.counter)
        args = (P(self.rays_o), P(self.rays_d), P(m.density_bitfield), float(m.bound), self.dt_gamma,
                self.max_steps, N, m.cascade, m.grid_size, M, P(self.nears), P(self.fars), P(self.xyzs),
                P(self.dirs), P(self.deltas), P(self.rays), cnt, P(self.noises), P(self.march_ws),
                self.march_ws.numel())
        if adam:  # + the pending Adam (march launch) and the bookkeeping + MLP packs (emit launch)
            pk = self._pk
            nat.check(lib.ngp_march_rays_train_prebuilt_adam(
                *args, P(self.state), 2.0, 0.5, self.growth_interval, 1, P(self.loss_ray), 2, pk["w"], pk["ins"],
                pk["hid"], pk["nl"], pk["img"], ctypes.byref(self._job), s), "march_rays_train_adam")
        elif tail:  # + the deferred scaler bookkeeping and the MLP packs (see _body)
            pk = self._pk
            nat.check(lib.ngp_march_rays_train_prebuilt_tail(
                *args, P(self.state), 2.0, 0.5, self.growth_interval, 1, P(self.loss_ray), 2, pk["w"], pk["ins"],
                pk["hid"], pk["nl"], pk["img"], s), "march_rays_train_tail")
        else:
            nat.check(lib.ngp_march_rays_train_prebuilt(*args, s), "march_rays_train")
        self._tick("march_rays_train+adam" if adam else "march_rays_train")

    def _network(self, draw=False, adam_split=False):
        lib, P, s = nat.lib(), nat.ptr, nat.stream_of(self.rays_o)
        m, e = self.model, self.enc
        M, N, cnt = self.M, self.N, P(self.counter)
        chk = nat.check
        pk = self._pk
        grid_args = (e.input_dim, e.level_dim, e.num_levels, self.S, e.base_resolution, e.gridtype_id,
                     int(e.align_corners), e.interp_id, s)
        table, tdt = (self.params[0], _F32) if self.table32 else (self.w_half[0], _F16)
        if self.dp and self._dp_tail:
            # + the deferred bookkeeping of the shard update (when the head did
            # not run it: batch drawn ahead) and the MLP packs of the gathered weights
            chk(lib.ngp_grid_encode_forward_fused_tail(P(self.xyzs), float(m.bound), P(table), tdt, P(e.offsets),
                                                       P(self.enc_out), M, cnt, *grid_args[:-1], P(self.state), 2.0,
                                                       0.5, self.growth_interval, 1, P(self.loss_ray), N, 2, pk["w"],
                                                       pk["ins"], pk["hid"], pk["nl"], pk["img"], s),
                "grid_encode_forward_fused_tail")
        elif adam_split and self._tail_in_fwd:
            # + the update's deferred bookkeeping and the MLP packs (the march
            # launch emitted the samples and left its tail row to this launch)
            chk(lib.ngp_grid_encode_forward_fused_tail(P(self.xyzs), float(m.bound), P(table), tdt, P(e.offsets),
                                                       P(self.enc_out), M, cnt, *grid_args[:-1], P(self.state), 2.0,
                                                       0.5, self.growth_interval, 1, P(self.loss_ray), N, 2, pk["w"],
                                                       pk["ins"], pk["hid"], pk["nl"], pk["img"], s),
                "grid_encode_forward_fused_tail")
        else:
            chk(lib.ngp_grid_encode_forward_fused(P(self.xyzs), float(m.bound), P(table), tdt, P(e.offsets),
                                                  P(self.enc_out), M, cnt, *grid_args[:-1], 0, s),
                "grid_encode_fused")
        self._tick("grid_encode_forward")
        sn, cn, img, pk = self.sig_net, self.col_net, self.mlp_img, self._pk
        if self.dp and not self._dp_tail:  # after the all-gather of the fp16 forward copy (see _sample)
            chk(lib.ngp_ffmlp_pack(2, pk["w"], pk["ins"], pk["hid"], pk["nl"], pk["img"], s), "ffmlp_pack")
        if self._one_fwd:  # both networks in one launch (ngp_nerf_forward)
            chk(lib.ngp_nerf_forward(P(self.enc_out), P(img[0]), P(img[1]), M, cnt, sn.hidden_dim, sn.num_layers,
                                     cn.hidden_dim, cn.num_layers, P(self.h_sigma), P(self.sigma),
                                     P(self.color_in), P(self.dirs), float(m.density_scale), P(self.color_out), s),
                "nerf_forward")
            self._tick("ffmlp_forward")
        else:
            chk(lib.ngp_nerf_sigma_forward(P(self.enc_out), P(self.w_half[1]), P(img[0]), M, cnt, 32, sn.hidden_dim,
                                           sn.num_layers, P(self.h_sigma), P(self.sigma), P(self.color_in),
                                           P(self.dirs), float(m.density_scale), _PAIR, s), "sigma_mlp")
            self._tick("ffmlp_forward_sigma")
            chk(lib.ngp_ffmlp_forward_rows(P(self.color_in), P(self.w_half[2]), P(img[1]), M, cnt, 32, 16,
                                           cn.hidden_dim, cn.num_layers, _RELU, _NONE, P(self.color_out), s),
                "color_mlp")
            self._tick("ffmlp_forward_color")
        # the live rows (a nonzero gradient) listed by the composite: both
        # backwards then run over them only (the other rows' products are zeros)
        live = self._live and draw
        if live:
            lv = self._live_bufs
            chk(lib.ngp_nerf_composite_loss_live(P(self.sigma), P(self.color_out), P(self.h_sigma), P(self.deltas),
                                                 P(self.rays), M, N, self.T_thresh, float(m.density_scale),
                                                 P(self.rgba), 4, P(self.bg), P(self.state), P(self.g_color_out),
                                                 P(self.g_h), None, None, P(self.loss_ray), P(lv["ray_rows"]),
                                                 P(lv["cnt"]), P(lv["rows"]), P(lv["total"]), s),
                "composite_loss_live")
        else:
            chk(lib.ngp_nerf_composite_loss(P(self.sigma), P(self.color_out), P(self.h_sigma), P(self.deltas),
                                            P(self.rays), M, N, self.T_thresh, float(m.density_scale),
                                            P(self.rgba), 4, P(self.bg), P(self.state), P(self.g_color_out),
                                            P(self.g_h), None, None, P(self.loss_ray), s), "composite_loss")
        self._tick("composite_loss")
        if self._one_bwd:  # both networks' backward in one launch (ngp_nerf_backward)
            timing = P(self.grid_ws) + self._grid_timing_at if self._grid_timing_at else None
            if live:
                chk(lib.ngp_nerf_backward_live(P(self.g_color_out), P(self.color_in), P(img[1]), P(self.g_h),
                                               P(self.enc_out), P(img[0]), P(self.g_enc), M, P(lv["rows"]),
                                               P(lv["total"]), sn.hidden_dim, sn.num_layers, cn.hidden_dim,
                                               cn.num_layers, P(self.mlp_ws[0]), self.mlp_ws[0].numel(),
                                               P(self.mlp_ws[1]), self.mlp_ws[1].numel(), timing, s),
                    "nerf_backward_live")
            else:
                chk(lib.ngp_nerf_backward(P(self.g_color_out), P(self.color_in), P(img[1]), P(self.g_h),
                                          P(self.enc_out), P(img[0]), P(self.g_enc), M, cnt, sn.hidden_dim,
                                          sn.num_layers, cn.hidden_dim, cn.num_layers, P(self.mlp_ws[0]),
                                          self.mlp_ws[0].numel(), P(self.mlp_ws[1]), self.mlp_ws[1].numel(),
                                          timing, s),
                    "nerf_backward")
            self._tick("ffmlp_backward")
        else:
            self._mlp_backward_split(lib, P, s, M, cnt, img)
        self._grid_backward(lib, P, s, M, cnt, draw, grid_args)
        if self.dp:
            self._guard()

    def _mlp_backward_split(self, lib, P, s, M, cnt, img):
        chk, sn, cn = nat.check, self.sig_net, self.col_net
        # color backward: its input gradient's geo columns land in g_h[:, 1:16]
        chk(lib.ngp_ffmlp_backward_rows(P(self.g_color_out), P(self.color_in), P(self.w_half[2]), P(img[1]), M,
                                        cnt, 32, 16, cn.hidden_dim, cn.num_layers, _RELU, P(self.g_h),
                                        None, _F16, _DEFER | _GEO, P(self.mlp_ws[1]), self.mlp_ws[1].numel(), s),
            "color_mlp_backward")
        self._tick("ffmlp_backward_color")
        chk(lib.ngp_ffmlp_backward_rows(P(self.g_h), P(self.enc_out), P(self.w_half[1]), P(img[0]), M, cnt, 32,
                                        16, sn.hidden_dim, sn.num_layers, _RELU, P(self.g_enc), None, _F16,
                                        _DEFER | _PAIR, P(self.mlp_ws[0]), self.mlp_ws[0].numel(), s),
            "sigma_mlp_backward")
        self._tick("ffmlp_backward_sigma")

    def _grid_backward(self, lib, P, s, M, cnt, draw, grid_args):
        chk, m, e, pk = nat.check, self.model, self.enc, self._pk
        bargs = (P(self.g_enc), P(self.xyzs), float(m.bound), P(e.offsets), P(self.grads[0]), M, cnt,
                 *grid_args[:-1], self._offsets_host, P(self.grid_ws), self.grid_ws.numel(), self._grid_flags,
                 self._inf_flag)
        if self._split_reduce:
            chk(lib.ngp_ffmlp_reduce(2, pk["ws"], pk["B"], pk["ins"], pk["hid"], pk["nl"], pk["gw"], _F16,
                                     self._inf_flag, s), "ffmlp_reduce")
            self._tick("ffmlp_reduce")
            chk(lib.ngp_grid_encode_backward_fused(*bargs, s), "grid_backward_fused")
        elif draw and self._live:
            # over the live rows (the MLP backward wrote g_enc for those only)
            lv = self._live_bufs
            largs = (P(self.g_enc), P(self.xyzs), float(m.bound), P(e.offsets), P(self.grads[0]), M, P(lv["rows"]),
                     P(lv["total"]), *grid_args[:-1], self._offsets_host, P(self.grid_ws), self.grid_ws.numel(),
                     self._grid_flags, self._inf_flag)
            chk(lib.ngp_grid_encode_backward_fused_reduce_batch_live(*largs, 2, pk["ws"], pk["B"], pk["ins"],
                                                                     pk["hid"], pk["nl"], pk["gw"], self._inf_flag,
                                                                     ctypes.byref(self._batch_job), s),
                "grid_backward_fused_reduce_batch_live")
            self._ahead = True
        elif draw:
            # + the next step's batch, as another column of the bin launch
            chk(lib.ngp_grid_encode_backward_fused_reduce_batch(*bargs, 2, pk["ws"], pk["B"], pk["ins"], pk["hid"],
                                                                pk["nl"], pk["gw"], self._inf_flag,
                                                                ctypes.byref(self._batch_job), s),
                "grid_backward_fused_reduce_batch")
            self._ahead = True
        else:
            # the MLP dW reduce rides in the grid backward's bin launch (same sums)
            chk(lib.ngp_grid_encode_backward_fused_reduce(*bargs, 2, pk["ws"], pk["B"], pk["ins"], pk["hid"],
                                                          pk["nl"], pk["gw"], self._inf_flag, s),
                "grid_backward_fused_reduce")
        if not draw:
            # this backward consumed the batch in the buffers and drew none: a
            # batch drawn ahead earlier is spent, the next step draws its own
            self._ahead = False
        self._tick("grid_encode_backward")

    def _optimizer(self, defer=False, prechecked=False, table_half=None):
        """GradScaler inf check + Adam (unscaled fp16 grads, LambdaLR) + scaler
        update. defer: the scaler / LR / loss bookkeeping is left to the next
        step head (_sample), which runs right after it in a step. prechecked
        (world 1): the grads are a step's, whose kernels set the found-inf
        flag, so no sweep over them checks it again. table_half (world 1, fp32
        table): an fp16 buffer the sweep fills with half(table) as well, every
        value (NGP_ADAM_SHADOW_ALL; the density query's copy)."""
        lib, P, s = nat.lib(), nat.ptr, nat.stream_of(self.rays_o)
        o, chk, N, cnt = self._opt, nat.check, self.N, P(self.counter)
        # world 1 zeroes the grads here; data parallel: the shard is the reduce-scatter's
        # output, and the flat gradient (which the collective has read) is cleared
        # for the next backward in the same graph
        if self.dp:
            self.flat_grad.zero_()
        half, zg = o["half"], int(not self.dp)
        if table_half is not None:  # the table section first (plan.sections), world 1 only
            assert not self.dp and self.table32 and self.lo == 0
            half = _vp_array([nat.ptr(table_half)] + [o["half"][q] for q in range(1, o["n"])])
            zg |= _SHADOW_ALL
        args = (o["n"], o["params"], o["grads"], o["m"], o["v"], half, o["sizes"], self.lr, self.betas[0],
                self.betas[1], self.eps, self.iters, zg, 1.0)
        # inside a step or a flush (world 1) the found-inf flag was set by the
        # backward's kernels; otherwise (direct calls, the averaged shard) the grads are swept
        mode = _PRECHECKED if (defer or prechecked) and not self.dp else _SCAN
        if defer:
            chk(lib.ngp_fused_optimizer_update(*args, mode, P(self.state), s), "fused_optimizer_update")
        else:
            chk(lib.ngp_fused_optimizer_step(*args, 2.0, 0.5, self.growth_interval, mode, N, cnt, None,
                                             P(self.loss_ray), P(self.state), s), "fused_optimizer_step")
        self._tick("optimizer")

    def _dp_body(self):
        """One data-parallel step with an update pending, as one captured
        sequence: Adam of this rank's shard (+ the gradient clear), the
        all-gather of the fp16 forward copy on RCCL's stream while the batch is
        drawn and marched, the network (+ guard), the reduce-scatter."""
        self._optimizer(defer=True)
        work = self._gather_half(wait=False)
        self._dp_pre()
        if work is not None:
            work.wait()
        self._network(draw=self._draw_ahead)
        self._reduce()

    def _dp_pre(self):
        """Data parallel, before the all-gather is joined: the batch (drawn
        ahead by the last backward: only the bin cursors are cleared; else the
        head launch draws it) and the march."""
        if self._ahead:
            if self._grid_counter_bytes:
                self.grid_ws[:self._grid_counter_bytes].zero_()
        else:
            self._sample()
        self._march()

    def step(self):
        """One training iteration (the optimizer half lags by one step, see
        the module docstring)."""
        if not self.dp:
            # gloo: the graphs hold the body only, the exchange runs here
            host_x = self._xchg is not None and not self._nccl
            if self._ring and self._pending:  # timing ring: graphs with event nodes
                self._ring[self._ring_i % len(self._ring)][0].replay()
                self._ring_i += 1
            elif self.graph is not None and self._pending:
                self.graph.replay()
            elif self._fresh is not None and not self._pending and self._ahead:
                self._fresh.replay()  # captured with the batch drawn ahead; leaves it drawn ahead
            else:
                self._xbody(self._pending)
                self.eager_steps += 1
                host_x = False
            if host_x:
                self._xchg()
        elif self._dp_whole is not None and self._pending and self._ahead == self._pre_ahead:
            self._dp_whole.replay()  # the whole step, collectives included (dp_graph)
        else:
            g = self.graph if self._pending else None
            work = None
            if self._pending:
                if g:
                    g["opt"].replay()
                else:
                    self._optimizer(defer=True)
                work = self._gather_half(wait=False)
            if g and self._ahead != self._pre_ahead:  # captured in the other batch state
                g = None
            if g:
                g["pre"].replay()
            else:
                self._dp_pre()
            if work is not None:
                work.wait()
            if g:
                g["net"].replay()
            else:
                self._network(draw=self._draw_ahead)
            self._reduce()
        self._pending = True
        self.model.local_step += 1

    def run(self, k):
        """k training iterations. With a multi-step graph (capture(multi=S),
        world 1) it replays floor(k / S) times -- S steps back to back in one
        graph launch, so the per-launch gap between graph replays is paid once
        per S steps -- and step() runs the rest. The graphs hold a pending
        update at their head, so after a flush() (update_density, checkpoint,
        read-outs) the first iteration runs as step()."""
        g, S = self.graph_multi, self._multi
        if g is not None and (not self.dp or self._dp_whole is not None) and not self._ring:
            # single steps until the state is the graph's: an update pending
            # (after a flush) and, data parallel, the batch state it was captured in
            while k > 0 and (not self._pending or (self.dp and self._ahead != self._pre_ahead)):
                self.step()
                k -= 1
            for _ in range(k // S):
                g.replay()
                self.model.local_step += S
            k -= (k // S) * S
        for _ in range(k):
            self.step()

    def flush(self, table_half=None, defer_end=False):
        """Apply the pending optimizer step (before reading or saving the
        parameters, or evaluating); data parallel: every rank then holds the
        full fp32 masters and fp16 forward copies. defer_end (world 1): the
        update's scaler / LR / loss bookkeeping is left pending for the
        caller's next launch that carries it (update_density's query)."""
        if self._pending:
            # the pending grads are the last step's: its kernels (and the
            # exchange's reduce) set the found-inf flag
            self._optimizer(prechecked=True, table_half=table_half, defer=defer_end and not self.dp)
            self._gather_half(wait=True)
            self._gather_masters()
            self._pending = False
        # sparse_exchange: lists that overflowed since the last flush are grown
        # (a skipped update is never silent)
        if self._xchg is not None and self._xchg.check():
            self._recapture()

    def capture(self, warmup=2, ring=0, multi=1):
        """hipGraph(s) of the step body. World 1: one graph (optimizer of the
        previous gradients, sample, march, network). Data parallel over RCCL:
        the whole step, collectives included (_dp_body); with gloo or
        options dp_graph=False, three graphs (optimizer | sample + march | network)
        with the collectives between them. ring=R (world 1): R further copies of the body graph
        with an event-record node after each launch; step() then replays
        them in turn (instead of the plain graph) and `ring_times` reads the
        per-launch device times of the last R replays. multi=S (world 1, and
        the whole data-parallel step): also a graph of S consecutive step
        bodies, replayed by run()."""
        for _ in range(warmup):
            self.step()
        torch.cuda.synchronize()
        self._drain_watchdog()
        if ring and not self.dp:
            self._ring, self._ring_i = [], 0
            try:
                for _ in range(ring):
                    g = torch.cuda.CUDAGraph()
                    self._events, self._capturing = [], True
                    with torch.cuda.graph(g):
                        self._tick("start")
                        self._xbody(True, graph=True)
                    self._ring.append((g, self._events))
            except Exception:
                self._ring = []
                raise
            finally:
                self._events, self._capturing = None, False
            return
        if not self.dp:
            self._ring, self._ring_i = [], 0  # step() would replay an older timing ring first
            if self._xchg is not None and self._nccl:
                self._capture_replicated(multi)
                return
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self._xbody(True, graph=True)
            # ... and the body of the first step after a flush (no update
            # pending, the batch drawn ahead by the last backward): so a
            # training loop's flush points (density updates, read-outs) cost no
            # eager step
            self._fresh = None
            if self._draw_ahead and self._ahead:
                gf = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gf):
                    self._xbody(False, graph=True)
                self._fresh = gf
            self.graph_multi, self._multi = None, 1
            if multi > 1 and (self._xchg is None or self._nccl):
                gm = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gm):
                    for _ in range(multi):
                        self._xbody(True, graph=True)
                self.graph_multi, self._multi = gm, multi
        elif self._dp_graph and self._nccl:
            # the whole data-parallel step in one graph, the collectives on
            # RCCL's stream forked from and joined to the capture stream: the
            # all-gather of the fp16 forward copy beside sample + march, then
            # the network, the guard and the reduce-scatter (no host round trip
            # between them; multi=S: S steps per graph as in world 1)
            self._dp_whole = None
            self.graph_multi, self._multi = None, 1
            self._pre_ahead = self._ahead  # the batch state the graph assumes (and leaves)
            err = None
            try:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self._dp_body()
                if multi > 1:
                    gm = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gm):
                        for _ in range(multi):
                            self._dp_body()
                    self.graph_multi, self._multi = gm, multi
                self._dp_whole = g
            except RuntimeError as e:  # a stack that cannot capture the collectives
                err = e
            # every rank takes the same form: a capture that failed on one rank
            # only would otherwise leave the ranks issuing different collective
            # sequences. Capture records without running, so no
            # collective of a step has run on any rank yet.
            torch.cuda.synchronize()
            ok = torch.tensor([0 if err is not None else 1], dtype=torch.int32, device=self.dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 0:
                print(f"FusedTrainer: whole-step capture failed on {'this' if err is not None else 'another'} rank "
                      f"({err!r:.200}); collectives between graphs on every rank", file=sys.stderr)
                self._dp_whole = None
                self._dp_graph = False
                self.graph_multi, self._multi = None, 1
                self._ahead = self._pre_ahead  # the batch state before the recording
                self.capture(warmup=0)  # the three graphs, no extra step
        else:
            graphs = {k: torch.cuda.CUDAGraph() for k in ("opt", "pre", "net")}
            with torch.cuda.graph(graphs["opt"]):
                self._optimizer(defer=True)
            self._pre_ahead = self._ahead
            with torch.cuda.graph(graphs["pre"]):
                self._dp_pre()
            with torch.cuda.graph(graphs["net"]):
                self._network(draw=self._draw_ahead)
            self.graph = graphs
        # capture recorded the launches without running them: the pending
        # update is still pending and the next step() replays it first

    def _drain_watchdog(self):
        """Before a capture over RCCL: wait until the process group's watchdog
        has retired every eager collective. Its poll queries each work's end
        event, and HIP answers a query of an event last recorded on a stream
        that has since joined a capture with hipErrorCapturedEvent, which ends
        the watchdog thread and aborts the process (seen once in a round-7
        bench run: an eager collective's work still listed when the next
        capture forked RCCL's stream)."""
        if not self._nccl:
            return
        wait = getattr(dist.distributed_c10d._get_default_group(), "_wait_for_pending_works", None)
        if wait is not None:
            wait()

    def _capture_replicated(self, multi):
        """sparse_exchange over RCCL: the world-1 body graphs with the
        exchange's all-gather inside them. Every rank takes the same form
        (ADVICE r05): a capture that fails on one rank would leave it eager
        while the others replay graphs, and their collective sequences would
        differ. Capture records without running, so no collective has run."""
        self.graph = self._fresh = self.graph_multi = None
        self._multi = 1
        ahead = self._ahead
        err = None
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._xbody(True, graph=True)
            gf = None
            if self._draw_ahead and self._ahead:
                gf = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gf):
                    self._xbody(False, graph=True)
            gm = None
            if multi > 1:
                gm = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gm):
                    for _ in range(multi):
                        self._xbody(True, graph=True)
        except RuntimeError as e:  # a stack that cannot capture the collective
            err = e
        torch.cuda.synchronize()
        ok = torch.tensor([0 if err is not None else 1], dtype=torch.int32, device=self.dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0:
            print(f"FusedTrainer: replicated-step capture failed on {'this' if err is not None else 'another'} rank "
                  f"({err!r:.200}); eager steps on every rank", file=sys.stderr)
            self._ahead = ahead  # the batch state before the recording
            return
        self.graph, self._fresh = g, gf
        if gm is not None:
            self.graph_multi, self._multi = gm, multi

    # ----------------------------------------------------------- read-outs
    def _state_f(self):
        return self.state.view(torch.float32)

    def _state_i(self):
        return self.state.view(torch.int32)

    def live_fraction(self):
        """Live rows (a nonzero gradient) over samples in the last step the
        backwards ran over the live rows only (live_rows), else None."""
        if not self._live:
            return None
        torch.cuda.synchronize()
        n = self.sample_count()
        return int(self._live_bufs["total"][0]) / max(n, 1)

    @property
    def last_loss(self):
        self.flush()
        return float(self._state_f()[2].item())

    @property
    def scale(self):
        self.flush()
        return float(self._state_f()[0].item())

    @property
    def optimizer_steps(self):
        self.flush()
        return int(self._state_i()[6].item())

    def sample_count(self):
        """Samples of the last step's batch."""
        return int(self._recent_counts(1)[0].item())

    def device_errors(self, clear=True):
        """The in-launch emit's error word (ngp_march_rays_train_error_offset:
        a bounded cross-workgroup wait ran out, so some step's sample offsets
        were wrong); 0 when every step was sound. A host sync."""
        m = self.model
        at = int(nat.lib().ngp_march_rays_train_error_offset(self.N, self.max_steps, m.cascade, m.grid_size))
        w = self.march_ws[at:at + 4].view(torch.int32)
        v = int(w.item())
        if clear and v:
            w.zero_()
        return v

    def adam_groups(self):
        """World 1, an update pending: the table's 4-parameter groups the
        pending Adam leaves unchanged (moments and gradient zero: it stores
        nothing for them), the other groups whose gradient is zero (it does
        not clear them), and all groups (ngp_head.h adam_idle / grad_set).
        None when no update is pending or the parameters are sharded."""
        if self.dp or not self._pending:
            return None
        torch.cuda.synchronize()
        n4 = self.params[0].numel() // 4
        m = self.exp_avg[:4 * n4].view(-1, 4)
        v = self.exp_avg_sq[:4 * n4].view(-1, 4)
        g = self.flat_grad[:4 * n4].view(torch.int16).view(-1, 4)
        idle = (m == 0).all(1) & (v == 0).all(1) & ((g & 0x7fff) == 0).all(1)
        zero_g = (g == 0).all(1) & ~idle
        return int(idle.sum()), int(zero_g.sum()), int(n4)

    def fit_exchange(self, margin=2.0):
        """sparse_exchange: size the touched-entry lists to margin x the
        longest list since the last fit (nerf/exchange.py), for the steady
        regime of training (the default lists hold every pair and cannot
        overflow); graphs captured before are captured again. Call it at the
        same step on every rank. Returns the lists' capacity."""
        if self._xchg is None:
            return None
        cap = self._xchg.fit(margin)
        self._recapture()
        return cap

    def _recapture(self):
        """Capture the graphs again (they hold the exchange's old buffers)."""
        if self.graph is not None or self._ring:
            ring, multi = len(self._ring), self._multi
            self.capture(warmup=0, multi=multi)
            if ring:  # (the plain capture drops the timing ring)
                self.capture(warmup=0, ring=ring)

    @property
    def exchange_overflows(self):
        """sparse_exchange: steps whose update every rank skipped because some
        rank's touched-entry list was longer than the lists' capacity (0 when
        every step applied its update; a host read). None otherwise."""
        return self._xchg.overflows if self._xchg is not None else None

    # ------------------------------------------------------ checkpoints
    # StepState as int32 words: 0 scale (f32), 4 growth tracker, 6 Adam steps,
    # 7 LambdaLR epoch, 8 finished iterations, 9 sampler draws
    _S_SCALE, _S_GROWTH, _S_ADAM, _S_EPOCH, _S_ITER, _S_DRAW = 0, 4, 6, 7, 8, 9

    def _moments(self):
        """Full-length Adam moments (data parallel: all-gathered from the shards)."""
        if not self.dp:
            return self.exp_avg, self.exp_avg_sq
        full = []
        for t in (self.exp_avg, self.exp_avg_sq):
            out = torch.empty(self.total, dtype=t.dtype, device=t.device)
            if self._nccl:
                dist.all_gather_into_tensor(out, t)
            else:
                host = torch.empty(self.total, dtype=t.dtype)
                dist.all_gather_into_tensor(host, t.cpu())
                out.copy_(host)
            full.append(out)
        return full

    def checkpoint(self, full=True, epoch=0, stats=None):
        """The reference trainer's checkpoint dict (nerf/utils.py save_checkpoint
        :1175-1211): epoch, global_step, stats, mean_count / mean_density, the
        model's state_dict and, with full, the optimizer / lr_scheduler / scaler
        state_dicts in torch's own formats (torch.optim.Adam over
        model.get_params(lr), LambdaLR, GradScaler load them), so checkpoints
        move between the reference's trainer and this one. `fused` carries the
        sampler's draw counter (not part of the reference format)."""
        self.flush()
        si = self.state.view(torch.int32).cpu()
        scale = float(self.state.view(torch.float32)[self._S_SCALE].item())
        adam_steps, ep, it = int(si[self._S_ADAM]), int(si[self._S_EPOCH]), int(si[self._S_ITER])
        m = self.model
        state = {"epoch": epoch, "global_step": it,
                 "stats": stats if stats is not None else {"loss": [], "valid_loss": [], "results": [],
                                                           "checkpoints": [], "best_result": None},
                 "mean_count": self.mean_count, "mean_density": self.mean_density,
                 "model": m.state_dict(),
                 # draw: batches drawn; ahead: the last of them is the next step's (drawn during
                 # the last backward, draw_ahead), which a restored trainer draws again
                 "fused": {"draw": int(si[self._S_DRAW]), "ahead": int(self._ahead)}}
        if full:
            m1, m2 = self._moments()
            # param indices follow model.get_params: encoder [0], sigma_net [1], encoder_dir [], color_net [2]
            opt_state = {}
            for i, (a, p) in enumerate(zip(self._starts, self.params)):
                n = p.numel()
                opt_state[i] = {"step": torch.tensor(float(adam_steps)),
                                "exp_avg": m1[a:a + n].view(p.shape).clone(),
                                "exp_avg_sq": m2[a:a + n].view(p.shape).clone()}
            group = {"lr": self.lr * 0.1 ** min(ep / self.iters, 1), "betas": tuple(self.betas), "eps": self.eps,
                     "weight_decay": 0, "amsgrad": False, "maximize": False, "foreach": None,
                     "capturable": False, "differentiable": False, "fused": None, "initial_lr": self.lr}
            state["optimizer"] = {"state": opt_state,
                                  "param_groups": [dict(group, params=ids) for ids in ([0], [1], [], [2])]}
            lr_now = self.lr * 0.1 ** min(ep / self.iters, 1)
            state["lr_scheduler"] = {"base_lrs": [self.lr] * 4, "last_epoch": ep, "_step_count": ep + 1,
                                     "_get_lr_called_within_step": False, "_last_lr": [lr_now] * 4,
                                     "lr_lambdas": [None] * 4}
            state["scaler"] = {"scale": scale, "growth_factor": 2.0, "backoff_factor": 0.5,
                               "growth_interval": self.growth_interval, "_growth_tracker": int(si[self._S_GROWTH])}
        return state

    def load_checkpoint(self, state, model_only=False):
        """Inverse of checkpoint() (and loader of the reference's checkpoint
        dicts, nerf/utils.py load_checkpoint :1237-1290): model weights and
        buffers, mean_count / mean_density, then Adam moments, step counts,
        LR epoch and GradScaler state."""
        self.flush()
        m = self.model
        if "model" not in state:  # a bare state_dict
            m.load_state_dict(state)
            self.sync_half()
            return
        m.load_state_dict(state["model"], strict=False)  # copies into the flat buffers' views
        self.sync_half()
        self._mean_count_pending, self._mean_density_pending = None, False
        m.mean_count = state.get("mean_count", m.mean_count)
        m.mean_density = state.get("mean_density", m.mean_density)
        self.refresh_occupancy()
        if model_only:
            return
        si = self.state.view(torch.int32)
        si[self._S_ITER] = int(state.get("global_step", 0))
        self._ahead = False
        if "fused" in state:
            draw = int(state["fused"]["draw"])
            if state["fused"].get("ahead"):
                # redraw the saved trainer's next batch (same draw index, so the same
                # rays); its draw re-records the last step's counts from the counter
                draw -= 1
                self.counter.copy_(self.model.step_counter[(draw - 1) & 15])
            si[self._S_DRAW] = draw
        if "optimizer" in state:
            st = state["optimizer"]["state"]
            for i, (a, p) in enumerate(zip(self._starts, self.params)):
                if i not in st:
                    continue
                for key, dst in (("exp_avg", self.exp_avg), ("exp_avg_sq", self.exp_avg_sq)):
                    full = st[i][key].to(self.dev, torch.float32).reshape(-1)
                    lo, hi = self.plan.owned(i)  # this rank's part of tensor i
                    if lo < hi:
                        dst[a + lo - self.lo:a + hi - self.lo].copy_(full[lo:hi])
                si[self._S_ADAM] = int(float(st[i]["step"]))
        if "lr_scheduler" in state:
            si[self._S_EPOCH] = int(state["lr_scheduler"]["last_epoch"])
        if "scaler" in state:
            self.state.view(torch.float32)[self._S_SCALE] = float(state["scaler"]["scale"])
            si[self._S_GROWTH] = int(state["scaler"]["_growth_tracker"])

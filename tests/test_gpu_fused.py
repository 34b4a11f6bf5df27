"""GPU: the fused train step (nerf/fused.py) against the autograd step.

The autograd path (NeRFNetwork.render through the reference-API autograd
Functions, torch loss, GradScaler, torch Adam) is the anchor. Both are fed the
same batch (the fused sampler's rays / target / background, zero march noise),
then compared stage by stage: sample counts (bit-exact), loss, gradients of
all three parameter tensors, and the Adam update from identical gradients.
"""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(cuda, num_rays=1024, mean_count=30000, bound=1, dt_gamma=0.0, occ="boxes", grid_timing=False,
           options=None):
    from nerf.fused import FusedTrainer
    from nerf.network_ff import NeRFNetwork
    from nerf.provider import SyntheticLego, lego_bitfield, sphere_bitfield
    torch.manual_seed(0)
    model = NeRFNetwork(bound=bound, cuda_ray=True, density_thresh=10).to(cuda)
    with torch.no_grad():  # a non-trivial field: larger table values than the 1e-4 init
        model.encoder.embeddings.normal_(0, 0.05)
    bits = (lego_bitfield if occ == "boxes" else sphere_bitfield)(cascade=model.cascade, bound=float(bound))
    model.density_bitfield.copy_(torch.from_numpy(bits).to(cuda))
    ref = copy.deepcopy(model)
    data = SyntheticLego(cuda, num_rays=num_rays)
    M = mean_count + 128 - mean_count % 128  # what run_cuda's align=128 makes of mean_count
    ref.mean_count = mean_count
    ft = FusedTrainer(model, data, M=M, seed=3, dt_gamma=dt_gamma, grid_timing=grid_timing, options=options)
    return model, ref, data, ft


def _ref_forward_backward(ref, ft, scale):
    rays_o, rays_d = ft.rays_o.clone(), ft.rays_d.clone()
    rgba, bg = ft.rgba.clone(), ft.bg.clone()
    ref.train()
    with torch.autocast("cuda", dtype=torch.float16):
        out = ref.render(rays_o[None], rays_d[None], staged=False, bg_color=bg[None], perturb=False,
                         force_all_rays=False, dt_gamma=ft.dt_gamma, max_steps=1024)
        pred = out["image"][0]
        gt = rgba[:, :3] * rgba[:, 3:] + bg * (1 - rgba[:, 3:])
        loss = ((pred - gt) ** 2).mean(-1).mean()
    (loss * scale).backward()
    return loss


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def test_lego_sampler(cuda):
    import raymarching
    model, ref, data, ft = _setup(cuda)
    ft._sample()
    torch.cuda.synchronize()
    n = ft.rays_d.norm(dim=-1)
    assert torch.allclose(n, torch.ones_like(n), atol=1e-5)
    poses_t = data.poses[:, :3, 3]
    assert ((ft.rays_o[:1] - poses_t).abs().sum(-1) == 0).any()        # origin = a pose centre
    assert torch.equal(ft.rays_o, ft.rays_o[:1].expand_as(ft.rays_o))  # one pose per step
    tgt = data.target(ft.rays_o, ft.rays_d)
    assert torch.allclose(tgt, ft.rgba, atol=1e-6)
    assert 0.05 < float(ft.rgba[:, 3].mean()) < 0.95
    nears, fars = raymarching.near_far_from_aabb(ft.rays_o, ft.rays_d, model.aabb_train, model.min_near)
    assert torch.equal(nears, ft.nears) and torch.equal(fars, ft.fars)
    assert 0.0 <= float(ft.bg.min()) and float(ft.bg.max()) < 1.0
    assert int(ft.counter.abs().sum()) == 0
    # a new step draws a new batch (the sampler bumps its own draw counter)
    r0 = ft.rays_d.clone()
    d0 = int(ft._state_i()[9])
    ft._sample()
    assert int(ft._state_i()[9]) == d0 + 1
    assert not torch.equal(r0, ft.rays_d)


# Config 2 (Lego: bound 1, one cascade, dt_gamma 0) and the Fox-like Config 3
# shape (bound 2, two cascades, dt_gamma 1/128: the serially marched rays)
@pytest.mark.parametrize("bound,dt_gamma", [(1, 0.0), (2, 1 / 128)])
def test_fused_forward_backward_matches_autograd(cuda, bound, dt_gamma):
    model, ref, data, ft = _setup(cuda, bound=bound, dt_gamma=dt_gamma)
    assert model.cascade == (1 if bound == 1 else 2)
    ft._sample()
    ft.noises.zero_()  # the autograd call below marches with perturb=False
    ft._forward_backward()
    torch.cuda.synchronize()
    scale = ft.scale
    loss = _ref_forward_backward(ref, ft, scale)
    torch.cuda.synchronize()
    # identical march (same rays, near/far, noise): same sample count
    assert int(ft.counter[0]) == int(ref.step_counter[0, 0]) > 0
    fused_loss = float(ft.loss_ray.double().sum()) / ft.N
    lv = float(loss.detach())
    assert abs(fused_loss - lv) <= 1e-3 * abs(lv) + 1e-7
    names = ["embeddings", "sigma_net", "color_net"]
    refs = [ref.encoder.embeddings.grad, ref.sigma_net.weights.grad, ref.color_net.weights.grad]
    for name, g, r in zip(names, ft.grads, refs):
        assert torch.isfinite(g.float()).all(), name
        assert r.abs().max() > 0, name
        assert _rel(g, r) < 1e-2, (name, _rel(g, r))


def test_fused_optimizer_matches_torch_adam_and_scaler(cuda):
    model, ref, data, ft = _setup(cuda)
    ft._sample()
    ft._forward_backward()
    torch.cuda.synchronize()
    scale = ft.scale
    params_ref = [p.detach().clone() for p in ft.params]
    grads16 = [g.clone() for g in ft.grads]
    ft._optimizer()
    torch.cuda.synchronize()
    # torch: GradScaler(unscale) + Adam(0.9, 0.99, eps 1e-15) + LambdaLR on fp32 grads
    ps = [torch.nn.Parameter(p.clone()) for p in params_ref]
    for p, g in zip(ps, grads16):
        p.grad = g.float()
    opt = torch.optim.Adam(ps, lr=1e-2, betas=(0.9, 0.99), eps=1e-15)
    scaler = torch.amp.GradScaler("cuda", init_scale=scale)
    scaler.scale(torch.ones((), device=cuda))  # initialises the scaler's scale tensor
    scaler.step(opt)
    scaler.update()
    for name, a, b, p0 in zip(["emb", "sigma", "color"], ft.params, ps, params_ref):
        assert torch.allclose(a.detach(), b.detach(), rtol=1e-5, atol=1e-7), name
        assert not torch.equal(a.detach(), p0), name  # the step moved the parameter
    assert all(int(g.abs().sum()) == 0 for g in ft.grads)   # grads zeroed for the next step
    assert ft.optimizer_steps == 1
    # fp16 forward copies refreshed from the fp32 masters: the MLPs always; the
    # table only when it is kept (data parallel), world 1 reads the fp32 table
    if not ft.table32:
        assert torch.equal(ft.w_half[0], ft.params[0].detach().half())
    assert torch.equal(ft.w_half[1], ft.params[1].detach().half())
    assert torch.equal(ft.w_half[2], ft.params[2].detach().half())


def test_fused_optimizer_leaves_untouched_groups_and_clears_the_grad(cuda):
    """The sweep stores nothing for a 4-value group Adam leaves unchanged
    (moments +0 and gradient +-0 give m' = v' = +0 and p' = p exactly) and
    clears only the gradient groups with a bit set (-0 included): after one
    update the untouched groups keep their p / m / v bits, the other groups
    move as torch's Adam moves them, and the whole gradient is +0."""
    _, _, _, ft = _setup(cuda)
    n = ft.params[0].numel() // 4 * 4
    grp = torch.arange(n, device=cuda) // 4
    kind = grp % 4  # 0: untouched, 1: gradient only, 2: moments only, 3: untouched with -0 grads
    gen = torch.Generator(device=cuda).manual_seed(7)
    g = torch.randn(n, device=cuda, generator=gen) * 0.01
    g = torch.where(kind == 1, g, torch.zeros_like(g)).half()
    g[kind == 3] = -0.0
    ft.grads[0].view(-1)[:n] = g
    m0 = torch.where(kind == 2, torch.randn(n, device=cuda, generator=gen) * 1e-3, torch.zeros(n, device=cuda))
    v0 = torch.where(kind == 2, torch.rand(n, device=cuda, generator=gen) * 1e-6, torch.zeros(n, device=cuda))
    ft.exp_avg[:n] = m0
    ft.exp_avg_sq[:n] = v0
    p0 = ft.flat_param[:n].clone()
    scale = ft.scale
    ft._optimizer()
    torch.cuda.synchronize()
    p1, m1, v1 = ft.flat_param[:n], ft.exp_avg[:n], ft.exp_avg_sq[:n]
    idle = (kind == 0) | (kind == 3)
    for a, b in ((p1, p0), (m1, m0), (v1, v0)):
        assert torch.equal(a[idle].view(torch.int32), b[idle].view(torch.int32))
    assert int((ft.flat_grad.view(torch.int16) != 0).sum()) == 0  # every bit cleared, -0 too
    # the moved groups against torch.optim.Adam (+ GradScaler's unscale) from the same state
    q = torch.nn.Parameter(p0.clone())
    q.grad = g.float() / scale
    opt = torch.optim.Adam([q], lr=1e-2, betas=(0.9, 0.99), eps=1e-15)
    opt.state[q] = {"step": torch.tensor(0.0), "exp_avg": m0.clone(), "exp_avg_sq": v0.clone()}
    opt.step()
    moved = ~idle
    assert not torch.equal(p1[moved], p0[moved])
    # (atol: a tiny v makes some updates ~0.1, p - update then cancels to ~1e-3)
    assert torch.allclose(p1[moved], q.detach()[moved], rtol=1e-5, atol=1e-6)
    assert torch.allclose(m1[moved], opt.state[q]["exp_avg"][moved], rtol=1e-5, atol=1e-12)
    assert torch.allclose(v1[moved], opt.state[q]["exp_avg_sq"][moved], rtol=1e-5, atol=1e-15)


def test_adam_groups_count_what_the_sweep_skips(cuda):
    """FusedTrainer.adam_groups (the bench's algorithmic-byte accounting for the
    sweep's skipped stores) against a direct count over the pending update's
    state, and the bytes it leads to between the all-read (16 B) and the
    all-written (28 B) bounds per table value."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    _, _, _, ft = _setup(cuda)
    assert ft.adam_groups() is None  # no update pending
    for _ in range(4):
        ft.step()
    idle, zero_g, total = ft.adam_groups()
    n = ft.params[0].numel() // 4 * 4
    m, v = ft.exp_avg[:n].view(-1, 4), ft.exp_avg_sq[:n].view(-1, 4)
    g = ft.flat_grad[:n].float().view(-1, 4)
    gb = ft.flat_grad[:n].view(torch.int16).view(-1, 4)
    want_idle = ((m == 0).all(1) & (v == 0).all(1) & (g == 0).all(1))
    assert idle == int(want_idle.sum()) and total == n // 4 and 0 < idle < total
    assert zero_g == int(((gb == 0).all(1) & ~want_idle).sum())
    n_tab = ft.params[0].numel()
    ab = bench.adam_bytes(ft, (idle, zero_g, total)) - bench.adam_bytes(ft) + 28 * n_tab
    assert 16 * n_tab < ab < 28 * n_tab


def test_march_launch_adam_equals_plain_sweep(cuda):
    """Adam inside the march launch (the default: the software-pipelined sweep
    beside the march waves) against the plain sweep of a flush, on the same
    pending gradient of a fresh table (most groups still untouched, whose
    stores both sweeps drop): parameters and moments bit for bit, after
    several steps so the moments are a mix of touched and untouched."""
    _, _, _, a = _setup(cuda)
    _, _, _, b = _setup(cuda)
    for t in (a, b):
        for _ in range(4):
            t.step()
    torch.cuda.synchronize()
    assert torch.equal(a.flat_grad.view(torch.int16), b.flat_grad.view(torch.int16))
    a.step()   # applies the pending update in its march launch (and runs one more forward/backward)
    b.flush()  # applies it with the plain sweep
    torch.cuda.synchronize()
    assert a._march_adam
    for x, y in zip(a.params, b.params):
        assert torch.equal(x.detach(), y.detach())
    assert torch.equal(a.exp_avg, b.exp_avg) and torch.equal(a.exp_avg_sq, b.exp_avg_sq)
    idle = ((a.exp_avg == 0) & (a.exp_avg_sq == 0)).float().mean()
    assert 0.05 < float(idle) < 1.0  # untouched table entries took part


def test_fused_optimizer_skips_on_inf(cuda):
    model, ref, data, ft = _setup(cuda)
    before = [p.detach().clone() for p in ft.params]
    ft.grads[1][3] = float("inf")
    s0 = ft.scale
    ft._optimizer()
    torch.cuda.synchronize()
    for a, b in zip(ft.params, before):
        assert torch.equal(a.detach(), b)
    assert ft.scale == s0 * 0.5 and ft.optimizer_steps == 0
    assert all(int(torch.isinf(g.float()).sum()) == 0 for g in ft.grads)


@pytest.mark.parametrize("deferred", [False, True])
def test_fused_optimizer_skips_when_unscale_overflows(cuda, deferred):
    """A scale backed off to 0 makes 1/scale inf: torch's unscale turns every
    grad (zeros included) into NaN/inf and GradScaler skips. The fp16 grads
    themselves are finite, so only the optimizer can see it."""
    model, ref, data, ft = _setup(cuda)
    ft.grads[1][3] = 0.5
    before = [p.detach().clone() for p in ft.params]
    ft._state_f()[0] = 0.0
    ft._optimizer(defer=deferred)
    if deferred:  # the bookkeeping runs in the next step head
        ft._sample()
    torch.cuda.synchronize()
    for a, b in zip(ft.params, before):
        assert torch.equal(a.detach(), b)
    assert float(ft._state_f()[0]) == 0.0 and int(ft._state_i()[6]) == 0  # backed off, no Adam step
    assert int(ft._state_i()[5]) == 0  # the flag was consumed by the scaler update


def test_pipelined_steps_match_serial_steps(cuda):
    """step() overlaps the previous step's optimizer with sampling + marching
    (and replays a captured graph of that): after flush() the parameters must
    be bit-identical to running sample -> forward/backward -> optimizer
    serially the same number of times."""
    _, _, _, a = _setup(cuda)
    _, _, _, b = _setup(cuda)
    for _ in range(3):
        a.step()
    a.capture(warmup=2)
    for _ in range(4):
        a.step()
    a.flush()
    for _ in range(3 + 2 + 4):
        b._sample()
        b._forward_backward()
        b._optimizer()
    b.flush()  # (the current buffer of the fused-Adam table made buffer 0, as a.flush() did)
    torch.cuda.synchronize()
    for x, y in zip(a.params, b.params):
        assert torch.equal(x.detach(), y.detach())
    assert a.optimizer_steps == b.optimizer_steps
    # every batch's sample count; `a` drew its next batch during the last backward
    # (options draw_ahead), which recorded the last count in step_counter already
    assert torch.equal(a._recent_counts(9), b._recent_counts(9))
    assert (a._recent_counts(9) > 0).all()
    # the scaler / loss bookkeeping (deferred into the march emit launch in world 1)
    assert a.scale == b.scale and a.last_loss == b.last_loss
    assert int(a._state_i()[7]) == int(b._state_i()[7])  # LambdaLR epoch


def test_multi_step_graph_equals_single_steps(cuda):
    """run(k) with a graph of S step bodies (capture(multi=S), what the bench
    replays) equals k single-step replays bit for bit, remainder included:
    parameters, optimizer steps, sample counts, scaler and loss."""
    _, _, _, a = _setup(cuda)
    _, _, _, b = _setup(cuda)
    for t in (a, b):
        for _ in range(2):
            t.step()
    a.capture(warmup=2, multi=4)
    b.capture(warmup=2)
    a.run(11)  # two multi-step replays + 3 single steps
    for _ in range(11):
        b.step()
    assert a.model.local_step == b.model.local_step
    a.flush()
    b.flush()
    torch.cuda.synchronize()
    for x, y in zip(a.params, b.params):
        assert torch.equal(x.detach(), y.detach())
    assert a.optimizer_steps == b.optimizer_steps
    assert torch.equal(a._recent_counts(15), b._recent_counts(15))
    assert a.scale == b.scale and a.last_loss == b.last_loss


class _CountingGraph:
    def __init__(self, g):
        self.g, self.replays = g, 0

    def replay(self):
        self.replays += 1
        self.g.replay()


def test_run_after_flush_replays_multi_step_graph(cuda):
    """After a flush() (update_density, checkpoints, read-outs) nothing is
    pending; run(k) then runs one step() and replays the multi-step graph for
    the rest, bit for bit equal to k single steps."""
    _, _, _, a = _setup(cuda)
    _, _, _, b = _setup(cuda)
    for t in (a, b):
        t.step()
    a.capture(warmup=2, multi=4)
    b.capture(warmup=2)
    a.graph_multi = _CountingGraph(a.graph_multi)
    for t in (a, b):
        t.flush()
        assert not t._pending
    a.run(10)  # one step(), two 4-step replays, one step()
    assert a.graph_multi.replays == 2
    for _ in range(10):
        b.step()
    a.flush()
    b.flush()
    torch.cuda.synchronize()
    for x, y in zip(a.params, b.params):
        assert torch.equal(x.detach(), y.detach())
    assert a.optimizer_steps == b.optimizer_steps and a.model.local_step == b.model.local_step


def test_first_step_after_flush_replays_its_graph(cuda):
    """capture() also records the first step after a flush (no update pending,
    batch drawn ahead); replaying it equals the eager step bit for bit, over
    several flush points, and counts as one replay each."""
    _, _, _, a = _setup(cuda)
    _, _, _, b = _setup(cuda)
    for t in (a, b):
        t.step()
        t.capture(warmup=2)
    assert a._fresh is not None
    a._fresh = _CountingGraph(a._fresh)
    b._fresh = None  # eager after each flush
    for _ in range(3):
        for t in (a, b):
            t.flush()
            for _ in range(3):
                t.step()
    assert a._fresh.replays == 3
    a.flush()
    b.flush()
    torch.cuda.synchronize()
    for x, y in zip(a.params, b.params):
        assert torch.equal(x.detach(), y.detach())
    assert torch.equal(a.state, b.state)
    assert a.optimizer_steps == b.optimizer_steps and a.model.local_step == b.model.local_step


@pytest.mark.parametrize("bound,dt_gamma", [(1, 0.0), (2, 1 / 128)])
def test_fused_training_reduces_loss_and_captures(cuda, bound, dt_gamma):
    model, ref, data, ft = _setup(cuda, num_rays=4096, mean_count=100000, bound=bound, dt_gamma=dt_gamma)
    losses = []
    for _ in range(4):
        ft.step()
        losses.append(ft.last_loss)
    ft.capture()
    for _ in range(60):
        ft.step()
    torch.cuda.synchronize()
    late = ft.last_loss
    assert np.isfinite(late) and late < losses[0], (losses, late)
    assert ft.optimizer_steps >= 60
    assert ft.device_errors() == 0  # no in-launch emit wait ran out


def test_mlp_fused_epilogues_match_unfused(cuda):
    """The fused step's MLP calls against the unfused ones, bit for bit: the
    prepacked-image path vs per-call packing, the sigma network with its glue
    epilogue vs ffmlp forward + ngp_nerf_glue_forward, the color backward that
    writes its geo-feature gradient into g_h[:, 1:16] vs plain backward +
    ngp_nerf_glue_backward, and the deferred two-network dW reduce."""
    import ctypes

    import _ngp_native as nat
    lib, P, s = nat.lib(), nat.ptr, None
    g = torch.Generator(device="cpu").manual_seed(4)
    B, n = 5000, 4700
    cnt = torch.tensor([n, 0], dtype=torch.int32, device=cuda)
    nets = [(32, 64, 2), (32, 64, 3)]
    ws = []
    for i, h, nl in nets:
        npar = h * (i + h * (nl - 1) + 16)
        ws.append(((torch.rand(npar, generator=g) - 0.5) * 0.3).half().to(cuda))
    x = torch.randn(B, 32, generator=g).half().to(cuda)
    d = torch.randn(B, 3, generator=g)
    dirs = (d / d.norm(dim=-1, keepdim=True)).to(cuda)
    imgs = [torch.zeros(int(lib.ngp_ffmlp_image_bytes(i, h, nl)), dtype=torch.uint8, device=cuda)
            for i, h, nl in nets]
    arr = lambda ts: (ctypes.c_void_p * len(ts))(*[P(t) if t is not None else None for t in ts])  # noqa: E731
    u32 = lambda v: (ctypes.c_uint32 * len(v))(*v)  # noqa: E731
    nat.check(lib.ngp_ffmlp_pack(2, arr(ws), u32([a for a, _, _ in nets]), u32([b for _, b, _ in nets]),
                                 u32([c for _, _, c in nets]), arr(imgs), s), "pack")
    # sigma network + glue
    h_ref = torch.zeros(B, 16, dtype=torch.half, device=cuda)
    sig_ref, ci_ref = torch.zeros(B, device=cuda), torch.zeros(B, 32, dtype=torch.half, device=cuda)
    nat.check(lib.ngp_ffmlp_forward_rows(P(x), P(ws[0]), None, B, P(cnt), 32, 16, 64, 2, 0, 6, P(h_ref), s), "f")
    nat.check(lib.ngp_nerf_glue_forward(P(h_ref), P(dirs), 1.0, P(sig_ref), P(ci_ref), B, P(cnt), s), "glue")
    h, sig = torch.zeros_like(h_ref), torch.zeros_like(sig_ref)
    ci = torch.zeros_like(ci_ref)
    nat.check(lib.ngp_nerf_sigma_forward(P(x), P(ws[0]), P(imgs[0]), B, P(cnt), 32, 64, 2, P(h), P(sig), P(ci),
                                         P(dirs), 1.0, 0, s), "sigma_fwd")
    torch.cuda.synchronize()
    assert torch.equal(h[:n].view(torch.int16), h_ref[:n].view(torch.int16))
    assert torch.equal(sig[:n], sig_ref[:n]), int((sig[:n] != sig_ref[:n]).sum())
    bad = (ci[:n].view(torch.int16) != ci_ref[:n].view(torch.int16))
    assert not bad.any(), (int(bad.sum()), bad.nonzero()[:8].tolist(), ci[:n][bad][:8].tolist(), ci_ref[:n][bad][:8].tolist())
    assert int(h[n:].view(torch.int16).abs().sum()) == 0  # rows past the count untouched
    # color network forward: image vs per-call packing
    o_ref, o = (torch.zeros(B, 16, dtype=torch.half, device=cuda) for _ in range(2))
    nat.check(lib.ngp_ffmlp_forward_rows(P(ci), P(ws[1]), None, B, P(cnt), 32, 16, 64, 3, 0, 6, P(o_ref), s), "f")
    nat.check(lib.ngp_ffmlp_forward_rows(P(ci), P(ws[1]), P(imgs[1]), B, P(cnt), 32, 16, 64, 3, 0, 6, P(o), s), "f")
    # backward: color with geo output + sigma, deferred reduce of both
    go = torch.randn(B, 16, generator=g).half().to(cuda)
    gh0 = torch.randn(B, 16, generator=g).half().to(cuda)  # column 0: the density gradient
    wsb = [torch.zeros(int(lib.ngp_ffmlp_backward_workspace_bytes(B, i, 16, h, nl)), dtype=torch.uint8,
                       device=cuda) for i, h, nl in nets]
    gi_c = torch.zeros(B, 32, dtype=torch.half, device=cuda)
    gw_ref = [torch.zeros(t.numel(), dtype=torch.half, device=cuda) for t in ws]
    gh_ref = gh0.clone()
    nat.check(lib.ngp_ffmlp_backward_rows(P(go), P(ci), P(ws[1]), None, B, P(cnt), 32, 16, 64, 3, 0, P(gi_c),
                                          P(gw_ref[1]), 1, 0, P(wsb[1]), wsb[1].numel(), s), "b")
    nat.check(lib.ngp_nerf_glue_backward(P(gi_c), P(gh_ref), B, P(cnt), s), "glue_b")
    gx_ref = torch.zeros(B, 32, dtype=torch.half, device=cuda)
    nat.check(lib.ngp_ffmlp_backward_rows(P(gh_ref), P(x), P(ws[0]), None, B, P(cnt), 32, 16, 64, 2, 0, P(gx_ref),
                                          P(gw_ref[0]), 1, 0, P(wsb[0]), wsb[0].numel(), s), "b")
    torch.cuda.synchronize()
    gh = gh0.clone()
    gw = [torch.zeros_like(t) for t in gw_ref]
    gx = torch.zeros_like(gx_ref)
    nat.check(lib.ngp_ffmlp_backward_rows(P(go), P(ci), P(ws[1]), P(imgs[1]), B, P(cnt), 32, 16, 64, 3, 0, P(gh),
                                          None, 1, 3, P(wsb[1]), wsb[1].numel(), s), "b_geo")
    nat.check(lib.ngp_ffmlp_backward_rows(P(gh), P(x), P(ws[0]), P(imgs[0]), B, P(cnt), 32, 16, 64, 2, 0, P(gx),
                                          None, 1, 1, P(wsb[0]), wsb[0].numel(), s), "b_defer")
    nat.check(lib.ngp_ffmlp_reduce(2, arr([wsb[1], wsb[0]]), u32([B, B]), u32([32, 32]), u32([64, 64]),
                                   u32([3, 2]), arr([gw[1], gw[0]]), 1, None, s), "reduce")
    torch.cuda.synchronize()
    assert torch.equal(o[:n].view(torch.int16), o_ref[:n].view(torch.int16))
    assert torch.equal(gh[:n].view(torch.int16), gh_ref[:n].view(torch.int16))
    assert torch.equal(gx[:n].view(torch.int16), gx_ref[:n].view(torch.int16))
    for a, b in zip(gw, gw_ref):
        assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    # pair-major ([16][B][2], the grid's level-major layout) input and input gradient
    xp = x.view(B, 16, 2).permute(1, 0, 2).contiguous()
    h2, sig2, ci2 = torch.zeros_like(h_ref), torch.zeros_like(sig_ref), torch.zeros_like(ci_ref)
    nat.check(lib.ngp_nerf_sigma_forward(P(xp), P(ws[0]), P(imgs[0]), B, P(cnt), 32, 64, 2, P(h2), P(sig2),
                                         P(ci2), P(dirs), 1.0, 4, s), "sigma_fwd_pair")
    gxp = torch.zeros_like(gx_ref)
    gw2 = torch.zeros_like(gw_ref[0])
    nat.check(lib.ngp_ffmlp_backward_rows(P(gh), P(xp), P(ws[0]), P(imgs[0]), B, P(cnt), 32, 16, 64, 2, 0, P(gxp),
                                          P(gw2), 1, 4, P(wsb[0]), wsb[0].numel(), s), "b_pair")
    torch.cuda.synchronize()
    assert torch.equal(h2[:n].view(torch.int16), h_ref[:n].view(torch.int16))
    assert torch.equal(sig2[:n], sig_ref[:n])
    gx_rows = gxp.view(16, B, 2).permute(1, 0, 2).reshape(B, 32)
    assert torch.equal(gx_rows[:n].view(torch.int16), gx_ref[:n].view(torch.int16))
    assert torch.equal(gw2.view(torch.int16), gw_ref[0].view(torch.int16))
    # both backwards in one launch (ngp_nerf_backward) against the two calls on
    # the pair-major input: input gradients bit for bit; dW summed in another
    # order (chunks dealt to other waves), so within fp16 rounding of the
    # same fp32 sums
    gh1, gxp1 = gh0.clone(), torch.zeros_like(gx_ref)
    nat.check(lib.ngp_ffmlp_backward_rows(P(go), P(ci), P(ws[1]), P(imgs[1]), B, P(cnt), 32, 16, 64, 3, 0, P(gh1),
                                          None, 1, 3, P(wsb[1]), wsb[1].numel(), s), "b_geo")
    nat.check(lib.ngp_ffmlp_backward_rows(P(gh1), P(xp), P(ws[0]), P(imgs[0]), B, P(cnt), 32, 16, 64, 2, 0,
                                          P(gxp1), None, 1, 5, P(wsb[0]), wsb[0].numel(), s), "b_pair_defer")
    gw_two = [torch.zeros_like(t) for t in gw_ref]
    nat.check(lib.ngp_ffmlp_reduce(2, arr([wsb[1], wsb[0]]), u32([B, B]), u32([32, 32]), u32([64, 64]),
                                   u32([3, 2]), arr([gw_two[1], gw_two[0]]), 1, None, s), "reduce")
    gh2, gxp2 = gh0.clone(), torch.zeros_like(gx_ref)
    wsm = [torch.full_like(w, 7) for w in wsb]  # stale slab contents must not leak through
    nat.check(lib.ngp_nerf_backward(P(go), P(ci), P(imgs[1]), P(gh2), P(xp), P(imgs[0]), P(gxp2), B, P(cnt),
                                    64, 2, 64, 3, P(wsm[0]), wsm[0].numel(), P(wsm[1]), wsm[1].numel(), None, s),
              "nerf_bwd")
    gw_one = [torch.zeros_like(t) for t in gw_ref]
    nat.check(lib.ngp_ffmlp_reduce(2, arr([wsm[1], wsm[0]]), u32([B, B]), u32([32, 32]), u32([64, 64]),
                                   u32([3, 2]), arr([gw_one[1], gw_one[0]]), 1, None, s), "reduce")
    torch.cuda.synchronize()
    assert torch.equal(gh2.view(torch.int16), gh1.view(torch.int16))  # column 0 kept, rows past n untouched
    assert torch.equal(gxp2.view(torch.int16), gxp1.view(torch.int16))
    for a, b in zip(gw_one, gw_two):
        a, b = a.float(), b.float()
        assert torch.all((a - b).abs() <= 2.0 ** -10 * b.abs() + 1e-6), float((a - b).abs().max())


@pytest.mark.parametrize("count", [4700, (256 * 9 + 128) * 32 - 5, (256 * 11 + 17) * 32])
def test_nerf_backward_half_chunks_equal_two_calls(cuda, count):
    """k_nerf_bwd splits a workgroup's last round of 1 or 2 chunks into
    16-sample halves: against the two per-network calls (colour backward with
    its geo-feature epilogue, then the sigma backward on the pair-major
    encodings; whole chunks), input gradients bit for bit and dW within fp16
    rounding of the same sums; the counts give workgroups 1, 2 and 3 chunks in
    their last round."""
    import ctypes

    import _ngp_native as nat
    lib, P, s = nat.lib(), nat.ptr, None
    g = torch.Generator(device="cpu").manual_seed(11)
    B = 96000
    cnt = torch.tensor([count, 0], dtype=torch.int32, device=cuda)
    nets = [(32, 64, 2), (32, 64, 3)]
    ws = [((torch.rand(h * (i + h * (nl - 1) + 16), generator=g) - 0.5) * 0.3).half().to(cuda) for i, h, nl in nets]
    imgs = [torch.zeros(int(lib.ngp_ffmlp_image_bytes(i, h, nl)), dtype=torch.uint8, device=cuda)
            for i, h, nl in nets]
    arr = lambda ts: (ctypes.c_void_p * len(ts))(*[P(t) if t is not None else None for t in ts])  # noqa: E731
    u32 = lambda v: (ctypes.c_uint32 * len(v))(*v)  # noqa: E731
    nat.check(lib.ngp_ffmlp_pack(2, arr(ws), u32([a for a, _, _ in nets]), u32([b for _, b, _ in nets]),
                                 u32([c for _, _, c in nets]), arr(imgs), s), "pack")
    xp = torch.randn(16, B, 2, generator=g).half().to(cuda)   # pair-major encodings
    ci = torch.randn(B, 32, generator=g).half().to(cuda)
    go = torch.randn(B, 16, generator=g).half().to(cuda)
    gh0 = torch.randn(B, 16, generator=g).half().to(cuda)
    wsb = [torch.zeros(int(lib.ngp_ffmlp_backward_workspace_bytes(B, i, 16, h, nl)), dtype=torch.uint8,
                       device=cuda) for i, h, nl in nets]
    # two calls
    gh_t, gx_t = gh0.clone(), torch.zeros(16, B, 2, dtype=torch.half, device=cuda)
    nat.check(lib.ngp_ffmlp_backward_rows(P(go), P(ci), P(ws[1]), P(imgs[1]), B, P(cnt), 32, 16, 64, 3, 0, P(gh_t),
                                          None, 1, 3, P(wsb[1]), wsb[1].numel(), s), "b_geo")
    nat.check(lib.ngp_ffmlp_backward_rows(P(gh_t), P(xp), P(ws[0]), P(imgs[0]), B, P(cnt), 32, 16, 64, 2, 0,
                                          P(gx_t), None, 1, 5, P(wsb[0]), wsb[0].numel(), s), "b_pair_defer")
    gw_t = [torch.zeros(t.numel(), dtype=torch.half, device=cuda) for t in ws]
    nat.check(lib.ngp_ffmlp_reduce(2, arr([wsb[1], wsb[0]]), u32([B, B]), u32([32, 32]), u32([64, 64]),
                                   u32([3, 2]), arr([gw_t[1], gw_t[0]]), 1, None, s), "reduce")
    # one launch
    gh, gx = gh0.clone(), torch.zeros(16, B, 2, dtype=torch.half, device=cuda)
    wsm = [torch.full_like(w, 7) for w in wsb]  # stale slab contents must not leak through
    nat.check(lib.ngp_nerf_backward(P(go), P(ci), P(imgs[1]), P(gh), P(xp), P(imgs[0]), P(gx), B, P(cnt),
                                    64, 2, 64, 3, P(wsm[0]), wsm[0].numel(), P(wsm[1]), wsm[1].numel(), None, s),
              "nerf_bwd")
    gw = [torch.zeros(t.numel(), dtype=torch.half, device=cuda) for t in ws]
    nat.check(lib.ngp_ffmlp_reduce(2, arr([wsm[1], wsm[0]]), u32([B, B]), u32([32, 32]), u32([64, 64]),
                                   u32([3, 2]), arr([gw[1], gw[0]]), 1, None, s), "reduce")
    torch.cuda.synchronize()
    assert torch.equal(gh[:count].view(torch.int16), gh_t[:count].view(torch.int16))
    assert torch.equal(gx[:, :count].view(torch.int16), gx_t[:, :count].view(torch.int16))
    assert int(gx[:, count:].view(torch.int16).abs().sum()) == 0  # rows past the count untouched
    for a, b in zip(gw, gw_t):
        a, b = a.float(), b.float()
        assert torch.isfinite(a).all() and torch.all((a - b).abs() <= 2.0 ** -10 * b.abs() + 1e-6), \
            float((a - b).abs().max())


@pytest.mark.parametrize("bound,dt_gamma", [(1, 0.0), (2, 1 / 128)])
def test_march_emit_in_launch_equals_emit_launch(cuda, bound, dt_gamma):
    """The march + Adam launch emits the samples itself (ticketed ray blocks,
    block totals published as agent-scope words; the default) against the
    separate emit launch (options emit_inline=False): samples, rays, counter
    and the trained parameters bit for bit, step after step."""
    _, _, _, a = _setup(cuda, bound=bound, dt_gamma=dt_gamma)
    _, _, _, b = _setup(cuda, bound=bound, dt_gamma=dt_gamma, options=dict(emit_inline=False))
    for it in range(5):
        a.step()
        b.step()
        torch.cuda.synchronize()
        assert torch.equal(a.counter, b.counter), (it, a.counter.tolist(), b.counter.tolist())
        n = a.sample_count()
        assert n > 0 and n == b.sample_count()
        assert torch.equal(a.rays, b.rays)
        for x, y in ((a.xyzs, b.xyzs), (a.dirs, b.dirs), (a.deltas, b.deltas)):
            assert torch.equal(x[:n].view(torch.int32), y[:n].view(torch.int32)), it
    a.flush()
    b.flush()
    for x, y in zip(a.params, b.params):
        assert torch.equal(x.detach(), y.detach())
    assert a.device_errors() == 0


def test_tail_in_grid_forward_equals_emit_tail(cuda):
    """The step's tail row (deferred scaler / LR / loss bookkeeping + MLP
    fragment packs) in the grid forward's launch (the default; with the
    in-launch emit the march is then one launch) against the tail row of the
    emit launch (options tail_in_fwd=False): parameters, moments and the step
    state bit for bit, eager and captured, across an overflow-free run."""
    _, _, _, a = _setup(cuda)
    _, _, _, b = _setup(cuda, options=dict(tail_in_fwd=False))
    assert a._tail_in_fwd and not b._tail_in_fwd
    for t in (a, b):
        for _ in range(3):
            t.step()
        t.capture(warmup=1, multi=4)
        t.run(9)
        t.flush()
    torch.cuda.synchronize()
    for x, y in zip(a.params, b.params):
        assert torch.equal(x.detach(), y.detach())
    assert torch.equal(a.exp_avg, b.exp_avg) and torch.equal(a.exp_avg_sq, b.exp_avg_sq)
    assert torch.equal(a.state, b.state)
    for x, y in zip(a.mlp_img, b.mlp_img):
        assert torch.equal(x, y)


@pytest.mark.parametrize("bound,dt_gamma,occ", [(1, 0.0, "boxes"), (2, 1 / 128, "boxes"), (1, 0.0, "ball")])
def test_live_row_backwards_equal_all_row_backwards(cuda, bound, dt_gamma, occ):
    """The backwards over the live rows only (the default: the composite
    lists the rows with a nonzero gradient, the MLP backward and the grid bin
    kernel walk that list) against the backwards over every row (options
    live_rows=False): the loss
    and the encoding gradient of each live row bit for bit, the grid gradient
    bit for bit (dead rows add exact zeros, live rows keep their order), the
    MLP weight gradients to fp16-accumulation tolerance (other 32-row chunks);
    then eager and captured runs stay within tolerance of each other."""
    _, _, _, a = _setup(cuda, bound=bound, dt_gamma=dt_gamma, occ=occ)
    _, _, _, b = _setup(cuda, bound=bound, dt_gamma=dt_gamma, occ=occ, options=dict(live_rows=False))
    assert a._live and not b._live
    a.step()
    b.step()
    torch.cuda.synchronize()
    n = a.sample_count()
    assert n > 0 and n == b.sample_count()
    lv = a._live_bufs
    total = int(lv["total"][0])
    rows = lv["rows"][:total].long()
    gh, gc = b.g_h[:n].float(), b.g_color_out[:n].float()
    live_ref = torch.nonzero((gh != 0).any(dim=1) | (gc != 0).any(dim=1)).flatten()
    assert 0 < total <= n
    assert torch.equal(torch.sort(rows).values, live_ref), (total, live_ref.numel())
    ea, eb = a.g_enc.view(16, -1, 2), b.g_enc.view(16, -1, 2)
    assert torch.equal(ea[:, rows].view(torch.int16), eb[:, rows].view(torch.int16))
    assert torch.equal(a.grads[0].view(torch.int16) if a.grads[0].dtype == torch.float16 else a.grads[0],
                       b.grads[0].view(torch.int16) if b.grads[0].dtype == torch.float16 else b.grads[0])
    for x, y in zip(a.grads[1:], b.grads[1:]):
        x, y = x.float(), y.float()
        assert torch.isfinite(x).all() and _rel(x, y) < 1e-3, _rel(x, y)
    assert a.last_loss == b.last_loss  # (flushes: after the gradient checks)
    for t in (a, b):
        for _ in range(3):
            t.step()
        t.capture(warmup=1, multi=4)
        t.run(9)
        t.flush()
    torch.cuda.synchronize()
    for x, y in zip(a.params, b.params):
        assert torch.isfinite(x).all() and _rel(x.detach(), y.detach()) < 1e-3, _rel(x.detach(), y.detach())
    assert abs(a.last_loss - b.last_loss) <= 1e-3 * abs(b.last_loss)


def test_grad_guard_poisons_every_shard(cuda):
    """ngp_grad_guard (data-parallel GradScaler guard): an inf/nan anywhere in
    the rank's gradient puts a NaN at the head of every rank's chunk; a finite
    gradient is left untouched and the flag is cleared either way."""
    import _ngp_native as nat
    _, _, _, ft = _setup(cuda)
    world, chunk = 4, 1024
    g = torch.randn(world * chunk + 64, device=cuda).half()
    ref = g.clone()
    nat.check(nat.lib().ngp_grad_guard(nat.ptr(g), g.numel(), chunk, world, nat.ptr(ft.state),
                                       nat.stream_of(g)), "grad_guard")
    torch.cuda.synchronize()
    assert torch.equal(g, ref)
    g[3000] = float("inf")
    nat.check(nat.lib().ngp_grad_guard(nat.ptr(g), g.numel(), chunk, world, nat.ptr(ft.state),
                                       nat.stream_of(g)), "grad_guard")
    torch.cuda.synchronize()
    heads = g[torch.arange(world, device=cuda) * chunk].float()
    assert torch.isnan(heads).all()
    g[torch.arange(world, device=cuda) * chunk] = ref[torch.arange(world, device=cuda) * chunk]
    g[3000] = ref[3000]
    assert torch.equal(g, ref)
    assert int(ft.state.view(torch.int32)[11].item()) == 0  # local_inf cleared


def test_step_overflow_skips_via_kernel_flags(cuda):
    """Inside a step the optimizer trusts the found-inf flag the grid backward
    and the MLP reduce set (no sweep over the grads): a loss scale that makes
    the fp16 grads overflow must skip the update and back the scale off."""
    _, _, _, ft = _setup(cuda)
    ft.state.view(torch.float32)[0] = 2.0 ** 40  # GradScaler scale
    before = [p.detach().clone() for p in ft.params]
    ft.step()   # grads overflow
    ft.step()   # applies the pending update (kernel-flag mode): skipped
    ft.flush()  # the second step's update (its kernels' flag, as in a step): skipped as well
    torch.cuda.synchronize()
    assert ft.optimizer_steps == 0
    assert ft.scale == 2.0 ** 38
    for a, b in zip(ft.params, before):
        assert torch.equal(a.detach(), b)


def test_checkpoint_roundtrip_and_torch_formats(cuda):
    """checkpoint() is the reference trainer's checkpoint dict (nerf/utils.py
    save_checkpoint): torch's Adam / LambdaLR / GradScaler load its optimizer,
    lr_scheduler and scaler entries, and a trainer restored from it continues
    bit-identically to the one that saved it."""
    from nerf.network_ff import NeRFNetwork
    _, _, _, a = _setup(cuda)
    for _ in range(3):
        a.step()
    ck = a.checkpoint()
    assert {"epoch", "global_step", "stats", "mean_count", "mean_density", "model", "optimizer",
            "lr_scheduler", "scaler"} <= set(ck)
    assert ck["global_step"] == 3 and set(ck["model"]) >= {"encoder.embeddings", "sigma_net.weights",
                                                           "color_net.weights", "density_bitfield"}
    m2 = NeRFNetwork(bound=1, cuda_ray=True).to(cuda)
    opt = torch.optim.Adam(m2.get_params(1e-2), lr=1e-2, betas=(0.9, 0.99), eps=1e-15)
    opt.load_state_dict(ck["optimizer"])
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda it: 0.1 ** min(it / 30000, 1))
    sched.load_state_dict(ck["lr_scheduler"])
    scaler = torch.amp.GradScaler("cuda")
    scaler.load_state_dict(ck["scaler"])
    assert scaler.get_scale() == a.scale
    assert torch.equal(opt.state[m2.encoder.embeddings]["exp_avg"], ck["optimizer"]["state"][0]["exp_avg"])
    # resume: a differently initialised trainer restored from the checkpoint
    _, _, _, b = _setup(cuda)
    with torch.no_grad():
        for p in b.params:
            p.add_(0.01)
    b.sync_half()
    b.load_checkpoint(ck)
    for _ in range(3):
        a.step()
        b.step()
    a.flush()
    b.flush()
    torch.cuda.synchronize()
    for x, y in zip(a.params, b.params):
        assert torch.equal(x.detach(), y.detach())
    assert a.optimizer_steps == b.optimizer_steps and a.scale == b.scale


def test_checkpoint_after_update_density_has_reference_bookkeeping(cuda):
    """update_density does update_extra_state's bookkeeping (renderer.py:584,
    593-596): mean_density = mean(clamp(grid, 0)), mean_count = int(mean of the
    last min(16, local_step) batches' sample counts), local_step = 0; the
    checkpoint carries those values, and a loaded checkpoint's values are kept."""
    model, _, _, ft = _setup(cuda)
    counts = []
    for _ in range(5):
        ft.step()
        counts.append(ft.sample_count())
    assert model.local_step == 5
    ft.update_density()
    assert model.local_step == 0
    want_density = float(torch.mean(model.density_grid.clamp(min=0)).item())
    ck = ft.checkpoint()
    assert abs(ck["mean_density"] - want_density) <= 1e-6 * want_density and want_density > 0
    assert ck["mean_count"] == int(sum(counts) / len(counts)), (ck["mean_count"], counts)
    for _ in range(20):  # more than 16 batches since the update: the last 16 count
        ft.step()
        counts.append(ft.sample_count())
    ft.update_density()
    assert ft.mean_count == int(sum(counts[-16:]) / 16)
    ck2 = ft.checkpoint()
    ck2["mean_density"], ck2["mean_count"] = 12.5, 777
    ft.load_checkpoint(ck2)
    assert ft.mean_density == 12.5 and ft.mean_count == 777 and ft.checkpoint()["mean_count"] == 777


def test_grid_backward_is_deterministic(cuda):
    """The binned backward sums every bin exactly (int64 fixed point), also
    the bins several work units share (their partial sums meet in an int64
    slot): two backward passes of one batch give bit-identical table grads."""
    _, _, _, ft = _setup(cuda, num_rays=4096, mean_count=400000, occ="ball")
    ft._sample()
    ft._forward_backward()
    g1 = ft.grads[0].clone()
    n = ft.sample_count()
    ft.flat_grad.zero_()
    ft.grid_ws[:ft._grid_counter_bytes].zero_()  # the bin cursors (the step head clears them in a step)
    ft._network()
    torch.cuda.synchronize()
    assert n > 250000 and g1.abs().sum() > 0
    assert torch.equal(g1.view(torch.int16), ft.grads[0].view(torch.int16))


def test_grid_backward_self_timing_counts_graph_replays(cuda):
    """grid_timing (NGP_GRID_TIMING; the bench's roofline clock): every grid backward of
    the captured step opens a ring entry with its samples and the accumulate
    closes it; the spans are positive and a step's worth."""
    _, _, _, ft = _setup(cuda, num_rays=4096, mean_count=120000, grid_timing=True)
    assert ft._grid_timing_at > ft._grid_counter_bytes
    ft.step()
    ft.capture(warmup=1)
    ft.grid_timing_reset()
    counts = []
    for _ in range(5):
        ft.step()
        torch.cuda.synchronize()
        counts.append(min(ft.sample_count(), ft.M))
    calls, ms, samples = ft.grid_timing()
    assert calls == 5 and samples == counts
    assert all(1e-3 < v < 5.0 for v in ms), ms
    assert ft.grid_timing(last=2)[1] == ms[-2:]


def test_grid_timing_off_by_default(cuda):
    """The self-timing ring is bench instrumentation: off unless asked for."""
    _, _, _, ft = _setup(cuda)
    assert ft._grid_timing_at == 0 and ft.grid_timing() is None


def test_plain_capture_after_ring_capture_replays_plain_graph(cuda):
    """capture() after capture(ring=R) drops the timing ring, so
    step() replays the newly captured graph."""
    _, _, _, ft = _setup(cuda)
    ft.step()
    ft.capture(warmup=1)
    # a timing ring left by an earlier capture(ring=R) (ROCm 7 refuses its event
    # nodes, so it is stood in for here: step() would replay it first)
    ft._ring, ft._ring_i = [(ft.graph, [])], 0
    ft.capture(warmup=1)
    assert ft._ring == [] and ft.graph is not None
    ft.graph = _CountingGraph(ft.graph)
    ft.step()
    assert ft.graph.replays == 1


def test_composite_loss_large_densities_match_serial(cuda):
    """The fused composite's prefix-sum transmittance against the reference's
    serial loop (raymarching.cu composite_rays_train_forward) at the densities a
    hard-surfaced scene trains into: sigma * delta far above the running
    prefix, and sigma = inf (exp overflow of a large density logit). The
    serial T *= 1 - alpha stays finite there; so must the fused form."""
    import ctypes
    import _ngp_native as nat
    _, _, _, ft = _setup(cuda)
    rng = np.random.default_rng(5)
    N, S = 48, 96
    M = N * S
    sigma = rng.uniform(0, 30, M).astype(np.float32)
    for r in range(0, N, 3):  # a huge density a few samples into every third ray
        sigma[r * S + 2 + r % 7] = [1e9, 3e7, np.inf][r % 3]
    deltas = np.stack([rng.uniform(0.002, 0.01, M), rng.uniform(0.002, 0.01, M)], -1).astype(np.float32)
    col = rng.normal(0, 2, (M, 16)).astype(np.float16)
    h = rng.normal(0, 1, (M, 16)).astype(np.float16)
    rays = np.stack([np.arange(N), np.arange(N) * S, np.full(N, S)], -1).astype(np.int32)
    gt = rng.uniform(0, 1, (N, 4)).astype(np.float32)
    bg = rng.uniform(0, 1, (N, 3)).astype(np.float32)
    T_thresh = 1e-4
    # serial reference (fp64 accumulation, fp32 sigma * delta and half sigmoid)
    rgb = (1 / (1 + np.exp(-col[:, :3].astype(np.float32)))).astype(np.float16).astype(np.float64)
    want = np.zeros((N, 3))
    for r in range(N):
        T, acc, ws = 1.0, np.zeros(3), 0.0
        for k in range(r * S, r * S + S):
            with np.errstate(over="ignore", invalid="ignore"):
                alpha = 1.0 - np.exp(-float(np.float32(sigma[k]) * np.float32(deltas[k, 0])))
            w = alpha * T
            acc += w * rgb[k]
            ws += w
            T *= 1 - alpha
            if T < T_thresh:
                break
        want[r] = acc + (1 - ws) * bg[r]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    d_sigma, d_col, d_h, d_del, d_rays, d_gt, d_bg = map(t, (sigma, col, h, deltas, rays, gt, bg))
    g_col = torch.zeros(M, 16, dtype=torch.float16, device=cuda)
    g_h = torch.zeros(M, 16, dtype=torch.float16, device=cuda)
    img = torch.zeros(N, 3, device=cuda)
    ws_out = torch.zeros(N, device=cuda)
    loss = torch.zeros(N, device=cuda)
    P = nat.ptr
    nat.check(nat.lib().ngp_nerf_composite_loss(
        P(d_sigma), P(d_col), P(d_h), P(d_del), P(d_rays), M, N, T_thresh, 1.0, P(d_gt), 4, P(d_bg),
        P(ft.state), P(g_col), P(g_h), P(img), P(ws_out), P(loss), nat.stream_of(img)), "composite_loss")
    torch.cuda.synchronize()
    got = img.double().cpu().numpy()
    assert np.isfinite(got).all() and torch.isfinite(loss).all()
    assert torch.isfinite(g_col.float()).all() and torch.isfinite(g_h.float()).all()
    np.testing.assert_allclose(got, want, rtol=1e-4, atol=1e-5)


def test_composite_loss_termination_near_threshold(cuda, parity_report):
    """the fused composite's early stop (T = exp(-prefix
    sum of sigma delta), DPP scans) against the reference's serial fp32
    T *= 1 - alpha (raymarching.cu:540-567, 647-690; oracle/ngp_oracle.c).
    Rays are built so the serial T crosses T_thresh right at a chosen sample,
    by a relative margin from ~1e-6 (a few float ulps) up to 1e-2, across one
    and two 64-sample chunks. The terminating sample is the last row whose
    density gradient is nonzero (the composite writes exact zeros past it, the
    live-row set). Required: the same terminating sample whenever the serial
    T is more than 1e-4 (relative) away from T_thresh at the crossing, and on
    every ray of a random batch; the rate inside the band is reported (DESIGN
    §5 lists it)."""
    import _ngp_native as nat
    _, _, _, ft = _setup(cuda)
    rng = np.random.default_rng(11)
    N, S, T_thresh = 4096, 128, np.float32(1e-4)
    L = -np.log(np.float64(T_thresh))
    kstar = rng.integers(2, S - 8, N)
    margin_class = rng.integers(0, 5, N)  # relative T margin ~ 9.2 x {1e-7, 1e-6, 1e-5, 1e-4, 1e-3}
    eps = np.array([1e-7, 1e-6, 1e-5, 1e-4, 1e-3])[margin_class] * rng.choice([-1.0, 1.0], N)
    c = L / (kstar + 1) * (1 + eps)  # sigma * delta per sample: T after sample kstar ~ T_thresh exp(-L eps)
    delta = np.float32(0.01)
    sig_ray = (c / delta).astype(np.float32)
    rand_rays = N // 8  # the last eighth: random densities (no engineered crossing)
    sigma = np.repeat(sig_ray, S)
    sigma[-rand_rays * S:] = rng.uniform(0, 60, rand_rays * S).astype(np.float32)
    M = N * S
    deltas = np.stack([np.full(M, delta, np.float32), np.full(M, delta, np.float32)], -1)

    def serial_stop(sig):  # fp32, the reference's order; index of the first sample with T < T_thresh, else S - 1
        # margin: how close the serial T comes to T_thresh (relative) at the
        # crossing, on either side of it (the last T above and the first below)
        T = np.ones(N, np.float32)
        stop = np.full(N, S - 1)
        margin = np.full(N, np.inf)
        done = np.zeros(N, bool)
        for k in range(S):
            sd = (sig[:, k] * delta).astype(np.float32)
            alpha = (np.float32(1) - np.exp(-sd)).astype(np.float32)
            Tp = T
            T = (T * (np.float32(1) - alpha)).astype(np.float32)
            hit = ~done & (T < T_thresh)
            stop[hit] = k
            margin[hit] = np.minimum(Tp[hit].astype(np.float64) / np.float64(T_thresh) - 1.0,
                                     1.0 - T[hit].astype(np.float64) / np.float64(T_thresh))
            done |= hit
        return stop, margin

    want, rel = serial_stop(sigma.reshape(N, S))
    col = rng.normal(0, 2, (M, 16)).astype(np.float16)
    h = rng.normal(0, 1, (M, 16)).astype(np.float16)
    rays = np.stack([np.arange(N), np.arange(N) * S, np.full(N, S)], -1).astype(np.int32)
    gt = rng.uniform(0, 1, (N, 4)).astype(np.float32)
    bg = rng.uniform(0, 1, (N, 3)).astype(np.float32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    d_sigma, d_col, d_h, d_del, d_rays, d_gt, d_bg = map(t, (sigma, col, h, deltas, rays, gt, bg))
    g_col = torch.zeros(M, 16, dtype=torch.float16, device=cuda)
    g_h = torch.zeros(M, 16, dtype=torch.float16, device=cuda)
    img = torch.zeros(N, 3, device=cuda)
    ws_out = torch.zeros(N, device=cuda)
    loss = torch.zeros(N, device=cuda)
    P = nat.ptr
    nat.check(nat.lib().ngp_nerf_composite_loss(
        P(d_sigma), P(d_col), P(d_h), P(d_del), P(d_rays), M, N, float(T_thresh), 1.0, P(d_gt), 4, P(d_bg),
        P(ft.state), P(g_col), P(g_h), P(img), P(ws_out), P(loss), nat.stream_of(img)), "composite_loss")
    torch.cuda.synchronize()
    nz = lambda g: ((g.view(torch.int16) & 0x7fff) != 0).any(1).cpu().numpy()  # noqa: E731
    live = (nz(g_h) | nz(g_col)).reshape(N, S)  # the live-row set: a nonzero gradient in some component
    assert live[:, 0].all()  # every ray's first sample carries a gradient
    got = S - 1 - np.argmax(live[:, ::-1], axis=1)  # last live row: every row past it is exactly zero
    assert live.sum(1).mean() >= 0.99 * (got + 1).mean()  # (a row before it is zero only by underflow)
    eng = np.arange(N) < N - rand_rays
    far = eng & (rel > 1e-4)
    assert far.sum() > N // 3
    bad_far = far & (got != want)
    bf = np.argwhere(bad_far).ravel()[:6]
    assert not bad_far.any(), (int(bad_far.sum()), [(int(r), int(got[r]), int(want[r]), int(kstar[r]),
                                                      float(rel[r]), float(eps[r])) for r in bf])
    assert (got[~eng] == want[~eng]).all()
    near = eng & ~far
    mism = near & (got != want)
    assert (np.abs(got[mism] - want[mism]) <= 1).all()  # one sample either side
    assert (rel[mism] <= 3e-5).all()  # only where the serial T is within a few fp32 ulps x samples of T_thresh
    assert (got[eng & ~mism] == want[eng & ~mism]).all()
    parity_report(f"fused composite early stop vs serial fp32: {int(far.sum())} rays with the crossing > 1e-4 "
                  f"from T_thresh and {int((~eng).sum())} random rays identical; within 1e-4: "
                  f"{int(mism.sum())}/{int(near.sum())} differ by one sample "
                  f"(largest margin among them {float(rel[mism].max()) if mism.any() else 0.0:.2e})")


def test_long_run_stays_finite_without_overflow(cuda):
    """400 captured steps at the bench configuration: the loss stays finite and
    GradScaler does not spiral down (before the composite's exclusive-prefix fix,
    large trained densities made runs overflow and spiral into NaN losses;
    tools/stability.py runs the longer multi-seed version)."""
    from nerf.fused import FusedTrainer
    from nerf.network_ff import NeRFNetwork
    from nerf.provider import SyntheticLego, lego_bitfield
    torch.manual_seed(3)
    m = NeRFNetwork(bound=1, cuda_ray=True).to(cuda)
    m.density_bitfield.copy_(torch.from_numpy(lego_bitfield()).to(cuda))
    ft = FusedTrainer(m, SyntheticLego(cuda, num_rays=4096), M=101762, seed=3)
    ft.capture()
    for _ in range(400):
        ft.step()
    torch.cuda.synchronize()
    assert ft.scale == 65536.0  # no GradScaler backoff (the overflow spiral's first symptom)
    assert np.isfinite(ft.last_loss) and ft.last_loss < 0.01
    assert torch.isfinite(ft.flat_param).all()


def test_grid_forward_fp32_table_equals_fp16_copy(cuda):
    """World 1 feeds the grid forward the fp32 table (each value rounded to half
    on load) instead of an fp16 copy: bit-identical encodings."""
    import _ngp_native as nat
    from nerf.fused import _F16, _F32
    _, _, _, ft = _setup(cuda)
    ft._sample()
    ft._march()
    e, m, P = ft.enc, ft.model, nat.ptr
    outs = []
    for table, dt in ((ft.params[0].detach(), _F32), (ft.params[0].detach().half(), _F16)):
        out = torch.full_like(ft.enc_out, float("nan"))
        nat.check(nat.lib().ngp_grid_encode_forward_fused(
            P(ft.xyzs), float(m.bound), P(table), dt, P(e.offsets), P(out), ft.M, P(ft.counter), e.input_dim,
            e.level_dim, e.num_levels, ft.S, e.base_resolution, e.gridtype_id, int(e.align_corners), e.interp_id,
            0, nat.stream_of(out)), "grid_encode_fused")
        outs.append(out)
    torch.cuda.synchronize()
    n = int(ft.counter[0])
    # out_layout 0: [L, M, C] (the sigma MLP reads it pair-major); rows past n are not computed
    outs = [o.view(e.num_levels, ft.M, e.level_dim)[:, :n] for o in outs]
    assert n > 0 and torch.isfinite(outs[0].float()).all()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("bound,dt_gamma", [(1, 0.0), (2, 1 / 128)])
def test_one_launch_forward_equals_split_forward(cuda, bound, dt_gamma):
    """ngp_nerf_forward (sigma + colour networks in one launch) against the
    two launches (ngp_nerf_sigma_forward + ngp_ffmlp_forward_rows) on the same
    batch: h, sigma, color_in, rgb logits, loss and the MLP gradients
    bit-identical."""
    outs = []
    for split in (True, False):
        model, ref, data, ft = _setup(cuda, bound=bound, dt_gamma=dt_gamma, options=dict(split_fwd=split))
        assert ft._one_fwd == (not split)
        ft._sample()
        ft._forward_backward()
        torch.cuda.synchronize()
        n = int(ft.counter[0])
        assert n > 0
        outs.append((n, ft.h_sigma[:n].clone(), ft.sigma[:n].clone(), ft.color_in[:n].clone(),
                     ft.color_out[:n].clone(), [g.clone() for g in ft.grads], ft.loss_ray.clone()))
    (n0, *a), (n1, *b) = outs
    assert n0 == n1
    for name, x, y in zip(["h", "sigma", "color_in", "color_out"], a[:4], b[:4]):
        assert torch.equal(x, y), name
    # MLP grads: fixed-order slab reduce; the table grad: exact bin sums
    for x, y in zip(a[4], b[4]):
        assert torch.equal(x.view(torch.int16), y.view(torch.int16))
    assert torch.equal(a[5], b[5])

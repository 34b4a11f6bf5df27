"""GPU: the benched fused train step (nerf/fused.py) against the CPU oracle.

One FusedTrainer forward + backward on a fixed batch (the fused sampler's rays,
target and background; zero march noise) and `oracle.pipeline.amp_train_step`
on the same batch and parameters (fp16 table and MLP weights, the reference's
autocast casts restated). Two comparisons:

* stage by stage: each HIP stage against the oracle applied to the HIP
  stage's own inputs (march, grid forward, sigma MLP + trunc_exp + SH glue,
  colour MLP, composite + loss + composite backward + sigmoid / trunc_exp
  backward, both MLP backwards, grid backward), so a wrong stage is named;
* end to end: the oracle run from the batch alone against the HIP outputs --
  per-sample sigma and RGB, the rendered image, the loss (north_star: 1e-3 rel)
  and the three parameter gradients.

Configs: Config 2 (Lego, bound 1, one cascade, dt_gamma 0), the Fox-shaped
Config 3 (bound 2, two cascades, dt_gamma 1/128, the bench leg's Fox-shaped
occupancy: >= 20 samples per ray, cascade-1 samples) and Config 5's single-GPU
shapes (Truck: 1920x1080 images, L16 log2T 22 = 39,625,280 table entries, the
binned backward's 1,024-bin levels with per-item flushes; bound 1).

Tolerances: HIP matmuls accumulate in fp32 (MFMA) and the oracle in float64;
both round every layer's output to fp16, so an output either matches bit for
bit or sits one fp16 rounding away (2^-11 relative) where the fp32 sum lands
near a rounding boundary, and such a flip moves later layers by a weight times
that ulp. `_close16` allows 2 fp16 ulps plus 1e-3 of the tensor's largest
magnitude (sums that cancel) and requires >= 98% of the values bit-identical.
"""
import numpy as np
import pytest
import torch

import oracle
from oracle.pipeline import amp_train_step

pytestmark = pytest.mark.gpu


def _setup(cuda, bound, dt_gamma, log2T=19, hw=(800, 800), num_rays=1024, mean_count=80000):
    from nerf.fused import FusedTrainer
    from nerf.network_ff import NeRFNetwork
    from nerf.provider import SyntheticLego, fox_bitfield, lego_bitfield
    torch.manual_seed(0)
    model = NeRFNetwork(bound=bound, cuda_ray=True, density_thresh=10, log2_hashmap_size=log2T).to(cuda)
    with torch.no_grad():  # a non-trivial field: larger table values than the 1e-4 init
        model.encoder.embeddings.normal_(0, 0.05)
    # bound 2: the Fox-shaped occupancy the bench's Config-3 leg marches (~30
    # samples per ray, cascade-1 cells); the Lego boxes at bound 2 give ~3
    occ = fox_bitfield if bound == 2 else lego_bitfield
    bits = occ(cascade=model.cascade, bound=float(bound))
    model.density_bitfield.copy_(torch.from_numpy(bits).to(cuda))
    data = SyntheticLego(cuda, H=hw[0], W=hw[1], num_rays=num_rays)
    M = mean_count + 128 - mean_count % 128
    # the table grads are materialised in grads[0] for the comparison
    return FusedTrainer(model, data, M=M, seed=3, dt_gamma=dt_gamma)


def _np(t):
    return t.detach().cpu().numpy()


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _close16(got, ref, what, min_equal=0.98, mag=None):
    """mag (backward input grads): the error scale of oracle.mlp_backward_error_bound
    (fp16 roundings of the deltas and ReLU units at the edge of zero), added
    to the tolerance."""
    got = np.asarray(got, np.float16)
    ref = np.asarray(ref, np.float16)
    assert got.shape == ref.shape, what
    g, r = got.astype(np.float64), ref.astype(np.float64)
    assert np.isfinite(g).all(), what
    tol = 2 * np.spacing(np.abs(ref)).astype(np.float64) + 1e-3 * np.abs(r).max()
    if mag is not None:
        tol = tol + mag
    bad = np.abs(g - r) > tol
    same = float((got.view(np.uint16) == ref.view(np.uint16)).mean())
    assert not bad.any(), (what, int(bad.sum()), g[bad][:6], r[bad][:6])
    assert same >= min_equal, (what, same)


def _fused_batch(ft):
    """Run the fused step's forward + backward on a fresh batch (zero march
    noise, so the oracle marches the same samples)."""
    ft._sample()
    ft.noises.zero_()
    ft._forward_backward()
    torch.cuda.synchronize()
    n = int(ft.counter[0])
    assert n <= ft.M, (n, ft.M)  # every sample fits the buffer (none dropped)
    return n


def _composite_image(ft):
    """The fused composite kernel again on the step's own inputs, with its
    optional image / weights_sum outputs (the step itself does not write them)."""
    import _ngp_native as nat
    P, N, M = nat.ptr, ft.N, ft.M
    img = torch.zeros(N, 3, device=ft.dev)
    ws = torch.zeros(N, device=ft.dev)
    gc = torch.zeros_like(ft.g_color_out)
    gh = torch.zeros_like(ft.g_h)
    loss = torch.zeros(N, device=ft.dev)
    nat.check(nat.lib().ngp_nerf_composite_loss(
        P(ft.sigma), P(ft.color_out), P(ft.h_sigma), P(ft.deltas), P(ft.rays), M, N, ft.T_thresh,
        float(ft.model.density_scale), P(ft.rgba), 4, P(ft.bg), P(ft.state), P(gc), P(gh), P(img), P(ws),
        P(loss), nat.stream_of(img)), "composite_loss")
    torch.cuda.synchronize()
    return _np(img), _np(ws), _np(gc), _np(gh), _np(loss)


def _oracle_inputs(ft):
    m = ft.model
    return dict(rays_o=_np(ft.rays_o), rays_d=_np(ft.rays_d), rgba=_np(ft.rgba), bg=_np(ft.bg),
                noises=np.zeros(ft.N, np.float32), bitfield=_np(m.density_bitfield),
                emb16=_np(ft.params[0]).astype(np.float16), offsets=_np(ft.enc.offsets),
                per_level_scale=ft.enc.per_level_scale, w_sigma16=_np(ft.w_half[1]),
                w_color16=_np(ft.w_half[2]), bound=float(m.bound), cascade=m.cascade, grid_size=m.grid_size,
                dt_gamma=ft.dt_gamma, max_steps=ft.max_steps, M=ft.M, density_scale=float(m.density_scale),
                T_thresh=ft.T_thresh, min_near=float(m.min_near), loss_scale=ft.scale)


# (bound, dt_gamma, log2T, (H, W)): Config 2, Config 3 (Fox-shaped), Config 5 (Truck)
CONFIGS = [(1, 0.0, 19, (800, 800)), (2, 1 / 128, 19, (800, 800)), (1, 0.0, 22, (1080, 1920))]
IDS = ["lego", "fox", "truck"]


@pytest.mark.parametrize("bound,dt_gamma,log2T,hw", CONFIGS, ids=IDS)
def test_fused_step_stages_match_oracle(cuda, parity_report, bound, dt_gamma, log2T, hw):
    ft = _setup(cuda, bound, dt_gamma, log2T, hw)
    if bound == 1:  # SURVEY §8 table sizes (bound 2 has a finer desired resolution)
        assert ft.enc.embeddings.shape[0] == (39625280 if log2T == 22 else 6119864)
    n = _fused_batch(ft)
    assert n > 1000
    if bound == 2:  # Config 3 marches: >= 20 samples / ray, some in cascade 1 (|x|max > 1, mip_from_pos)
        assert n >= 20 * ft.N, n / ft.N
        outer = int((np.abs(_np(ft.xyzs)[:n]).max(-1) > 1.0).sum())
        assert outer > 0.05 * n, outer
    inp = _oracle_inputs(ft)
    # ---- march (bit-exact: counts, ray offsets, samples)
    aabb = np.array([-bound] * 3 + [bound] * 3, np.float32)
    nears, fars = oracle.near_far_from_aabb(inp["rays_o"], inp["rays_d"], aabb, inp["min_near"])
    assert np.array_equal(_np(ft.nears).view(np.uint32), nears.view(np.uint32))
    assert np.array_equal(_np(ft.fars).view(np.uint32), fars.view(np.uint32))
    xyzs, dirs, deltas, rays, cnt = oracle.march_rays_train(
        inp["rays_o"], inp["rays_d"], float(bound), inp["bitfield"], ft.model.cascade, ft.model.grid_size,
        nears, fars, inp["noises"], M=ft.M, dt_gamma=dt_gamma)
    assert int(cnt[0]) == n and int(cnt[1]) == ft.N
    assert np.array_equal(_np(ft.rays), rays)
    for a, b in ((ft.xyzs, xyzs), (ft.dirs, dirs), (ft.deltas, deltas)):
        assert np.array_equal(_np(a)[:n].view(np.uint32), b[:n].view(np.uint32))
    # ---- grid forward on the HIP samples (bit-exact fp16, [L, M, 2] level-major)
    x01 = ((xyzs[:n] + np.float32(bound)) * np.float32(1.0 / (2.0 * bound))).astype(np.float32)
    enc_ref, _ = oracle.grid_encode_forward(x01, inp["emb16"], inp["offsets"], inp["per_level_scale"], 16)
    enc = _np(ft.enc_out).reshape(16, ft.M, 2)[:, :n].transpose(1, 0, 2).reshape(n, 32)
    assert np.array_equal(enc.view(np.uint16), enc_ref.view(np.uint16))
    # ---- sigma MLP + glue (trunc_exp * density_scale, SH, cat, cast)
    h = _np(ft.h_sigma)[:n]
    h_ref, _ = oracle.mlp_forward(enc, inp["w_sigma16"], 32, 16, 64, 2)
    _close16(h, h_ref, "sigma mlp")
    sig = _np(ft.sigma)[:n]
    np.testing.assert_allclose(sig, inp["density_scale"] * np.exp(h[:, 0].astype(np.float64)), rtol=1e-6)
    cin = _np(ft.color_in)[:n]
    cin_ref = np.concatenate([oracle.sh_encode(dirs[:n], 4).astype(np.float16), h[:, 1:16],
                              np.zeros((n, 1), np.float16)], -1)
    _close16(cin, cin_ref, "color_in", min_equal=0.999)
    # ---- colour MLP
    cout = _np(ft.color_out)[:n]
    cout_ref, _ = oracle.mlp_forward(cin, inp["w_color16"], 32, 16, 64, 3)
    _close16(cout, cout_ref, "color mlp")
    # ---- composite + loss + backward to the MLP outputs
    rgb = (1.0 / (1.0 + np.exp(-cout[:, :3].astype(np.float32)))).astype(np.float16).astype(np.float32)
    ws_ref, dp_ref, img_ref = oracle.composite_rays_train_forward(sig, rgb, deltas[:n], rays, ft.T_thresh)
    img, ws, gc, gh, loss_ray = _composite_image(ft)
    bg, rgba = inp["bg"], inp["rgba"]
    pred_ref = img_ref + (1 - ws_ref)[:, None] * bg
    gt = rgba[:, :3] * rgba[:, 3:] + bg * (1 - rgba[:, 3:])
    np.testing.assert_allclose(ws, ws_ref, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(img, pred_ref, rtol=1e-5, atol=1e-6)
    loss_ref = float(np.mean(np.mean((pred_ref.astype(np.float64) - gt) ** 2, -1)))
    assert abs(float(loss_ray.astype(np.float64).sum()) / ft.N - loss_ref) <= 1e-5 * loss_ref
    assert np.array_equal(gc, _np(ft.g_color_out)) and np.array_equal(gh[:, 0], _np(ft.g_h)[:, 0])
    N, S = ft.N, inp["loss_scale"]
    g_pred = (S * 2.0 / (3.0 * N)) * (pred_ref.astype(np.float64) - gt)
    g_ws = (-(g_pred * bg).sum(-1)).astype(np.float32)
    g_sig, g_rgb = oracle.composite_rays_train_backward(g_ws, np.zeros(N, np.float32), g_pred.astype(np.float32),
                                                        sig, rgb, deltas[:n], rays, ws_ref, dp_ref, img_ref,
                                                        ft.T_thresh)
    gc_ref = np.zeros((n, 16), np.float16)
    gc_ref[:, :3] = (g_rgb.astype(np.float16).astype(np.float32) * (1 - rgb) * rgb).astype(np.float16)
    gh0_ref = ((g_sig * np.float32(inp["density_scale"])) *
               np.exp(np.clip(h[:, 0].astype(np.float32), -15, 15))).astype(np.float16)
    # per-sample d loss / d (colour logits), d loss / d (log density): 1e-3 rel
    for got, ref, what in ((gc[:n], gc_ref, "grad rgb logits"), (gh[:n, 0], gh0_ref, "grad sigma logit")):
        g64, r64 = got.astype(np.float64), ref.astype(np.float64)
        assert _rel(g64, r64) <= 1e-3, (what, _rel(g64, r64))
        tol = 1e-3 * np.abs(r64) + 1e-3 * np.abs(r64).max()
        assert (np.abs(g64 - r64) <= tol).all(), (what, np.abs(g64 - r64).max())
    # ---- colour MLP backward: geo-feature grads into g_h[:, 1:16], dW
    gh_full = _np(ft.g_h)[:n]
    gcin_ref, gwc_ref = oracle.mlp_backward(gc[:n], cin, inp["w_color16"], 32, 16, 64, 3)
    mag_c, flip_c = oracle.mlp_backward_error_bound(gc[:n], cin, inp["w_color16"], 32, 16, 64, 3)
    mag_c = 4 * 2.0 ** -11 * mag_c + flip_c
    _close16(gh_full[:, 1:16], gcin_ref[:, 16:31], "color mlp grad_inputs", mag=mag_c[:, 16:31])
    gw_color = _np(ft.grads[2]).astype(np.float64)
    assert _rel(gw_color, gwc_ref) <= 1e-3, _rel(gw_color, gwc_ref)
    # ---- sigma MLP backward: encoding grads ([L, M, 2]) and dW
    genc = _np(ft.g_enc).reshape(16, ft.M, 2)[:, :n].transpose(1, 0, 2).reshape(n, 32)
    genc_ref, gws_ref = oracle.mlp_backward(gh_full, enc, inp["w_sigma16"], 32, 16, 64, 2)
    mag_s, flip_s = oracle.mlp_backward_error_bound(gh_full, enc, inp["w_sigma16"], 32, 16, 64, 2)
    mag_s = 3 * 2.0 ** -11 * mag_s + flip_s
    _close16(genc, genc_ref, "sigma mlp grad_inputs", mag=mag_s)
    gw_sigma = _np(ft.grads[1]).astype(np.float64)
    assert _rel(gw_sigma, gws_ref) <= 1e-3, _rel(gw_sigma, gws_ref)
    # ---- grid backward: fp16 table grad against the exact (float64 products)
    # scatter of the HIP encoding grads. The reference rounds every w * g to
    # half before its atomic (gridencoder.cu:322-328); the HIP path rounds run
    # sums / exact fixed-point bin sums once, so both sit
    # within fp16 rounding of the exact sum, and terms too small for a half
    # still count here
    gemb = _np(ft.grads[0]).astype(np.float64)
    gemb_ref = oracle.grid_encode_backward(genc.astype(np.float64), x01, inp["offsets"], 2,
                                           inp["per_level_scale"], 16)
    assert _rel(gemb, gemb_ref) <= 1e-3, _rel(gemb, gemb_ref)
    tol = 4e-3 * np.abs(gemb_ref) + 1e-3 * np.abs(gemb_ref).max()
    assert (np.abs(gemb - gemb_ref) <= tol).all(), np.abs(gemb - gemb_ref).max()
    assert np.all(gemb[gemb_ref == 0] == 0)  # nothing lands where no sample contributed
    parity_report(f"bound {bound} dt_gamma {dt_gamma:g} log2T {log2T} {hw[1]}x{hw[0]}: {n} samples, march/grid fwd "
                  f"bit-exact, d_rgb_logit rel {_rel(gc[:n], gc_ref):.1e}, d_sigma_logit rel "
                  f"{_rel(gh[:n, 0], gh0_ref):.1e}, dW color {_rel(gw_color, gwc_ref):.1e} sigma "
                  f"{_rel(gw_sigma, gws_ref):.1e}, table grad {_rel(gemb, gemb_ref):.1e}")


@pytest.mark.parametrize("bound,dt_gamma,log2T,hw", CONFIGS, ids=IDS)
def test_fused_step_end_to_end_matches_oracle(cuda, parity_report, bound, dt_gamma, log2T, hw):
    """north_star: rendered RGB / sigma within 1e-3 rel of the reference,
    sample counts / indices bit-exact; the oracle runs from the batch alone."""
    ft = _setup(cuda, bound, dt_gamma, log2T, hw)
    n = _fused_batch(ft)
    ref = amp_train_step(**_oracle_inputs(ft))
    assert int(ref["counter"][0]) == n and np.array_equal(_np(ft.rays), ref["rays"])
    # per-sample sigma and rgb (the MLP outputs agree bit for bit except at
    # fp16 rounding flips, see the module docstring)
    sig = _np(ft.sigma)[:n]
    assert _rel(sig, ref["sigma"]) <= 1e-3, _rel(sig, ref["sigma"])
    within = np.abs(sig - ref["sigma"]) <= 1e-3 * np.abs(ref["sigma"])
    assert within.mean() >= 0.99, within.mean()
    cout = _np(ft.color_out)[:n, :3].astype(np.float32)
    rgb = (1.0 / (1.0 + np.exp(-cout))).astype(np.float16).astype(np.float32)
    assert _rel(rgb, ref["rgb"]) <= 1e-3, _rel(rgb, ref["rgb"])
    assert (np.abs(rgb - ref["rgb"]) <= 1e-3 * np.abs(ref["rgb"])).mean() >= 0.99
    # rendered image (with background) and loss
    img, ws, _, _, loss_ray = _composite_image(ft)
    assert (np.abs(img - ref["pred"]) <= 1e-3 * np.abs(ref["pred"]) + 1e-6).all(), \
        np.abs(img - ref["pred"]).max()
    assert (np.abs(ws - ref["ws"]) <= 1e-3 * np.abs(ref["ws"]) + 1e-6).all()
    loss = float(loss_ray.astype(np.float64).sum()) / ft.N
    assert abs(loss - ref["loss"]) <= 1e-3 * ref["loss"], (loss, ref["loss"])
    report = {"samples": n, "sigma_rel": _rel(sig, ref["sigma"]), "rgb_rel": _rel(rgb, ref["rgb"]),
              "image_max_abs": float(np.abs(img - ref["pred"]).max()),
              "loss_rel": abs(loss - ref["loss"]) / ref["loss"]}
    # parameter gradients (loss-scaled fp16) against the oracle's float64 chain
    for got, want, what in ((ft.grads[0], ref["g_emb"], "embeddings"), (ft.grads[1], ref["gw_sigma"], "sigma_net"),
                            (ft.grads[2], ref["gw_color"], "color_net")):
        g = _np(got).astype(np.float64).reshape(want.shape)
        assert np.isfinite(g).all() and np.abs(want).max() > 0, what
        report[f"grad_{what}_rel"] = _rel(g, want)
        assert _rel(g, want) <= 5e-3, (what, _rel(g, want))
    parity_report(f"bound {bound} dt_gamma {dt_gamma:g} log2T {log2T} {hw[1]}x{hw[0]}: "
                  + ", ".join(f"{k} {v:.2e}" if isinstance(v, float) else f"{k} {v}" for k, v in report.items()))

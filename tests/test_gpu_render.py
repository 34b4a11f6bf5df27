"""GPU: the device-driven test render (nerf/fused_render.py) against the
reference-API inference loop (NeRFRenderer.run_cuda with training off: the
host loop over march_rays / network / composite_rays with
rays_alive[rays_alive >= 0] compaction, renderer.py:376-426).

Both march the same rays with the same bitfield and evaluate the same network
(fp16 table and MLPs under autocast): per-sample values agree bit for bit
except at fp16 rounding flips of the MLP outputs (tests/test_gpu_e2e_oracle.py),
so the images agree to 1e-3 (north_star) everywhere but on rays whose
T < T_thresh termination a flip moves by one sample.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _trained(cuda, bound=1, dt_gamma=0.0, steps=150):
    from nerf.fused import FusedTrainer
    from nerf.network_ff import NeRFNetwork
    from nerf.provider import SyntheticLego, fox_bitfield, lego_bitfield
    torch.manual_seed(0)
    model = NeRFNetwork(bound=bound, cuda_ray=True, density_thresh=10).to(cuda)
    bits = lego_bitfield() if bound == 1 else fox_bitfield()
    model.density_bitfield.copy_(torch.from_numpy(bits).to(cuda))
    data = SyntheticLego(cuda, num_rays=4096)
    ft = FusedTrainer(model, data, M=200000 if bound == 1 else 300000, seed=1, dt_gamma=dt_gamma)
    ft.run(steps)  # a partly trained field: rays terminate (T < T_thresh) as in a test render
    ft.flush()
    torch.cuda.synchronize()
    model.eval()
    return model, data


def _rays(data, H, W, pose=7):
    from nerf.utils import get_rays
    intr = data.intrinsics * np.array([W / data.W, H / data.H, W / data.W, H / data.H], np.float32)
    r = get_rays(data.poses[pose:pose + 1], intr, H, W, -1)
    return r["rays_o"], r["rays_d"]


def _compare(ref, got, what):
    ri, gi = ref["image"].reshape(-1, 3).float(), got["image"].reshape(-1, 3).float()
    assert torch.isfinite(gi).all(), what
    d = (ri - gi).abs().max(-1).values
    frac_close = float((d <= 1e-3).float().mean())
    assert frac_close >= 0.999, (what, frac_close, float(d.max()))
    assert float(d.mean()) <= 1e-4, (what, float(d.mean()))
    rd, gd = ref["depth"].reshape(-1), got["depth"].reshape(-1)
    fin = torch.isfinite(rd)
    assert torch.equal(fin, torch.isfinite(gd)), what
    assert float(((rd[fin] - gd[fin]).abs() <= 1e-3).float().mean()) >= 0.999, what
    return frac_close, float(d.max())


@pytest.mark.parametrize("bound,dt_gamma", [(1, 0.0), (2, 1 / 128)], ids=["lego", "fox"])
def test_fused_render_matches_reference_loop(cuda, parity_report, bound, dt_gamma):
    from nerf.fused_render import FusedRenderer
    model, data = _trained(cuda, bound, dt_gamma)
    H = W = 256
    ro, rd = _rays(data, H, W)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        ref = model.render(ro, rd, staged=True, bg_color=1, perturb=False, dt_gamma=dt_gamma, max_steps=1024)
    r = FusedRenderer(model, H * W, dt_gamma=dt_gamma)
    r.load_weights()
    r.capture()
    got = r.render(ro, rd, bg_color=1)
    torch.cuda.synchronize()
    ws = got["weights_sum"]
    assert float(ws.max()) > 0.5 and float(ws.min()) < 0.5  # opaque and see-through rays
    frac, dmax = _compare(ref, got, "graph")
    parity_report(f"bound {bound} dt_gamma {dt_gamma:g} {W}x{H}: {frac:.5f} of pixels within 1e-3, "
                  f"max |d| {dmax:.2e}, {r.iterations} device iterations")


def test_fused_render_graph_equals_eager_and_repeats(cuda):
    """The captured loop equals the eager launches bit for bit, and a second
    render of the same rays gives the same image (the alive list's order is
    unspecified, per-ray results are not)."""
    from nerf.fused_render import FusedRenderer
    model, data = _trained(cuda)
    H = W = 128
    ro, rd = _rays(data, H, W, pose=31)
    a = FusedRenderer(model, H * W, iters_per_graph=4)
    a.load_weights()
    eager = a.render(ro, rd)
    e_img = eager["image"].clone()
    a.capture()
    g1 = a.render(ro, rd)["image"].clone()
    g2 = a.render(ro, rd)["image"].clone()
    assert torch.equal(e_img, g1) and torch.equal(g1, g2)


def test_fused_render_empty_and_max_steps(cuda):
    """Edge cases: rays that miss the bound (near = far = FLT_MAX) end in the
    first iteration with the background; a tiny max_steps stops the loop with
    rays still alive, as the reference's `while step < max_steps`."""
    from nerf.fused_render import FusedRenderer
    model, data = _trained(cuda, steps=20)
    N = 1024
    ro = torch.tensor([[0.0, -5.0, 0.0]], device=cuda).expand(N, 3).contiguous()
    rd = torch.tensor([[0.0, 0.0, 1.0]], device=cuda).expand(N, 3).contiguous()  # parallel to the box, outside
    r = FusedRenderer(model, N)
    r.load_weights()
    out = r.render(ro, rd, bg_color=0.25)
    assert torch.equal(out["image"], torch.full_like(out["image"], 0.25))
    assert float(out["weights_sum"].abs().max()) == 0.0
    ro2, rd2 = _rays(data, 32, 32)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        ref = model.render(ro2, rd2, bg_color=1, perturb=False, max_steps=3)
    r2 = FusedRenderer(model, 32 * 32, max_steps=3)
    r2.load_weights()
    _compare(ref, r2.render(ro2, rd2), "max_steps 3")

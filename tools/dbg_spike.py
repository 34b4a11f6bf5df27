"""Fused eager run of one seed: at each step, which buffer first holds a
non-finite / outsized value (forward intermediates and grads)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch
from nerf.fused import FusedTrainer
from nerf.network_ff import NeRFNetwork
from nerf.provider import SyntheticLego, lego_bitfield
dev = torch.device("cuda:0")
seed = int(sys.argv[2]); steps = int(sys.argv[1])
torch.manual_seed(seed)
m = NeRFNetwork(bound=1, cuda_ray=True).to(dev)
m.density_bitfield.copy_(torch.from_numpy(lego_bitfield()).to(dev))
ft = FusedTrainer(m, SyntheticLego(dev, num_rays=4096), M=101762, seed=seed)
offs = m.encoder.offsets.cpu().tolist()
losses = []
for i in range(steps):
    ft.step(); torch.cuda.synchronize()
    n = int(ft.counter[0])
    sf = ft._state_f(); si = ft._state_i()
    losses.append(float(sf[2]))
    rep = {}
    for name in ("enc_out", "h_sigma", "sigma", "color_in", "color_out", "g_color_out", "g_h", "g_enc"):
        t = getattr(ft, name)[:n].float()
        bad = int((~torch.isfinite(t)).sum())
        rep[name] = (bad, round(float(t[torch.isfinite(t)].abs().max()), 3) if t.numel() else 0)
    for name, g in zip(("g_emb", "g_sig", "g_col"), ft.grads):
        t = g.float()
        fin = torch.isfinite(t)
        rep[name] = (int((~fin).sum()), round(float(t[fin].abs().max()), 2))
    anybad = any(v[0] for v in rep.values())
    if i % 20 == 0 or anybad:
        print(i, "n", n, "scale", float(sf[0]), "inf", int(si[5]), "loss", losses[-1], rep, flush=True)
    if anybad:
        t = ft.grads[0].float()
        idx = (~torch.isfinite(t)).nonzero().view(-1)[:8].cpu().tolist() if t.dim() == 1 else \
            (~torch.isfinite(t)).nonzero()[:8].cpu().tolist()
        print("  bad emb grad idx", idx, "offsets", offs)
        big = (t.abs() > 60000).nonzero()[:8].cpu().tolist()
        print("  big emb grad idx", big)
        if rep["g_enc"][0] or rep["g_h"][0]:
            ge = ft.g_enc[:n].float(); r = (~torch.isfinite(ge)).any(-1).nonzero().view(-1)[:5].cpu().tolist()
            print("  bad g_enc rows", r, "sigma", ft.sigma[r].tolist(), "h", ft.h_sigma[r].float().tolist()[:2])
        if i > 3 and sum(1 for v in rep.values() if v[0]) and rep["loss" if False else "sigma"][0]:
            break
    if losses[-1] != losses[-1]:
        print("loss nan at", i); break

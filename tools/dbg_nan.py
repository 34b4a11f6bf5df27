"""Where does a long fused training run go non-finite? Per-step state dump."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch
from nerf.fused import FusedTrainer
from nerf.network_ff import NeRFNetwork
from nerf.provider import SyntheticLego, lego_bitfield
dev = torch.device("cuda:0"); torch.manual_seed(0)
model = NeRFNetwork(bound=1, cuda_ray=True).to(dev)
model.density_bitfield.copy_(torch.from_numpy(lego_bitfield()).to(dev))
data = SyntheticLego(dev, num_rays=4096)
ft = FusedTrainer(model, data, M=101762)
graph = len(sys.argv) > 2 and sys.argv[2] == "graph"
if graph:
    ft.capture()
n = int(sys.argv[1])
prev = None
for i in range(n):
    ft.step()
    torch.cuda.synchronize()
    si, sf = ft._state_i(), ft._state_f()
    pf = [bool(torch.isfinite(t).all()) for t in (ft.flat_param, ft.flat_half.float())]
    gf = bool(torch.isfinite(ft.flat_grad.float()).all())
    row = (i, round(float(sf[0]), 1), int(si[5]), int(si[6]), round(float(sf[2]), 6), pf, gf, int(ft.counter[0]))
    if i % 25 == 0 or not all(pf) or not gf or (prev and prev[1] != row[1]):
        print(row, flush=True)
    if not all(pf):
        print("params went non-finite at step", i)
        for name, t in zip(["emb", "sig", "col"], ft.grads):
            print(name, "grad nonfinite", int((~torch.isfinite(t.float())).sum()))
        break
    prev = row

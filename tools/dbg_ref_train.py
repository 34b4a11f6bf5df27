"""The same long run through the reference-API autograd step (torch Adam +
GradScaler): does it overflow / go non-finite too?"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch
from nerf.network_ff import NeRFNetwork
from nerf.provider import SyntheticLego, lego_bitfield
from nerf.train import Trainer
dev = torch.device("cuda:0"); torch.manual_seed(int(sys.argv[2]) if len(sys.argv) > 2 else 0)
model = NeRFNetwork(bound=1, cuda_ray=True).to(dev)
model.density_bitfield.copy_(torch.from_numpy(lego_bitfield()).to(dev))
model.mean_count = 101762
data = SyntheticLego(dev, num_rays=4096)
tr = Trainer(model, data, update_density=False)
prev = None
for i in range(int(sys.argv[1])):
    loss = float(tr.train_step())
    sc = tr.scaler.get_scale()
    pf = all(bool(torch.isfinite(p).all()) for p in model.parameters())
    if i % 25 == 0 or sc != prev or loss != loss or not pf:
        h = None
        print((i, sc, round(loss, 6), pf), flush=True)
    prev = sc
    if not pf:
        print("params non-finite at", i); break

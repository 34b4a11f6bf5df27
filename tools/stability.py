"""Long-run stability: fused step (eager / graph) vs the reference-API autograd step, several
seeds; reports the first overflow (GradScaler backoff) and the first
non-finite loss / parameter of each run."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch
from nerf.fused import FusedTrainer
from nerf.network_ff import NeRFNetwork
from nerf.provider import SyntheticLego, lego_bitfield
from nerf.train import Trainer
dev = torch.device("cuda:0")
steps = int(sys.argv[1]); seeds = [int(s) for s in sys.argv[2].split(",")]; engines = sys.argv[3].split(",")


def make(seed):
    torch.manual_seed(seed)
    m = NeRFNetwork(bound=1, cuda_ray=True).to(dev)
    m.density_bitfield.copy_(torch.from_numpy(lego_bitfield()).to(dev))
    return m


for eng in engines:
    for seed in seeds:
        m = make(seed)
        data = SyntheticLego(dev, num_rays=4096)
        first_ovf = first_nan = None
        if eng == "autograd":
            m.mean_count = 101762
            tr = Trainer(m, data, update_density=False)
            prev = tr.scaler.get_scale()
        else:
            tr = FusedTrainer(m, data, M=101762, seed=seed)
            if eng == "graph":
                tr.capture()
            prev = 65536.0
        gmax = []
        for i in range(steps):
            if eng == "autograd":
                loss = float(tr.train_step()); sc = tr.scaler.get_scale()
                g = [float(p.grad.abs().max()) / sc if p.grad is not None else 0.0 for p in m.parameters()]
            else:
                tr.step(); torch.cuda.synchronize()
                si, sf = tr._state_i(), tr._state_f()
                sc = float(sf[0]); loss = float(sf[2])
                g = [float(t.float().abs().max()) / sc for t in tr.grads]
            if i % 100 == 0:
                gmax.append([round(x, 4) for x in g])
            if sc < prev and first_ovf is None:
                first_ovf = i
            prev = sc
            if loss != loss and first_nan is None:
                first_nan = i
                break
        pf = all(bool(torch.isfinite(p).all()) for p in m.parameters()) if eng == "autograd" else \
            bool(torch.isfinite(tr.flat_param).all())
        print(eng, seed, "first_ovf", first_ovf, "first_nan", first_nan, "scale", prev, "params_finite", pf,
              "gmax/100", gmax, flush=True)

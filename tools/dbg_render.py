import os, sys
ROOT = "/root/repo"
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd"), os.path.join(ROOT, "tools")]
import torch, raymarching
from nerf.fused import FusedTrainer
from nerf.network_ff import NeRFNetwork
from nerf.provider import SyntheticLego, lego_bitfield
from nerf.utils import get_rays
dev = torch.device("cuda:0"); torch.manual_seed(0)
model = NeRFNetwork(bound=1, cuda_ray=True).to(dev)
model.density_bitfield.copy_(torch.from_numpy(lego_bitfield()).to(dev))
data = SyntheticLego(dev, num_rays=4096)
ft = FusedTrainer(model, data, M=101762)
for _ in range(int(sys.argv[1])): ft.step()
ft.flush(); torch.cuda.synchronize()
print("params finite", [bool(torch.isfinite(p).all()) for p in model.parameters()], "loss", ft.last_loss)
model.eval()
rays = get_rays(data.poses[7:8], data.intrinsics, data.H, data.W, -1)
ro, rd = rays["rays_o"].view(-1, 3).contiguous(), rays["rays_d"].view(-1, 3).contiguous()
N = ro.shape[0]
with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
    nears, fars = raymarching.near_far_from_aabb(ro, rd, model.aabb_infer, model.min_near)
    print("nears finite", bool(torch.isfinite(nears).all()), float(nears.min()), float(fars.max()), "miss", int((nears >= fars).sum()))
    ws = torch.zeros(N, device=dev); depth = torch.zeros(N, device=dev); image = torch.zeros(N, 3, device=dev)
    alive = torch.arange(N, dtype=torch.int32, device=dev); rt = nears.clone(); step = 0; it = 0
    while step < 1024:
        na = alive.shape[0]
        if na <= 0: break
        ns = max(min(N // na, 8), 1)
        xyzs, dirs, deltas = raymarching.march_rays(na, ns, alive, rt, ro, rd, model.bound, model.density_bitfield, model.cascade, model.grid_size, nears, fars, 128, False, 0.0, 1024)
        s, c = model(xyzs, dirs)
        s = model.density_scale * s
        bad = lambda t: int((~torch.isfinite(t.float())).sum())
        if it < 6 or bad(s) or bad(c) or bad(image):
            print(it, na, ns, "xyz", bad(xyzs), "deltas", bad(deltas), "sig", bad(s), float(s.float().max()), "rgb", bad(c), "img", bad(image), "ws", bad(ws), "rt", bad(rt))
        raymarching.composite_rays(na, ns, alive, rt, s, c, deltas, ws, depth, image, 1e-4)
        if bad(image):
            print("image went bad at it", it); break
        alive = alive[alive >= 0]; step += ns; it += 1
    print("iters", it, "img bad", bad(image), "ws range", float(ws.min()), float(ws.max()))
with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
    for k in range(6):
        out = model.render(rays["rays_o"], rays["rays_d"], staged=True, bg_color=1, perturb=False, dt_gamma=0.0, max_steps=1024)
        torch.cuda.synchronize()
        im = out["image"].float()
        nb = ~torch.isfinite(im).all(-1)[0]
        print("render", k, "bad px", int(nb.sum()), "dtype", out["image"].dtype, "depth bad", int((~torch.isfinite(out["depth"])).sum()))
        if nb.any():
            idx = nb.nonzero()[:5, 0]
            print("  idx", idx.tolist(), im[0, idx].tolist(), "nears", nears[idx].tolist())

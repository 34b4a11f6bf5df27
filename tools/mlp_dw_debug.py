import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import numpy as np, torch
import oracle
import ffmlp.backend as fb
dev = torch.device("cuda:0")
rng = np.random.default_rng(0)
for B in (32, 64, 4112):
    in_dim, hidden, nl = 32, 64, 2
    npar = hidden * (in_dim + hidden * (nl - 1) + 16)
    w = (rng.standard_normal(npar) * 0.2).astype(np.float16)
    x = rng.standard_normal((B, in_dim)).astype(np.float16)
    g = rng.standard_normal((B, 16)).astype(np.float16)
    ref_gi, ref_gw = oracle.mlp_backward(g, x, w, in_dim, 16, hidden, nl)
    gi = torch.empty(B, in_dim, dtype=torch.half, device=dev)
    gw = torch.empty(npar, dtype=torch.float32, device=dev)
    fb._backend.ffmlp_backward(torch.from_numpy(g).to(dev), torch.from_numpy(x).to(dev), torch.from_numpy(w).to(dev),
                               None, B, in_dim, 16, hidden, nl, 0, 6, True, None, gi, gw)
    gw = gw.cpu().numpy()
    offs = [0, hidden * in_dim, hidden * in_dim + hidden * hidden, npar]
    for k, name in enumerate(["first", "hidden", "last"]):
        a, b = gw[offs[k]:offs[k + 1]], ref_gw[offs[k]:offs[k + 1]]
        print(B, name, "maxerr", float(np.abs(a - b).max()), "ref max", float(np.abs(b).max()))
    W1 = (gw[offs[2]:offs[3]]).reshape(16, hidden); R1 = ref_gw[offs[2]:offs[3]].reshape(16, hidden)
    print("last row0 got", np.round(W1[0, :8], 3), "ref", np.round(R1[0, :8], 3))

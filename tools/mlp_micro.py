"""Micro-benchmark of the fused MLP kernels (HIP events over back-to-back calls).
    NGP_HIP_LIB=<lib> python tools/mlp_micro.py [B]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch  # noqa: E402

import ffmlp.backend as fb  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 80000
dev = torch.device("cuda:0")
res = {}
for name, (i, h, nl) in {"sigma": (32, 64, 2), "color": (32, 64, 3)}.items():
    npar = h * (i + h * (nl - 1) + 16)
    w = (torch.rand(npar, device=dev) - 0.5).half() * 0.3
    x = torch.randn(B, i, device=dev).half()
    g = torch.randn(B, 16, device=dev).half()
    out = torch.empty(B, 16, device=dev, dtype=torch.half)
    gi = torch.empty(B, i, device=dev, dtype=torch.half)
    gw = torch.empty(npar, device=dev, dtype=torch.half)
    for _ in range(3):
        fb._backend.ffmlp_forward(x, w, B, i, 16, h, nl, 0, 6, None, out)
        fb._backend.ffmlp_backward(g, x, w, None, B, i, 16, h, nl, 0, 6, True, None, gi, gw)
    torch.cuda.synchronize()
    for kind in ("fwd", "bwd"):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            if kind == "fwd":
                fb._backend.ffmlp_forward(x, w, B, i, 16, h, nl, 0, 6, None, out)
            else:
                fb._backend.ffmlp_backward(g, x, w, None, B, i, 16, h, nl, 0, 6, True, None, gi, gw)
        e.record()
        torch.cuda.synchronize()
        res[f"{name}_{kind}_us"] = round(s.elapsed_time(e) / 20 * 1e3, 1)
print(os.environ.get("NGP_HIP_LIB", "default"), res)

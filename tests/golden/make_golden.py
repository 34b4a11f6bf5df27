"""Generates the golden fixtures in tests/golden/*.npz from the reference's
own CPU-runnable oracles (run once in the build container, where
/root/reference exists; the fixtures are data and travel, the reference does
not):

  * SHEncoder_torch  — testing/test_shencoder.py:8-89 (pure-torch SH, deg <= 5)
  * MLP              — testing/test_ffmlp.py:11-43 (bias-free nn.Linear stack,
                       FFMLP layer semantics)
  * trunc_exp        — activation.py:5-18

Only the class / function definitions are extracted (ast) and executed; the
scripts' module-level CUDA code never runs. Usage:
    python tests/golden/make_golden.py [/root/reference]
"""
import ast
import os
import sys

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.autograd import Function

HERE = os.path.dirname(os.path.abspath(__file__))
REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"


def extract(path, names):
    """Exec only the named top-level class/function defs of a reference file."""
    src = open(path).read()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, (ast.ClassDef, ast.FunctionDef)) and n.name in names]
    mod = ast.Module(body=keep, type_ignores=[])
    ns = {"torch": torch, "nn": nn, "F": F, "np": np, "math": __import__("math"),
          "Function": Function, "custom_fwd": torch.cuda.amp.custom_fwd,
          "custom_bwd": torch.cuda.amp.custom_bwd}
    exec(compile(mod, path, "exec"), ns)
    return ns


def sh_fixture():
    ns = extract(os.path.join(REF, "testing/test_shencoder.py"), {"SHEncoder_torch"})
    rng = np.random.default_rng(0)
    d = rng.standard_normal((512, 3))
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    d32 = d.astype(np.float32)
    out = {"inputs": d32}
    for deg in range(1, 6):
        enc = ns["SHEncoder_torch"](degree=deg)
        out[f"deg{deg}"] = enc(torch.from_numpy(d32)).numpy()
    np.savez_compressed(os.path.join(HERE, "sh_reference.npz"), **out)


def mlp_fixture():
    ns = extract(os.path.join(REF, "testing/test_ffmlp.py"), {"MLP"})
    out = {}
    for name, (i, o, h, nl) in {"sigma": (32, 16, 64, 2), "color": (32, 16, 64, 3),
                                "small": (16, 16, 32, 2)}.items():
        net = ns["MLP"](i, o, h, nl)  # reset_parameters: manual_seed(42), U(+-sqrt(3/h))
        torch.manual_seed(7)
        x = torch.randn(64, i, requires_grad=True)
        y = net(x)
        g = torch.randn_like(y)
        y.backward(g)
        flat = torch.cat([l.weight.detach().reshape(-1) for l in net.net])
        gflat = torch.cat([l.weight.grad.reshape(-1) for l in net.net])
        out[f"{name}_weights"] = flat.numpy()
        out[f"{name}_x"] = x.detach().numpy()
        out[f"{name}_y"] = y.detach().numpy()
        out[f"{name}_g"] = g.numpy()
        out[f"{name}_gx"] = x.grad.numpy()
        out[f"{name}_gw"] = gflat.numpy()
        out[f"{name}_dims"] = np.array([i, o, h, nl])
    np.savez_compressed(os.path.join(HERE, "mlp_reference.npz"), **out)


def trunc_exp_fixture():
    ns = extract(os.path.join(REF, "activation.py"), {"_trunc_exp"})
    x = torch.tensor([-30.0, -15.5, -3.0, 0.0, 1.5, 10.0, 15.0, 16.0, 20.0], requires_grad=True)
    y = ns["_trunc_exp"].apply(x)
    y.backward(torch.ones_like(y))
    np.savez_compressed(os.path.join(HERE, "trunc_exp_reference.npz"), x=x.detach().numpy(),
                        y=y.detach().numpy(), gx=x.grad.numpy())


if __name__ == "__main__":
    sh_fixture()
    mlp_fixture()
    trunc_exp_fixture()
    print("wrote", sorted(f for f in os.listdir(HERE) if f.endswith(".npz")))

"""Generates the golden fixtures in tests/golden/*.npz from the reference's
own CPU-runnable oracles (run once in the build container, where
/root/reference exists; the fixtures are data and travel, the reference does
not):

  * SHEncoder_torch  — testing/test_shencoder.py:8-89 (pure-torch SH, deg <= 5)
  * MLP              — testing/test_ffmlp.py:11-43 (bias-free nn.Linear stack,
                       FFMLP layer semantics)
  * trunc_exp        — activation.py:5-18
  * NeRFRenderer.run — nerf/renderer.py:126-254 (the pure-torch sampler and
                       compositing: uniform samples, alphas, cumprod weights,
                       weights_sum, depth, image with the white background),
                       called with upsample_steps=0, perturb=False, on a stub
                       `self` whose near/far is a torch slab test and whose
                       density / colour are an analytic field; the samples the
                       field saw and its outputs are recorded with the result
  * get_rays         — nerf/utils.py:52-136 (+ custom_meshgrid :45-49): whole
                       images (N=-1) and random pixel batches (N>0, seeded)
  * nerf_matrix_to_ngp — nerf/provider.py:19-27
  * FreqEncoder      — encoding.py:5-43 (the reference's pure-torch positional
                       encoding, the same layout as freqencoder's CUDA op with
                       max_freq_log2 = degree - 1, N_freqs = degree): outputs
                       and input grads for a seeded output grad
  * NeRFRenderer.update_extra_state / mark_untrained_grid — nerf/renderer.py
                       :433-598 (density-grid EMA, packbits, mean_density,
                       mean_count; the frustum mark) on a stub `self` with an
                       analytic density, raymarching.morton3D / _invert /
                       packbits bound to the oracle's CPU restatements; the
                       update's torch draws are served by a recording proxy
                       (below) and stored with the results

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
          "custom_bwd": torch.cuda.amp.custom_bwd, "pver": __import__("packaging.version").version}
    exec(compile(mod, path, "exec"), ns)
    return ns


def extract_method(path, cls, name, ns_extra=None):
    """Exec one method of a reference class as a plain function."""
    src = open(path).read()
    tree = ast.parse(src)
    klass = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == cls)
    fn = next(n for n in klass.body if isinstance(n, ast.FunctionDef) and n.name == name)
    fn.decorator_list = []
    mod = ast.Module(body=[fn], type_ignores=[])
    ns = {"torch": torch, "np": np, "F": F}
    ns.update(ns_extra or {})
    exec(compile(mod, path, "exec"), ns)
    return ns[name]


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


def _slab_near_far(rays_o, rays_d, aabb, min_near):
    """Stub raymarching.near_far_from_aabb for run() (torch, CPU): slab test,
    near clamped to min_near (raymarching.cu:91-145)."""
    inv = 1.0 / rays_d
    t0 = (aabb[:3] - rays_o) * inv
    t1 = (aabb[3:] - rays_o) * inv
    near = torch.minimum(t0, t1).amax(-1).clamp(min=min_near)
    far = torch.maximum(t0, t1).amin(-1)
    return near, far


def renderer_run_fixture():
    """NeRFRenderer.run (renderer.py:126-254) on an analytic field: a Gaussian
    density blob (sigma up to 40) and a position / direction dependent colour."""
    import types
    run = extract_method(os.path.join(REF, "nerf/renderer.py"), "NeRFRenderer", "run",
                         {"raymarching": types.SimpleNamespace(near_far_from_aabb=_slab_near_far)})
    rec = {}

    def density(x):
        rec["xyzs"] = x.detach().clone()
        sigma = 40.0 * torch.exp(-((x - torch.tensor([0.1, -0.05, 0.0])) ** 2).sum(-1) / 0.18)
        rec["sigma"] = sigma.detach().clone()
        return {"sigma": sigma, "geo_feat": torch.zeros(x.shape[0], 15)}

    def color(x, d, mask=None, geo_feat=None, **kw):
        rgb = torch.sigmoid(torch.stack([3 * x[:, 0] + d[:, 1], 2 * x[:, 1] - d[:, 0], x[:, 2] + 0.5 * d[:, 2]], -1))
        rec["rgb"] = rgb.detach().clone()
        return rgb

    bound = 1.0
    stub = types.SimpleNamespace(
        aabb_train=torch.tensor([-bound] * 3 + [bound] * 3), aabb_infer=torch.tensor([-bound] * 3 + [bound] * 3),
        training=True, min_near=0.2, density_scale=1.0, bg_radius=-1, density=density, color=color)
    g = torch.Generator().manual_seed(5)
    N, T = 96, 128
    cam = torch.tensor([0.3, -3.0, 0.8])
    tgt = (torch.rand(N, 3, generator=g) - 0.5) * 1.2
    rays_d = tgt - cam
    rays_d = rays_d / rays_d.norm(dim=-1, keepdim=True)
    rays_o = cam.expand(N, 3).contiguous()
    with torch.no_grad():
        out = run(stub, rays_o[None], rays_d[None], num_steps=T, upsample_steps=0, bg_color=None, perturb=False)
    nears, fars = _slab_near_far(rays_o, rays_d, stub.aabb_train, stub.min_near)
    np.savez_compressed(os.path.join(HERE, "renderer_run_reference.npz"), rays_o=rays_o.numpy(),
                        rays_d=rays_d.numpy(), nears=nears.numpy(), fars=fars.numpy(), num_steps=np.int32(T),
                        density_scale=np.float32(stub.density_scale), xyzs=rec["xyzs"].numpy(),
                        sigma=rec["sigma"].numpy(), rgb=rec["rgb"].numpy(), image=out["image"][0].numpy(),
                        weights_sum=out["weights_sum"].reshape(-1).numpy(), depth=out["depth"].reshape(-1).numpy())


def renderer_run_backward_fixture():
    """Autograd of NeRFRenderer.run's compositing (renderer.py:206-240): the
    gradients composite_rays_train_backward (raymarching.cu:601-691) and the
    fused composite + loss kernel must reproduce. The field is built from
    fp16-representable logits, as the fused step's MLP outputs are:
    sigma = exp(h0) (trunc_exp in range, activation.py:5-18) and
    rgb = half(sigmoid(logit)) (autocast's half sigmoid). h0 and the colour
    logits are the autograd leaves; two losses are differentiated on the same
    graph:
      * lin = sum(gI * image) + sum(gD * depth) + sum(gW * weights_sum), seeded
        gI / gD / gW (every term of the composite backward), recorded as
        d lin / d sigma and d lin / d rgb;
      * mse = mean((image - gt)^2) over rays and channels (the train step's
        MSELoss(reduction='none').mean(-1).mean(), nerf/utils.py), recorded as
        d mse / d h0 and d mse / d logit."""
    import types
    run = extract_method(os.path.join(REF, "nerf/renderer.py"), "NeRFRenderer", "run",
                         {"raymarching": types.SimpleNamespace(near_far_from_aabb=_slab_near_far)})
    rec = {}

    def density(x):
        h0 = (np.log(40.0) - ((x - torch.tensor([0.05, 0.1, -0.1])) ** 2).sum(-1) / 0.15).half().float()
        rec["h0"] = h0.detach().clone().requires_grad_(True)
        sigma = torch.exp(rec["h0"])
        rec["sigma"] = sigma
        return {"sigma": sigma, "geo_feat": torch.zeros(x.shape[0], 15)}

    def color(x, d, mask=None, geo_feat=None, **kw):
        logit = torch.stack([2 * x[:, 0] - d[:, 2], 3 * x[:, 1] + d[:, 0], -x[:, 2] + 0.7 * d[:, 1]], -1)
        rec["logit"] = logit.half().float().detach().clone().requires_grad_(True)
        rgb = torch.sigmoid(rec["logit"]).half().float()
        rec["rgb"] = rgb
        return rgb

    bound = 1.0
    stub = types.SimpleNamespace(
        aabb_train=torch.tensor([-bound] * 3 + [bound] * 3), aabb_infer=torch.tensor([-bound] * 3 + [bound] * 3),
        training=True, min_near=0.2, density_scale=1.0, bg_radius=-1, density=density, color=color)
    g = torch.Generator().manual_seed(6)
    N, T = 80, 112
    cam = torch.tensor([-0.4, -2.8, 0.9])
    tgt = (torch.rand(N, 3, generator=g) - 0.5) * 1.3
    rays_d = tgt - cam
    rays_d = rays_d / rays_d.norm(dim=-1, keepdim=True)
    rays_o = cam.expand(N, 3).contiguous()
    out = run(stub, rays_o[None], rays_d[None], num_steps=T, upsample_steps=0, bg_color=None, perturb=False)
    image, depth, ws = out["image"][0], out["depth"].reshape(-1), out["weights_sum"].reshape(-1)
    gI, gD, gW = torch.randn(N, 3, generator=g), torch.randn(N, generator=g), torch.randn(N, generator=g)
    gt = torch.rand(N, 3, generator=g)
    sigma, rgb = rec["sigma"], rec["rgb"]
    lin = (gI * image).sum() + (gD * depth).sum() + (gW * ws).sum()
    d_sigma, d_rgb = torch.autograd.grad(lin, [sigma, rgb], retain_graph=True)
    mse = ((image - gt) ** 2).mean(-1).mean()
    d_h0, d_logit = torch.autograd.grad(mse, [rec["h0"], rec["logit"]])
    nears, fars = _slab_near_far(rays_o, rays_d, stub.aabb_train, stub.min_near)
    np.savez_compressed(os.path.join(HERE, "renderer_run_backward_reference.npz"), rays_o=rays_o.numpy(),
                        rays_d=rays_d.numpy(), nears=nears.numpy(), fars=fars.numpy(), num_steps=np.int32(T),
                        density_scale=np.float32(stub.density_scale), h0=rec["h0"].detach().numpy(),
                        logit=rec["logit"].detach().numpy(), sigma=sigma.detach().numpy(),
                        rgb=rgb.detach().numpy(), image=image.detach().numpy(), depth=depth.detach().numpy(),
                        weights_sum=ws.detach().numpy(), gI=gI.numpy(), gD=gD.numpy(), gW=gW.numpy(),
                        d_sigma=d_sigma.numpy(), d_rgb=d_rgb.numpy(), gt=gt.numpy(),
                        mse=np.float32(mse.item()), d_h0=d_h0.numpy(), d_logit=d_logit.numpy())


def get_rays_fixture():
    ns = extract(os.path.join(REF, "nerf/utils.py"), {"get_rays", "custom_meshgrid"})
    rng = np.random.default_rng(11)
    poses = []
    for _ in range(3):  # random rotations + translations, cam2world
        q = np.linalg.qr(rng.standard_normal((3, 3)))[0]
        p = np.eye(4)
        p[:3, :3], p[:3, 3] = q, rng.standard_normal(3) * 2
        poses.append(p)
    poses = torch.from_numpy(np.stack(poses).astype(np.float32))
    H, W = 24, 40
    intr = np.array([37.5, 36.0, 20.3, 11.7], np.float32)
    full = ns["get_rays"](poses, intr, H, W, -1)
    torch.manual_seed(21)
    part = ns["get_rays"](poses[:1], intr, H, W, 256)
    np.savez_compressed(os.path.join(HERE, "get_rays_reference.npz"), poses=poses.numpy(), intrinsics=intr,
                        H=np.int32(H), W=np.int32(W), rays_o=full["rays_o"].numpy(), rays_d=full["rays_d"].numpy(),
                        seed=np.int32(21), N=np.int32(256), inds_part=part["inds"].numpy(),
                        rays_o_part=part["rays_o"].numpy(), rays_d_part=part["rays_d"].numpy())


def nerf_matrix_fixture():
    ns = extract(os.path.join(REF, "nerf/provider.py"), {"nerf_matrix_to_ngp"})
    rng = np.random.default_rng(12)
    poses = rng.standard_normal((6, 4, 4)).astype(np.float32)
    args = [(0.33, [0, 0, 0]), (0.8, [0, 0, 0]), (0.33, [0.1, -0.2, 0.3])]
    out = np.stack([np.stack([ns["nerf_matrix_to_ngp"](p, scale=s, offset=o) for p in poses]) for s, o in args])
    np.savez_compressed(os.path.join(HERE, "nerf_matrix_reference.npz"), poses=poses,
                        scales=np.array([a[0] for a in args], np.float32),
                        offsets=np.array([a[1] for a in args], np.float32), out=out)


def freq_fixture():
    ns = extract(os.path.join(REF, "encoding.py"), {"FreqEncoder"})
    g = torch.Generator().manual_seed(13)
    res = {}
    for deg in (4, 10):
        enc = ns["FreqEncoder"](input_dim=3, max_freq_log2=deg - 1, N_freqs=deg, log_sampling=True)
        x = (torch.rand(257, 3, generator=g) * 2 - 1).requires_grad_(True)
        y = enc(x)
        gy = torch.randn(y.shape, generator=g)
        y.backward(gy)
        res.update({f"x{deg}": x.detach().numpy(), f"y{deg}": y.detach().numpy(),
                    f"gy{deg}": gy.numpy(), f"gx{deg}": x.grad.numpy()})
    np.savez_compressed(os.path.join(HERE, "freq_reference.npz"), **res)


class _DrawProxy:
    """Stands in for the `torch` module inside the exec'd update_extra_state:
    every attribute is torch's, except the three draws, which are served from
    a seeded numpy generator and recorded in call order:
      * randint(0, H, (N, 3)): distinct cells (a random subset of H^3);
      * randint(0, n_occ, [N]): distinct occupied picks where there are enough,
        wrapping around otherwise;
      * rand_like(x): k / 2^16 with k a hash of the row's cell, cascade and
        update, so a cell drawn twice in one update gets the same noise row and
        density, and upstream's index_put (which keeps an arbitrary duplicate)
        and the build's scatter-max agree.
    The values are exactly representable, so they travel as uint16 / int32."""

    def __init__(self, seed, H, bound_of):
        self._rng = np.random.default_rng(seed)
        self._H, self._bound_of = H, bound_of
        self.draws = []
        self.update = 0
        self.cas = 0

    def __getattr__(self, name):
        return getattr(torch, name)

    def randint(self, low, high, size, **kw):
        n = int(np.prod(size))
        if len(size) == 2:  # cells
            H = self._H
            cells = self._rng.choice(H ** 3, size=size[0], replace=False)
            out = np.stack([cells // (H * H), (cells // H) % H, cells % H], -1)
        else:  # picks into the occupied list
            perm = self._rng.permutation(int(high))
            out = np.resize(perm, n)
        t = torch.from_numpy(out.astype(np.int64)).reshape(size)
        self.draws.append(("randint", out.astype(np.int32).reshape(size)))
        return t

    def rand_like(self, x):
        H = self._H
        bound = self._bound_of(self.cas)
        hgs = bound / H
        c = torch.round((x / (bound - hgs) + 1) * (H - 1) / 2).to(torch.int64).numpy()  # the rows' cells
        key = (c[:, 0] * H + c[:, 1]) * H + c[:, 2] + (self.cas * 7919 + self.update * 104729) * H ** 3
        k = np.empty((x.shape[0], 3), np.uint16)
        for j in range(3):
            h = (key * 0x9E3779B1 + (j + 1) * 0x85EBCA77) & 0xFFFFFFFF
            h ^= h >> 15
            h = (h * 0x2C1B3C6D) & 0xFFFFFFFF
            h ^= h >> 12
            k[:, j] = (h & 0xFFFF).astype(np.uint16)
        self.draws.append(("rand", k))
        self.cas += 1
        return torch.from_numpy(k.astype(np.float32) * np.float32(2.0 ** -16))


def density_fixture():
    """update_extra_state (renderer.py:498-598) x 4 (2 full, 2 partial) and
    mark_untrained_grid (:433-496) on stubs: bound 2 / cascade 2 and bound 1 /
    cascade 1, grid 16^3. The density is an analytic blob (so no network is
    involved): sigma = 30 exp(-|x - c|^2 / 0.35)."""
    import types
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE))))
    import oracle
    rm = types.SimpleNamespace(
        morton3D=lambda c: torch.from_numpy(oracle.morton3D(c.numpy())),
        morton3D_invert=lambda i: torch.from_numpy(oracle.morton3D_invert(i.numpy())),
        packbits=lambda g, th, bf: torch.from_numpy(oracle.packbits(g.numpy(), float(th))))
    util = extract(os.path.join(REF, "nerf/utils.py"), {"custom_meshgrid"})
    H = 16
    out = {"H": np.int32(H)}
    for tag, bound, thresh in (("b2", 2, 10.0), ("b1", 1, 0.5)):
        cascade = 1 + int(np.ceil(np.log2(bound)))
        proxy = _DrawProxy(17 + bound, H, lambda cas: min(2 ** cas, bound))
        ns = {"raymarching": rm, "custom_meshgrid": util["custom_meshgrid"]}
        upd = extract_method(os.path.join(REF, "nerf/renderer.py"), "NeRFRenderer", "update_extra_state", ns)
        upd.__globals__["torch"] = proxy
        mark = extract_method(os.path.join(REF, "nerf/renderer.py"), "NeRFRenderer", "mark_untrained_grid", ns)
        centre = torch.tensor([0.15, -0.1, 0.05]) * bound

        def density(x):
            return {"sigma": 30.0 * torch.exp(-((x - centre) ** 2).sum(-1) / (0.35 * bound * bound))}

        stub = types.SimpleNamespace(
            cuda_ray=True, grid_size=H, cascade=cascade, bound=bound, density_scale=1.0, density_thresh=thresh,
            density_grid=torch.zeros(cascade, H ** 3), density_bitfield=torch.zeros(cascade * H ** 3 // 8,
                                                                                     dtype=torch.uint8),
            iter_density=0, mean_density=0.0, mean_count=-1, local_step=0,
            step_counter=torch.zeros(16, 2, dtype=torch.int32), density=density)
        # mark_untrained_grid: cameras on half a ring looking at the origin
        # (narrow field of view: the far corners stay unseen)
        poses = []
        for k in range(4):
            th = np.pi * k / 3
            eye = np.array([np.cos(th), np.sin(th), 0.5]) * 2.2 * bound
            z = -eye / np.linalg.norm(eye)  # the mark's frustum test looks along +z (renderer.py:482)
            x = np.cross([0.0, 0.0, 1.0], z)
            x /= np.linalg.norm(x)
            y = np.cross(z, x)
            p = np.eye(4)
            p[:3, 0], p[:3, 1], p[:3, 2], p[:3, 3] = x, y, z, eye
            poses.append(p)
        poses = np.stack(poses).astype(np.float32)
        intr = (40.0, 40.0, 10.0, 9.0)
        mark(stub, torch.from_numpy(poses), intr, S=64)
        out[f"{tag}_poses"], out[f"{tag}_intrinsics"] = poses, np.array(intr, np.float32)
        out[f"{tag}_marked"] = stub.density_grid.numpy().copy()
        counts = np.arange(1, 17, dtype=np.int32) * 1000 + bound * 7
        for u in range(4):
            if u == 2:
                stub.iter_density = 16  # partial updates from here on
            stub.step_counter[:, 0] = torch.from_numpy(counts + u)
            stub.local_step = (5, 16, 30, 0)[u]
            proxy.update, proxy.cas = u, 0
            n0 = len(proxy.draws)
            upd(stub)
            kinds = [k for k, _ in proxy.draws[n0:]]
            out[f"{tag}_u{u}_kinds"] = np.array([0 if k == "randint" else 1 for k in kinds], np.int8)
            for j, (k, v) in enumerate(proxy.draws[n0:]):
                out[f"{tag}_u{u}_d{j}"] = v
            out[f"{tag}_u{u}_step_counter"] = stub.step_counter.numpy().copy()
            out[f"{tag}_u{u}_grid"] = stub.density_grid.numpy().copy()
            out[f"{tag}_u{u}_bitfield"] = stub.density_bitfield.numpy().copy()
            out[f"{tag}_u{u}_mean_density"] = np.float64(stub.mean_density)
            out[f"{tag}_u{u}_mean_count"] = np.int64(stub.mean_count)
            out[f"{tag}_u{u}_local_step"] = np.int64(stub.local_step)
    np.savez_compressed(os.path.join(HERE, "density_reference.npz"), **out)


if __name__ == "__main__":
    sh_fixture()
    mlp_fixture()
    trunc_exp_fixture()
    renderer_run_fixture()
    renderer_run_backward_fixture()
    get_rays_fixture()
    nerf_matrix_fixture()
    freq_fixture()
    density_fixture()
    print("wrote", sorted(f for f in os.listdir(HERE) if f.endswith(".npz")))

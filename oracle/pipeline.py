"""CPU restatement of one instant-ngp train step — TEST INFRASTRUCTURE ONLY.

Used by bench.py's `cpu_baseline` leg (kind "port") and by tests. Built only
from the oracle restatements in this package: march_rays_train (C), hash-grid
encode forward/backward (C), the fused MLP forward/backward (numpy, fp32),
trunc_exp, SH (numpy), composite forward/backward (C) and Adam (numpy).
Single-threaded (BLAS pinned to one thread by the caller).
"""
import time

import numpy as np

import oracle

_ADAM = dict(lr=1e-2, b1=0.9, b2=0.99, eps=1e-15)


class CPUNeRF:
    """Parameters of NeRFNetwork (hashgrid L16 C2 T2^19, sigma FFMLP 32-64-64-16,
    colour FFMLP 32-64-64-64-16) held as numpy arrays; fp32 throughout."""

    def __init__(self, embeddings, offsets, per_level_scale, sigma_w, color_w, bitfield, bound=1.0,
                 cascade=1, grid_size=128):
        self.emb = np.ascontiguousarray(embeddings, np.float32)
        self.offsets = np.ascontiguousarray(offsets, np.int32)
        self.scale = per_level_scale
        self.sigma_w = np.ascontiguousarray(sigma_w, np.float32)
        self.color_w = np.ascontiguousarray(color_w, np.float32)
        self.bitfield = bitfield
        self.bound = bound
        self.cascade = cascade
        self.grid_size = grid_size
        self.state = {k: (np.zeros_like(v), np.zeros_like(v))
                      for k, v in (("emb", self.emb), ("sigma", self.sigma_w), ("color", self.color_w))}
        self.t = 0

    @staticmethod
    def _mlp_fwd(x, w, in_dim, hidden, nl):
        mats = oracle.mlp_layers(w, in_dim, 16, hidden, nl)
        hs = [x]
        h = x
        for i, W in enumerate(mats):
            z = h @ W.T
            h = np.maximum(z, 0) if i < len(mats) - 1 else z
            hs.append(h)
        return h, hs, mats

    @staticmethod
    def _mlp_bwd(g, hs, mats):
        gws = [None] * len(mats)
        d = g
        for i in range(len(mats) - 1, -1, -1):
            gws[i] = d.T @ hs[i]
            gi = d @ mats[i]
            d = gi * (hs[i] > 0) if i > 0 else gi
        return d, np.concatenate([x.reshape(-1) for x in gws])

    def train_step(self, rays_o, rays_d, gt_rgba, bg, noises, max_steps=1024, T_thresh=1e-4):
        N = rays_o.shape[0]
        aabb = np.array([-self.bound] * 3 + [self.bound] * 3, np.float32)
        nears, fars = oracle.near_far_from_aabb(rays_o, rays_d, aabb, 0.2)
        xyzs, dirs, deltas, rays, cnt = oracle.march_rays_train(
            rays_o, rays_d, self.bound, self.bitfield, self.cascade, self.grid_size, nears, fars,
            noises, max_steps=max_steps)
        M = max(int(cnt[0]), 1)
        xyzs, dirs, deltas = xyzs[:M], dirs[:M], deltas[:M]
        x01 = ((xyzs + self.bound) / (2 * self.bound)).astype(np.float32)
        enc, _ = oracle.grid_encode_forward(x01, self.emb, self.offsets, self.scale, 16)
        h, hs_s, mats_s = self._mlp_fwd(enc, self.sigma_w, 32, 64, 2)
        sigma = np.exp(h[:, 0])
        sh = oracle.sh_encode(dirs, 4)
        cin = np.concatenate([sh, h[:, 1:16], np.zeros((M, 1), np.float32)], -1).astype(np.float32)
        c, hs_c, mats_c = self._mlp_fwd(cin, self.color_w, 32, 64, 3)
        rgb = 1 / (1 + np.exp(-c[:, :3]))
        ws, dp, img = oracle.composite_rays_train_forward(sigma, rgb, deltas, rays, T_thresh)
        a = gt_rgba[:, 3:]
        gt = gt_rgba[:, :3] * a + bg * (1 - a)
        pred = img + (1 - ws)[:, None] * bg
        loss = float(np.mean((pred - gt) ** 2))
        g_pred = (2.0 / (N * 3)) * (pred - gt)
        g_img = g_pred.astype(np.float32)
        g_ws = -(g_pred * bg).sum(-1).astype(np.float32)
        g_sig, g_rgb = oracle.composite_rays_train_backward(g_ws, np.zeros(N, np.float32), g_img,
                                                            sigma, rgb, deltas, rays, ws, dp, img, T_thresh)
        g_c = np.zeros((M, 16), np.float32)
        g_c[:, :3] = g_rgb * rgb * (1 - rgb)
        g_cin, gw_color = self._mlp_bwd(g_c, hs_c, mats_c)
        g_h = np.zeros((M, 16), np.float32)
        g_h[:, 0] = g_sig * np.exp(np.clip(h[:, 0], -15, 15))
        g_h[:, 1:16] = g_cin[:, 16:31]
        g_enc, gw_sigma = self._mlp_bwd(g_h, hs_s, mats_s)
        g_emb = oracle.grid_encode_backward(g_enc.astype(np.float32), x01, self.offsets, 2,
                                            self.scale, 16).astype(np.float32)
        self.t += 1
        for key, p, g in (("emb", self.emb, g_emb.reshape(self.emb.shape)),
                          ("sigma", self.sigma_w, gw_sigma), ("color", self.color_w, gw_color)):
            m, v = self.state[key]
            m += (1 - _ADAM["b1"]) * (g - m)
            v *= _ADAM["b2"]
            v += (1 - _ADAM["b2"]) * g * g
            bc1 = 1 - _ADAM["b1"] ** self.t
            bc2 = 1 - _ADAM["b2"] ** self.t
            p -= (_ADAM["lr"] / bc1) * m / (np.sqrt(v) / np.sqrt(bc2) + _ADAM["eps"])
        return loss, M


def _f16(x):
    return np.asarray(x, np.float32).astype(np.float16)


def amp_train_step(rays_o, rays_d, rgba, bg, noises, bitfield, emb16, offsets, per_level_scale, w_sigma16,
                   w_color16, bound=1.0, cascade=1, grid_size=128, dt_gamma=0.0, max_steps=1024, M=None,
                   density_scale=1.0, T_thresh=1e-4, min_near=0.2, loss_scale=1.0):
    """Forward + backward of one reference train step under AMP (`-O`: fp16
    autocast + GradScaler), every intermediate returned so the HIP step can be
    compared stage by stage and end to end.

    Follows nerf/utils.py train_step (:453-497: gt = rgb*a + bg*(1-a), MSE
    .mean(-1).mean()), renderer.run_cuda's train branch (renderer.py:257-375),
    network_ff.forward (:51-74) and the autocast casts of the reference ops:
      * grid_encode: inputs (x+bound)/(2*bound) in fp32, table cast to half,
        half results (grid.py:52-56, gridencoder.cu:161-184: oracle C);
      * FFMLP: half in / half out, fp16 storage between layers (ffmlp.py:15-48);
      * trunc_exp: custom_fwd(cast_inputs=float32) -> fp32 sigma (activation.py);
      * SH: fp32 (sphere_harmonics.py), cat with the half geo features promotes
        to fp32, colour FFMLP casts it back to half;
      * sigmoid on the half colour output -> half rgb; composite casts to fp32
        (raymarching.py:240);
      * backward: every cast back to half where autocast cast forward (the
        rgb grad, the sigmoid / trunc_exp grads, the MLP input grads).
    The loss scale multiplies the backward seed as (loss * scale).backward()."""
    ro = np.ascontiguousarray(rays_o, np.float32)
    rd = np.ascontiguousarray(rays_d, np.float32)
    N = ro.shape[0]
    aabb = np.array([-bound] * 3 + [bound] * 3, np.float32)
    nears, fars = oracle.near_far_from_aabb(ro, rd, aabb, min_near)
    xyzs, dirs, deltas, rays, cnt = oracle.march_rays_train(
        ro, rd, bound, bitfield, cascade, grid_size, nears, fars, noises, M=M, dt_gamma=dt_gamma,
        max_steps=max_steps)
    m = min(int(cnt[0]), xyzs.shape[0])
    xyzs, dirs, deltas = xyzs[:m], dirs[:m], deltas[:m]
    # torch: tensor / python scalar is a multiply by the fp32 reciprocal
    x01 = ((xyzs + np.float32(bound)) * np.float32(1.0 / (2.0 * bound))).astype(np.float32)
    enc, _ = oracle.grid_encode_forward(x01, np.asarray(emb16, np.float16), offsets, per_level_scale, 16)
    h, _ = oracle.mlp_forward(enc, w_sigma16, 32, 16, 64, 2)                     # half [m, 16]
    h0 = h[:, 0].astype(np.float32)
    sigma = (np.float32(density_scale) * np.exp(h0)).astype(np.float32)
    sh = oracle.sh_encode(dirs, 4)
    color_in = np.concatenate([_f16(sh), h[:, 1:16], np.zeros((m, 1), np.float16)], -1)
    color_out, _ = oracle.mlp_forward(color_in, w_color16, 32, 16, 64, 3)        # half [m, 16]
    c = color_out[:, :3].astype(np.float32)
    rgb = _f16(1.0 / (1.0 + np.exp(-c))).astype(np.float32)
    ws, depth, image = oracle.composite_rays_train_forward(sigma, rgb, deltas, rays, T_thresh)
    bgf = np.asarray(bg, np.float32)
    a = np.asarray(rgba, np.float32)[:, 3:]
    gt = np.asarray(rgba, np.float32)[:, :3] * a + bgf * (1 - a)
    pred = image + (1 - ws)[:, None] * bgf
    loss = float(np.mean(np.mean((pred.astype(np.float64) - gt) ** 2, -1)))
    # (loss * scale).backward()
    g_pred = (loss_scale * 2.0 / (3.0 * N)) * (pred.astype(np.float64) - gt)
    g_img = g_pred.astype(np.float32)
    g_ws = (-(g_pred * bgf).sum(-1)).astype(np.float32)
    g_sig, g_rgb = oracle.composite_rays_train_backward(g_ws, np.zeros(N, np.float32), g_img, sigma, rgb,
                                                        deltas, rays, ws, depth, image, T_thresh)
    g_c = np.zeros((m, 16), np.float16)
    g_c[:, :3] = _f16(_f16(g_rgb).astype(np.float32) * (1 - rgb) * rgb)    # sigmoid_backward in half
    g_cin, gw_color = oracle.mlp_backward(g_c, color_in, w_color16, 32, 16, 64, 3)
    g_h = np.zeros((m, 16), np.float16)
    g_h[:, 0] = _f16((g_sig * np.float32(density_scale)) * np.exp(np.clip(h0, -15, 15)))
    g_h[:, 1:16] = g_cin[:, 16:31]
    g_enc, gw_sigma = oracle.mlp_backward(g_h, enc, w_sigma16, 32, 16, 64, 2)
    g_emb = oracle.grid_encode_backward(g_enc, x01, offsets, 2, per_level_scale, 16)
    return dict(nears=nears, fars=fars, xyzs=xyzs, dirs=dirs, deltas=deltas, rays=rays, counter=cnt, x01=x01,
                enc=enc, h=h, sigma=sigma, color_in=color_in, color_out=color_out, rgb=rgb, ws=ws, depth=depth,
                image=image, pred=pred, gt=gt, loss=loss, g_sigma=g_sig, g_rgb=g_rgb, g_color_out=g_c, g_h=g_h,
                g_color_in=g_cin, gw_color=gw_color, g_enc=g_enc, gw_sigma=gw_sigma, g_emb=g_emb)


def time_cpu_baseline(model, batches, budget_s=20.0):
    """Run train steps on `batches` (list of (rays_o, rays_d, rgba, bg, noises))
    until the budget is spent; returns (rays/s, steps, rays, seconds, mean M)."""
    t0 = time.perf_counter()
    rays = steps = 0
    ms = []
    for b in batches:
        _, m = model.train_step(*b)
        rays += b[0].shape[0]
        steps += 1
        ms.append(m)
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return rays / dt, steps, rays, dt, float(np.mean(ms))

"""Shared synthetic inputs for the parity tests (seeded, CPU generators)."""
import math

import numpy as np


from nerf.provider import LEGO_BOXES, box_bitfield  # noqa: E402,F401


def lego_boxes():
    return LEGO_BOXES


def lego_rays(N, H=800, W=800, seed=0, radius=4.0311 * 0.8, camera_angle_x=0.6911112):
    """N random pixel rays from random ring poses (nerf_synthetic convention)."""
    rng = np.random.default_rng(seed)
    focal = 0.5 * W / math.tan(0.5 * camera_angle_x)
    theta = rng.uniform(0, 2 * np.pi, N)
    phi = np.deg2rad(rng.uniform(15, 60, N))
    cam = np.stack([radius * np.cos(phi) * np.cos(theta), radius * np.cos(phi) * np.sin(theta),
                    radius * np.sin(phi)], -1)
    fwd = -cam / np.linalg.norm(cam, axis=-1, keepdims=True)
    up = np.array([0, 0, 1.0])
    right = np.cross(fwd, up); right /= np.linalg.norm(right, axis=-1, keepdims=True)
    upv = np.cross(right, fwd)
    px = rng.uniform(0, W, N); py = rng.uniform(0, H, N)
    dx = (px - W / 2) / focal; dy = (py - H / 2) / focal
    d = fwd + dx[:, None] * right - dy[:, None] * upv
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    return cam.astype(np.float32), d.astype(np.float32)


def close16(got, ref, what="", min_equal=0.98, rel_norm=1e-3):
    """fp16 outputs of an fp32-accumulating kernel against the float64 oracle
    rounded to fp16: each value bit-identical or within 2 fp16 ulps plus 1e-3
    of the largest magnitude (sums that cancel), >= min_equal of the values
    bit-identical, and the whole tensor within rel_norm."""
    import numpy as np
    got = np.asarray(got).astype(np.float16)
    ref = np.asarray(ref).astype(np.float16)
    assert got.shape == ref.shape, what
    g, r = got.astype(np.float64), ref.astype(np.float64)
    assert np.isfinite(g).all(), what
    tol = 2 * np.spacing(np.abs(ref)).astype(np.float64) + 1e-3 * np.abs(r).max()
    bad = np.abs(g - r) > tol
    assert not bad.any(), (what, int(bad.sum()), g[bad][:6], r[bad][:6])
    same = float((got.view(np.uint16) == ref.view(np.uint16)).mean())
    assert same >= min_equal, (what, same)
    assert np.linalg.norm(g - r) <= rel_norm * np.linalg.norm(r), (what, np.linalg.norm(g - r) / np.linalg.norm(r))

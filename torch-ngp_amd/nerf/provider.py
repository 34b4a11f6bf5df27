"""Synthetic 'Lego-like' dataset (SURVEY §8(d) Config 2): the real
nerf_synthetic/lego images are not available offline, so the scene is an
analytic solid (union of three coloured boxes) seen from 100 ring poses in
the nerf_synthetic convention, converted with nerf_matrix_to_ngp exactly as
the reference provider does (nerf/provider.py:19-27). Rays/targets are
produced on the GPU each step like the reference's preload + collate path
(provider.py:442-564, utils.py:52-136)."""
import math

import numpy as np
import torch

from .utils import get_rays

LEGO_BOXES = [((-0.5, -0.35, -0.3), (0.5, 0.35, 0.1)),
              ((-0.2, -0.2, 0.1), (0.2, 0.2, 0.45)),
              ((-0.45, -0.3, -0.3), (-0.25, 0.3, 0.3))]
LEGO_COLORS = [(0.95, 0.75, 0.1), (0.8, 0.1, 0.1), (0.3, 0.3, 0.3)]


def nerf_matrix_to_ngp(pose, scale=0.33, offset=(0, 0, 0)):
    return np.array([
        [pose[1, 0], -pose[1, 1], -pose[1, 2], pose[1, 3] * scale + offset[0]],
        [pose[2, 0], -pose[2, 1], -pose[2, 2], pose[2, 3] * scale + offset[1]],
        [pose[0, 0], -pose[0, 1], -pose[0, 2], pose[0, 3] * scale + offset[2]],
        [0, 0, 0, 1]], dtype=np.float32)


def _morton3(x, y, z):
    def expand(v):
        v = (v * 0x00010001) & 0xFF0000FF
        v = (v * 0x00000101) & 0x0F00F00F
        v = (v * 0x00000011) & 0xC30C30C3
        v = (v * 0x00000005) & 0x49249249
        return v
    x, y, z = (np.asarray(a, np.int64) for a in (x, y, z))
    return expand(x) | (expand(y) << 1) | (expand(z) << 2)


def box_bitfield(boxes=LEGO_BOXES, cascade=1, H=128, bound=1.0):
    """Occupancy bitfield [C*H^3/8] (Morton order, like packbits): a cell is
    occupied when its centre lies in any box; cascade c spans min(2^c, bound)."""
    i = np.arange(H)
    xx, yy, zz = (a.reshape(-1) for a in np.meshgrid(i, i, i, indexing="ij"))
    idx = _morton3(xx, yy, zz)
    grid = np.zeros((cascade, H ** 3), np.float32)
    for c in range(cascade):
        b = min(2 ** c, bound)
        cx, cy, cz = (((a + 0.5) / H * 2 - 1) * b for a in (xx, yy, zz))
        occ = np.zeros(H ** 3, bool)
        for lo, hi in boxes:
            occ |= ((cx >= lo[0]) & (cx <= hi[0]) & (cy >= lo[1]) & (cy <= hi[1]) &
                    (cz >= lo[2]) & (cz <= hi[2]))
        grid[c, idx] = occ
    flat = grid.reshape(-1, 8)
    bits = np.zeros(flat.shape[0], np.uint8)
    for k in range(8):
        bits |= (flat[:, k] > 0.5).astype(np.uint8) << k
    return bits


def lego_bitfield(cascade=1, H=128, bound=1.0):
    return box_bitfield(LEGO_BOXES, cascade, H, bound)


def sphere_bitfield(radius=0.7, cascade=1, H=128, bound=1.0):
    """Occupancy of the cells whose centre lies in a ball (a conservative,
    early-training grid around the Lego boxes, which it contains): ~80 samples
    per ray at the Lego cameras, inside SURVEY §8(d)'s 50-120 estimate."""
    i = np.arange(H)
    xx, yy, zz = (a.reshape(-1) for a in np.meshgrid(i, i, i, indexing="ij"))
    idx = _morton3(xx, yy, zz)
    grid = np.zeros((cascade, H ** 3), np.float32)
    for c in range(cascade):
        b = min(2 ** c, bound)
        cx, cy, cz = (((a + 0.5) / H * 2 - 1) * b for a in (xx, yy, zz))
        grid[c, idx] = (cx * cx + cy * cy + cz * cz) <= radius * radius
    flat = grid.reshape(-1, 8)
    bits = np.zeros(flat.shape[0], np.uint8)
    for k in range(8):
        bits |= (flat[:, k] > 0.5).astype(np.uint8) << k
    return bits


# A Fox-shaped solid for Config 3 (bound 2): head, snout, ears and body as
# ellipsoids (centre, radii) in ngp coordinates. The real data/fox images are
# not in the image; this occupancy gives the bench's Config-3 leg ~30 samples
# per ray at dt_gamma 1/128 from the ring cameras (62 % of rays hit it), where
# the Lego boxes at bound 2 give 2.7.
FOX_ELLIPSOIDS = [((0.0, 0.0, 0.13), (0.975, 0.78, 0.715)),
                  ((0.91, 0.0, -0.065), (0.585, 0.325, 0.286)),
                  ((-0.26, 0.455, 0.845), (0.195, 0.156, 0.39)),
                  ((-0.26, -0.455, 0.845), (0.195, 0.156, 0.39)),
                  ((-0.65, 0.0, -0.78), (0.91, 0.65, 0.65))]


def ellipsoid_bitfield(ellipsoids=FOX_ELLIPSOIDS, cascade=2, H=128, bound=2.0):
    """Occupancy of the cells whose centre lies in any ellipsoid (as
    box_bitfield: Morton order, cascade c spans min(2^c, bound))."""
    i = np.arange(H)
    xx, yy, zz = (a.reshape(-1) for a in np.meshgrid(i, i, i, indexing="ij"))
    idx = _morton3(xx, yy, zz)
    grid = np.zeros((cascade, H ** 3), np.float32)
    for c in range(cascade):
        b = min(2 ** c, bound)
        cx, cy, cz = (((a + 0.5) / H * 2 - 1) * b for a in (xx, yy, zz))
        occ = np.zeros(H ** 3, bool)
        for (x0, y0, z0), (rx, ry, rz) in ellipsoids:
            occ |= ((cx - x0) / rx) ** 2 + ((cy - y0) / ry) ** 2 + ((cz - z0) / rz) ** 2 <= 1
        grid[c, idx] = occ
    flat = grid.reshape(-1, 8)
    bits = np.zeros(flat.shape[0], np.uint8)
    for k in range(8):
        bits |= (flat[:, k] > 0.5).astype(np.uint8) << k
    return bits


def fox_bitfield(cascade=2, H=128, bound=2.0):
    return ellipsoid_bitfield(FOX_ELLIPSOIDS, cascade, H, bound)


class SyntheticLego:
    """100 ring poses at 800x800, camera_angle_x 0.6911112, radius 4.0311
    (scaled by `scale`, default 0.8 as in readme.md:139)."""

    def __init__(self, device, H=800, W=800, n_poses=100, scale=0.8, radius=4.0311,
                 camera_angle_x=0.6911112, num_rays=4096):
        self.device = device
        self.H, self.W = H, W
        self.num_rays = num_rays
        focal = 0.5 * W / math.tan(0.5 * camera_angle_x)
        self.intrinsics = np.array([focal, focal, W / 2, H / 2], dtype=np.float32)
        poses = []
        for k in range(n_poses):
            th = 2 * math.pi * k / n_poses
            ph = math.radians(30.0 + 15.0 * math.sin(3 * th))
            c = np.array([radius * math.cos(ph) * math.cos(th), radius * math.cos(ph) * math.sin(th),
                          radius * math.sin(ph)])
            back = c / np.linalg.norm(c)
            right = np.cross([0, 0, 1.0], back); right /= np.linalg.norm(right)
            up = np.cross(back, right)
            c2w = np.eye(4)
            c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = right, up, back, c
            poses.append(nerf_matrix_to_ngp(c2w, scale=scale))
        self.poses = torch.from_numpy(np.stack(poses)).to(device)
        lo = torch.tensor([b[0] for b in LEGO_BOXES], device=device)
        hi = torch.tensor([b[1] for b in LEGO_BOXES], device=device)
        # the solid lives in ngp coordinates already (x, y, z of the bound box)
        self.box_lo, self.box_hi = lo, hi
        self.box_rgb = torch.tensor(LEGO_COLORS, device=device)

    def target(self, rays_o, rays_d):
        """Analytic RGBA: colour of the nearest box hit, alpha 1; else alpha 0."""
        o = rays_o.reshape(-1, 1, 3)
        inv = 1.0 / rays_d.reshape(-1, 1, 3)
        t0 = (self.box_lo[None] - o) * inv
        t1 = (self.box_hi[None] - o) * inv
        tn = torch.minimum(t0, t1).amax(-1)
        tf = torch.maximum(t0, t1).amin(-1)
        hit = (tf >= tn) & (tf > 0)
        tn = torch.where(hit, tn, torch.full_like(tn, float("inf")))
        tmin, arg = tn.min(-1)
        alpha = torch.isfinite(tmin).float()
        rgb = self.box_rgb[arg] * alpha[:, None]
        return torch.cat([rgb, alpha[:, None]], -1).view(*rays_o.shape[:-1], 4)

    def sample(self, index=None):
        """One training batch: rays of `num_rays` random pixels of one random
        pose. Device-side RNG only (no host sync), so it can sit in a graph."""
        if index is None:
            index = torch.randint(0, self.poses.shape[0], (1,), device=self.device)
        else:
            index = torch.tensor([index], device=self.device)
        poses = self.poses.index_select(0, index)
        rays = get_rays(poses, self.intrinsics, self.H, self.W, self.num_rays)
        images = self.target(rays["rays_o"], rays["rays_d"])
        return {"H": self.H, "W": self.W, "rays_o": rays["rays_o"], "rays_d": rays["rays_d"],
                "images": images}


class NeRFDataset:
    """Real-scene loader for the reference's transforms*.json format
    (nerf/provider.py:127-440): blender splits (transforms_{train,val,test}.json,
    'trainval' = train + val) or one colmap-style transforms.json. Poses go
    through nerf_matrix_to_ngp(scale, offset) (:19-27); images are decoded with
    PIL (the reference uses cv2, absent here) to float RGB(A) / 255 and
    area-resized by 1/downscale (cv2.INTER_AREA there, PIL's box filter here);
    intrinsics come from fl_x/fl_y or camera_angle_x/y, cx/cy defaulting to the
    image centre (:419-434). sample() is the reference's collate for training
    (:442-508): num_rays random pixels of one random image, through get_rays,
    with their ground-truth colours gathered; on the GPU the same batch feeds
    nerf.train.Trainer exactly like SyntheticLego does."""

    def __init__(self, path, device, type="train", downscale=1, scale=0.33, offset=(0, 0, 0), num_rays=4096):
        import json
        import os

        from PIL import Image

        self.device, self.num_rays = device, num_rays
        if os.path.exists(os.path.join(path, "transforms.json")):
            self.mode = "colmap"
            with open(os.path.join(path, "transforms.json")) as f:
                transform = json.load(f)
            frames = transform["frames"]
        elif os.path.exists(os.path.join(path, "transforms_train.json")):
            self.mode = "blender"
            splits = ["train", "val"] if type == "trainval" else [type]
            frames, transform = [], None
            for sp in splits:
                with open(os.path.join(path, f"transforms_{sp}.json")) as f:
                    t = json.load(f)
                transform = transform or t
                frames += t["frames"]
        else:
            raise FileNotFoundError(f"NeRFDataset: no transforms*.json under {path}")
        H = W = None
        if "h" in transform and "w" in transform:
            H, W = int(transform["h"]) // downscale, int(transform["w"]) // downscale
        poses, images = [], []
        for fr in frames:
            fp = os.path.join(path, fr["file_path"])
            if self.mode == "blender" and "." not in os.path.basename(fp):
                fp += ".png"
            poses.append(nerf_matrix_to_ngp(np.array(fr["transform_matrix"], dtype=np.float32), scale, offset))
            img = Image.open(fp)
            img = img.convert("RGBA" if img.mode in ("RGBA", "LA", "P") else "RGB")
            if H is None:
                W, H = img.size[0] // downscale, img.size[1] // downscale
            if img.size != (W, H):
                img = img.resize((W, H), Image.BOX)
            images.append(np.asarray(img, dtype=np.float32) / 255.0)
        self.H, self.W = H, W
        self.poses = torch.from_numpy(np.stack(poses)).to(device)
        self.images = torch.from_numpy(np.stack(images)).to(device)
        if "fl_x" in transform or "fl_y" in transform:
            fl_x = (transform["fl_x"] if "fl_x" in transform else transform["fl_y"]) / downscale
            fl_y = (transform["fl_y"] if "fl_y" in transform else transform["fl_x"]) / downscale
        elif "camera_angle_x" in transform or "camera_angle_y" in transform:
            fl_x = W / (2 * math.tan(transform["camera_angle_x"] / 2)) if "camera_angle_x" in transform else None
            fl_y = H / (2 * math.tan(transform["camera_angle_y"] / 2)) if "camera_angle_y" in transform else None
            fl_x = fl_x if fl_x is not None else fl_y
            fl_y = fl_y if fl_y is not None else fl_x
        else:
            raise RuntimeError("NeRFDataset: no focal length (fl_x/fl_y or camera_angle_x/y) in the transforms")
        cx = transform["cx"] / downscale if "cx" in transform else W / 2
        cy = transform["cy"] / downscale if "cy" in transform else H / 2
        self.intrinsics = np.array([fl_x, fl_y, cx, cy], dtype=np.float32)
        self.radius = float(self.poses[:, :3, 3].norm(dim=-1).mean())

    def sample(self, index=None, generator=None):
        if index is None:
            index = int(torch.randint(0, self.poses.shape[0], (1,), generator=generator).item())
        poses = self.poses[index:index + 1]
        rays = get_rays(poses, self.intrinsics, self.H, self.W, self.num_rays, generator=generator)
        C = self.images.shape[-1]
        images = torch.gather(self.images[index:index + 1].view(1, -1, C), 1,
                              rays["inds"].unsqueeze(-1).expand(1, rays["inds"].shape[-1], C))
        return {"H": self.H, "W": self.W, "rays_o": rays["rays_o"], "rays_d": rays["rays_d"], "images": images,
                "index": index}

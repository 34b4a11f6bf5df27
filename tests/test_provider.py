"""CPU: the transforms*.json loader (nerf.provider.NeRFDataset) against the
reference's conventions (nerf/provider.py:19-27 pose conversion, :419-434
intrinsics, :313-344 image decoding/downscale), on a tiny scene written here."""
import json
import math

import numpy as np
import torch
from PIL import Image


def _scene(tmp_path, colmap=False):
    rng = np.random.default_rng(0)
    frames, imgs = [], []
    for k in range(3):
        th = 0.4 * k
        c2w = np.eye(4)
        c2w[:3, :3] = [[math.cos(th), 0, math.sin(th)], [0, 1, 0], [-math.sin(th), 0, math.cos(th)]]
        c2w[:3, 3] = [math.sin(th) * 4, 0.5, math.cos(th) * 4]
        img = (rng.random((6, 8, 4)) * 255).astype(np.uint8)
        Image.fromarray(img, "RGBA").save(tmp_path / f"r_{k}.png")
        frames.append({"file_path": f"./r_{k}" + (".png" if colmap else ""), "transform_matrix": c2w.tolist()})
        imgs.append(img)
    if colmap:
        t = {"fl_x": 7.0, "fl_y": 7.5, "cx": 4.2, "cy": 2.9, "h": 6, "w": 8, "frames": frames}
        (tmp_path / "transforms.json").write_text(json.dumps(t))
    else:
        t = {"camera_angle_x": 0.6911112, "frames": frames}
        for sp in ("train", "val", "test"):
            (tmp_path / f"transforms_{sp}.json").write_text(json.dumps(t))
    return frames, imgs


def test_blender_split_poses_intrinsics_images(tmp_path):
    from nerf.provider import NeRFDataset, nerf_matrix_to_ngp
    frames, imgs = _scene(tmp_path)
    ds = NeRFDataset(str(tmp_path), torch.device("cpu"), type="train", scale=0.8, num_rays=16)
    assert (ds.H, ds.W) == (6, 8) and ds.images.shape == (3, 6, 8, 4)
    for k, fr in enumerate(frames):
        ref = nerf_matrix_to_ngp(np.array(fr["transform_matrix"], np.float32), scale=0.8)
        assert np.array_equal(ds.poses[k].numpy(), ref)
        assert np.allclose(ds.images[k].numpy(), imgs[k] / 255.0)
    fl = 8 / (2 * math.tan(0.6911112 / 2))
    assert np.allclose(ds.intrinsics, [fl, fl, 4.0, 3.0])
    tv = NeRFDataset(str(tmp_path), torch.device("cpu"), type="trainval")
    assert tv.poses.shape[0] == 6
    g = torch.Generator().manual_seed(0)
    b = ds.sample(index=1, generator=g)
    assert b["rays_o"].shape == (1, 16, 3) and b["images"].shape == (1, 16, 4)
    assert torch.allclose(b["rays_d"].norm(dim=-1), torch.ones(1, 16), atol=1e-6)
    g = torch.Generator().manual_seed(0)
    inds = torch.randint(0, 48, size=[16], generator=g)
    assert torch.equal(b["images"][0], ds.images[1].view(-1, 4)[inds])


def test_colmap_transforms_and_downscale(tmp_path):
    from nerf.provider import NeRFDataset
    _scene(tmp_path, colmap=True)
    ds = NeRFDataset(str(tmp_path), torch.device("cpu"), downscale=2)
    assert ds.mode == "colmap" and (ds.H, ds.W) == (3, 4)
    assert np.allclose(ds.intrinsics, [3.5, 3.75, 2.1, 1.45])
    assert ds.images.shape == (3, 3, 4, 4)

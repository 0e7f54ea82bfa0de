"""Extract_Images (drop-in for model/extracting_images.py:15-133; the cfg4 caller,
imported by vis/render.py:13).

Same constructor and ``generate_images(data, render_dir, c2ws, fxfy, it, output_geo)``
signature, output files (img_out/, depth_out/ (.png + .npy), disp_out/, geo_out/) and
returned dict.  The frame is rendered by render_dist.render_image: eval mode on the HIP
path with a depth prior of ones (extracting_images.py:60-63), cut into contiguous ray
tiles over the ranks of an initialised process group and assembled by one all-gather
 -- on one process it is the whole frame on one GPU.

Image writing uses PIL instead of imageio / cv2 (absent here); the disparity colour map
is matplotlib's inferno, the map cv2.COLORMAP_INFERNO tabulates.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .common import arange_pixels
from .render_dist import render_image


def _write_png(path, arr):
    from PIL import Image
    Image.fromarray(np.ascontiguousarray(arr)).save(path)


def _inferno(u8):
    from matplotlib import colormaps
    return (colormaps["inferno"](u8.astype(np.float64) / 255.0)[..., :3] * 255.0 + 0.5).astype(np.uint8)


def _to_u8_range(x):
    """np.clip(255 / max * (x - min), 0, 255) as uint8 (extracting_images.py:117-118)."""
    return np.clip(255.0 / x.max() * (x - x.min()), 0, 255).astype(np.uint8)


class Extract_Images(object):
    def __init__(self, renderer, cfg, use_learnt_poses=True, use_learnt_focal=True, device=None, render_type=None):
        self.points_batch_size = 100000
        self.renderer = renderer
        self.resolution = cfg["extract_images"]["resolution"]
        self.device = device
        self.use_learnt_poses = use_learnt_poses
        self.use_learnt_focal = use_learnt_focal
        self.render_type = render_type

    def process_data_dict(self, data):
        """extracting_images.py:25-38."""
        return (data.get("img.camera_mat").to(self.device), data.get("img.scale_mat").to(self.device),
                data.get("img.idx"))

    def render_frame(self, camera_mat, world_mat, scale_mat, it):
        """(rgb [h,w,3], depth [h,w]) of the whole frame (eval z-depth, ones as depth prior)."""
        h, w = self.resolution
        pixels = arange_pixels(resolution=(h, w), device=self.device)[1]
        if self.render_type in (None, "nope_nerf"):
            rgb, depth = render_image(self.renderer, pixels, camera_mat, world_mat, scale_mat)
        else:                                     # other techniques: the reference's chunked loop
            rgb, depth = [], []
            with torch.no_grad():
                for p in torch.split(pixels, self.points_batch_size, dim=1):
                    o = self.renderer(p, torch.ones(1, p.shape[1], 1, device=self.device), camera_mat, world_mat,
                                      scale_mat, self.render_type, eval_=True, it=it, add_noise=False)
                    rgb.append(o["rgb"].reshape(-1, 3))
                    depth.append(o["depth_pred"].reshape(-1))
            rgb, depth = torch.cat(rgb), torch.cat(depth)
        return rgb.view(h, w, 3), depth.view(h, w)

    def generate_images(self, data, render_dir, c2ws, fxfy, it, output_geo):
        """extracting_images.py:40-133."""
        self.renderer.eval()
        camera_mat, scale_mat, img_idx = self.process_data_dict(data)
        img_idx = int(img_idx)
        world_mat = None
        if self.use_learnt_poses:
            world_mat = torch.inverse(c2ws[img_idx]).unsqueeze(0)
        if self.use_learnt_focal:
            camera_mat = torch.tensor([[[fxfy[0], 0, 0, 0], [0, -fxfy[1], 0, 0], [0, 0, -1, 0], [0, 0, 0, 1]]],
                                      dtype=torch.float32, device=self.device)
        h, w = self.resolution
        with torch.no_grad():
            rgb, depth = self.render_frame(camera_mat, world_mat, scale_mat, it)
        img_out = (rgb.cpu().numpy() * 255).astype(np.uint8)
        depth_out = depth.cpu().numpy()

        geo_out = None
        if output_geo:
            # Phong-shaded occupancy surface (rendering.py:199-258) in 1024-pixel chunks
            pixels = arange_pixels(resolution=(h, w), device=self.device)[1]
            with torch.no_grad():
                geo = torch.cat([self.renderer(p, None, camera_mat, world_mat, scale_mat, "phong_renderer", eval_=True,
                                               it=it, add_noise=False)["rgb"] for p in torch.split(pixels, 1024, dim=1)],
                                dim=1)
            geo_out = (geo.view(h, w, 3).cpu().numpy() * 255).astype(np.uint8)
            geo_dir = os.path.join(render_dir, "geo_out")
            os.makedirs(geo_dir, exist_ok=True)
            _write_png(os.path.join(geo_dir, str(img_idx).zfill(4) + ".png"), geo_out)

        dirs = {k: os.path.join(render_dir, k) for k in ("img_out", "depth_out", "disp_out")}
        for d in dirs.values():
            os.makedirs(d, exist_ok=True)
        np.save(os.path.join(dirs["depth_out"], "{}.npy".format(img_idx)), depth_out)
        disp_u8 = _inferno(_to_u8_range(1 / depth_out))
        depth_u8 = _to_u8_range(depth_out)
        name = str(img_idx).zfill(4) + ".png"
        _write_png(os.path.join(dirs["img_out"], name), img_out)
        _write_png(os.path.join(dirs["depth_out"], name), depth_u8)
        _write_png(os.path.join(dirs["disp_out"], name), disp_u8)
        return {"img": img_out, "depth": depth_u8, "geo": geo_out, "disp": disp_u8}

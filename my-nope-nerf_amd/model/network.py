"""Model wrapper (drop-in for model/network.py:7-33)."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class nope_nerf(nn.Module):
    def __init__(self, cfg, renderer, depth_estimator=None, device=None, **kwargs):
        super().__init__()
        self.renderer = renderer.to(device) if device is not None else renderer
        self.depth_estimator = depth_estimator.to(device) if depth_estimator is not None else None
        self.device = device

    def forward(self, p, ray_idx, camera_mat, world_mat, scale_mat, rendering_technique, it=0, eval_mode=False,
                depth_img=None, add_noise=True, img_size=None, depth_affine=None, **kw):
        """network.py:19-33: area-resize the depth prior to the image size, gather it at
        the sampled rays, render.  depth_affine (MI355X build): a function applied to the
        gathered values (the Trainer's scale / shift, commuted past the gather)."""
        depth = None
        if rendering_technique == "nope_nerf":
            d = depth_img
            if tuple(d.shape[-2:]) != tuple(img_size):
                d = F.interpolate(d, img_size, mode="area")     # identity when already H x W
            # index_select, not advanced indexing: its backward is one index_add (the ray
            # indices are distinct) instead of a sorted index_put (distortion learning)
            depth = torch.index_select(d.reshape(-1), 0, ray_idx.reshape(-1)).view(1, -1, 1)
            if depth_affine is not None:    # the Trainer's deferred depth-prior distortion
                depth = depth_affine(depth)
        return self.renderer(p, depth, camera_mat, world_mat, scale_mat, rendering_technique,
                             eval_=eval_mode, it=it, add_noise=add_noise, **kw)

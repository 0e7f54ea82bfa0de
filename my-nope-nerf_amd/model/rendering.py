"""Renderer on the MI355X path (drop-in for model/rendering.py).

``Renderer.forward`` / ``nope_nerf`` keep the reference signatures and out-dict keys
(rendering.py:22-168).  Ray generation is a handful of 4x4 / per-ray tensor ops; the
per-sample work (samples, encodings, MLP, heads, compositing) and its backward run as one
fused call into the nerf_hip kernels (field.render_field), so the reference's 64 000-sample
chunk loop (rendering.py:100-111), its ``cat``s and its ``cumprod`` never appear.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .common import get_mask, get_ndc_rays_fxfy, unproject_matrix
from .rays import camera_rays_hip
from .field import F_DIST_ALPHA, F_RELU, F_WHITE_BKGD, render_field, render_field_eval

epsilon = 1e-6  # rendering.py:9 (applied inside the composite kernel)


def camera_rays(pixels, depth, camera_mat, world_mat, scale_mat, normalise_ray=True):
    """rendering.py:52-80: origin, unit direction, ray-vector norm, guide distance d_src
    (= |P_depth - o|) and the depth-loss mask for pixels [1,R,2] with depth [1,R,1]."""
    M = unproject_matrix(camera_mat, world_mat, scale_mat)          # [1,4,4]
    R = pixels.shape[1]
    origin = M[:, :3, 3]                                            # M @ [0,0,0,1]
    cam = origin.unsqueeze(1).expand(1, R, 3)
    ones = torch.ones_like(pixels[..., :1])
    pix1 = torch.cat([pixels, ones, ones], dim=-1).transpose(1, 2)  # [x, y, 1, 1]
    p_world = (M @ pix1)[:, :3].transpose(1, 2)
    ray = p_world - cam
    ray_norm = ray.norm(2, 2)
    if depth is not None:
        pd = torch.cat([pixels * depth, depth, ones], dim=-1).transpose(1, 2)
        p_depth = (M @ pd)[:, :3].transpose(1, 2)
        d_src = torch.norm(p_depth - cam, p=2, dim=-1)
    else:
        d_src = torch.ones_like(ray_norm)
    if normalise_ray:
        ray = ray / ray_norm.unsqueeze(-1)
    else:
        d_src = d_src / ray_norm
    mask = (get_mask(d_src) & (d_src != 0))[0]                      # rendering.py:69-80
    return cam.reshape(-1, 3), ray.reshape(-1, 3), ray_norm[0], d_src[0], mask


class Renderer(nn.Module):
    def __init__(self, model, cfg, device=None, **kwargs):
        super().__init__()
        self._device = device
        self.depth_range = cfg["depth_range"]
        self.n_max_network_queries = cfg["n_max_network_queries"]
        self.white_background = cfg["white_background"]
        self.cfg = cfg
        self.model = model.to(device) if device is not None else model

    def forward(self, pixels, depth, camera_mat, world_mat, scale_mat, rendering_technique,
                add_noise=True, eval_=False, it=1000000, **kw):
        if rendering_technique == "nope_nerf":
            return self.nope_nerf(pixels, depth, camera_mat, world_mat, scale_mat, it=it,
                                  add_noise=add_noise, eval_=eval_, **kw)
        raise NotImplementedError(
            f"rendering_technique '{rendering_technique}' (phong / sphere tracing visualisation, "
            "rendering.py:203-460) is outside the MI355X hot path")

    def _flags(self) -> int:
        f = 0
        if self.cfg["dist_alpha"]:
            f |= F_DIST_ALPHA
        if self.white_background:
            f |= F_WHITE_BKGD
        if getattr(self.model, "occ_activation", "softplus") != "softplus":
            f |= F_RELU
        return f

    def nope_nerf(self, pixels, depth, camera_mat, world_mat, scale_mat, add_noise=False, it=100000,
                  eval_=False, noise=None, dense_depth=False):
        """rendering.py:36-168.  Extra keyword arguments of the MI355X build:
        ``noise`` injects the stratified U[0,1) tensor (1,R,S) instead of torch.rand;
        ``dense_depth`` returns unmasked depth_pred/depth_gt plus 'depth_mask' (R,) so the
        training step never needs the boolean-index host sync (rendering.py:151-153)."""
        cfg = self.cfg
        S = cfg["num_points"] - cfg.get("outside_steps", 0)
        near, far = float(self.depth_range[0]), float(self.depth_range[1])
        if pixels.is_cuda:       # two launches: the unprojection matrix, then every ray
            M = unproject_matrix(camera_mat, world_mat, scale_mat)
            cam, ray, view, ray_norm, d_src, mask = camera_rays_hip(
                M, pixels, depth, cfg["normalise_ray"], view_ones=not cfg["use_ray_dir"])
        else:
            cam, ray, ray_norm, d_src, mask = camera_rays(pixels, depth, camera_mat, world_mat, scale_mat,
                                                          cfg["normalise_ray"])
            view = -ray if cfg["use_ray_dir"] else torch.ones_like(ray)
        R = cam.shape[0]
        if cfg["sample_option"] == "ndc":        # rendering.py:169-181 (no jitter)
            fxfy = torch.cat([camera_mat[:, 0, 0], camera_mat[:, 1, 1]])
            pts_o, pts_d = get_ndc_rays_fxfy(fxfy, 1.0, cam, ray)
            near_s, far_s, nz = 0.0, 1.0, None
        else:                                    # rendering.py:183-198
            pts_o, pts_d = cam, ray
            near_s, far_s = near, far
            nz = None
            if add_noise:
                nz = noise if noise is not None else torch.rand(1, R, S, device=cam.device)
                nz = nz.reshape(R, S).float()
        flags = self._flags()
        if torch.is_grad_enabled():
            rgb, dist, alpha, z = render_field(self.model, pts_o, pts_d, view, nz, near_s, far_s, S, flags)
        else:
            rgb, dist, alpha, z = render_field_eval(self.model, pts_o, pts_d, view, near_s, far_s, S, flags) \
                if nz is None else render_field(self.model, pts_o, pts_d, view, nz, near_s, far_s, S, flags)
        if eval_ and cfg["normalise_ray"]:       # rendering.py:144-148
            dist = dist / ray_norm
            d_src = d_src / ray_norm
        if cfg["sample_option"] == "ndc":
            d_src = 1 - 1 / d_src
        out = {"rgb": rgb.reshape(1, -1, 3), "z_vals": z, "normal": None, "alpha": alpha}
        if eval_:
            out["depth_pred"], out["depth_gt"] = dist, d_src
        elif dense_depth:
            out["depth_pred"], out["depth_gt"], out["depth_mask"] = dist, d_src, mask
        else:                                    # rendering.py:151-153
            out["depth_pred"], out["depth_gt"] = dist[mask], d_src[mask]
        return out

"""CPU restatement of the NoPe-NeRF render + training step (the ORACLE).

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline.  The product path (``my-nope-nerf_amd/``) never
imports it and fails loudly when its HIP library is missing.

Parity status: **parity unpinned upstream.**  The reference repository ships no
tests, golden vectors or fixtures for this path, and importing
or running the reference was denied in the survey session;
that denial binds every later session.  This module is therefore a restatement
written from the reference *text*; it is pinned by
  (i)  analytic known-answer tests (tests/test_oracle_kat.py),
  (ii) fp64 finite-difference gradient checks (tests/test_oracle_grad.py),
  (iii) committed golden fixtures generated from it (tests/golden/, script
       tests/golden/make_golden.py) so that a later edit cannot drift silently.

Every function cites the reference file:line it restates.  It is written
functionally (device/dtype agnostic, no ``.cuda()``), with the stochastic parts of
the reference (``torch.rand`` stratified noise, ``randperm`` ray choice) injected
by the caller so that the HIP path can be fed bit-identical inputs.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

EPS_COMPOSITE = 1e-6  # model/rendering.py:9


# ----------------------------------------------------------------------------
# positional encoding + field MLP  (model/official_nerf.py)
# ----------------------------------------------------------------------------
def encode_position(x: torch.Tensor, levels: int, inc_input: bool = True) -> torch.Tensor:
    """official_nerf.py:99-119: [x, sin(2^0 x), cos(2^0 x), ..., sin(2^{L-1} x), cos(2^{L-1} x)]."""
    parts = [x] if inc_input else []
    for i in range(levels):
        scaled = (2.0 ** i) * x
        parts += [torch.sin(scaled), torch.cos(scaled)]
    return torch.cat(parts, dim=-1)


class OracleNerf(nn.Module):
    """official_nerf.py:8-44 (topology, parameter names, bias overrides).

    Parameter names are the reference's state_dict keys (layers0.*, layers1.*,
    fc_density, fc_feature, rgb_layers.0, fc_rgb) so the same state_dict loads
    into the oracle, the reference and the HIP module."""

    def __init__(self, hidden_dim: int = 256, pos_enc_levels: int = 10, dir_enc_levels: int = 4,
                 white_background: bool = False, dist_alpha: bool = False,
                 occ_activation: str = "softplus"):
        super().__init__()
        D = hidden_dim
        pin = (2 * pos_enc_levels + 1) * 3       # official_nerf.py:14
        din = (2 * dir_enc_levels + 1) * 3       # official_nerf.py:15
        self.dist_alpha = dist_alpha
        self.occ_activation = occ_activation
        self.layers0 = nn.Sequential(nn.Linear(pin, D), nn.ReLU(), nn.Linear(D, D), nn.ReLU(),
                                     nn.Linear(D, D), nn.ReLU(), nn.Linear(D, D), nn.ReLU())
        self.layers1 = nn.Sequential(nn.Linear(D + pin, D), nn.ReLU(), nn.Linear(D, D), nn.ReLU(),
                                     nn.Linear(D, D), nn.ReLU(), nn.Linear(D, D), nn.ReLU())
        self.fc_density = nn.Linear(D, 1)
        self.fc_feature = nn.Linear(D, D)
        self.rgb_layers = nn.Sequential(nn.Linear(D + din, D // 2), nn.ReLU())
        self.fc_rgb = nn.Linear(D // 2, 3)
        with torch.no_grad():                     # official_nerf.py:39-44
            self.fc_density.bias.fill_(0.1)
            self.fc_rgb.bias.fill_(0.8 if white_background else 0.02)

    def forward(self, p: torch.Tensor, ray_d: torch.Tensor):
        """official_nerf.py:60-96 with return_addocc=True -> (rgb, density/alpha)."""
        enc_p = encode_position(p, 10)            # hard-coded L=10 (official_nerf.py:61)
        x = self.layers0(enc_p)
        x = self.layers1(torch.cat([x, enc_p], dim=-1))
        sigma = self.fc_density(x)
        if self.occ_activation == "softplus":     # official_nerf.py:77-80
            sigma = F.softplus(sigma)
        else:
            sigma = sigma.relu()
        if not self.dist_alpha:                   # official_nerf.py:82-83
            sigma = 1 - torch.exp(-1.0 * sigma)
        enc_d = encode_position(ray_d, 4)         # hard-coded L=4 (official_nerf.py:87)
        feat = self.fc_feature(x)
        h = self.rgb_layers(torch.cat([feat, enc_d], dim=-1))
        rgb = torch.sigmoid(self.fc_rgb(h))
        return rgb, sigma

    def density_raw(self, p: torch.Tensor) -> torch.Tensor:
        """infer_occ (official_nerf.py:60-67): fc_density of the trunk."""
        enc_p = encode_position(p, 10)
        x = self.layers0(enc_p)
        x = self.layers1(torch.cat([x, enc_p], dim=-1))
        return self.fc_density(x)

    def occupancy(self, p: torch.Tensor) -> torch.Tensor:
        """forward(p, only_occupancy=True) (official_nerf.py:76-85)."""
        sigma = self.density_raw(p)
        sigma = F.softplus(sigma) if self.occ_activation == "softplus" else sigma.relu()
        return sigma if self.dist_alpha else 1 - torch.exp(-1.0 * sigma)

    def gradient(self, p: torch.Tensor) -> torch.Tensor:
        """official_nerf.py:46-58: -d(fc_density)/dp as [N, 1, 3]."""
        with torch.enable_grad():
            p = p.detach().requires_grad_(True)
            y = self.density_raw(p)
            g = torch.autograd.grad(y, p, torch.ones_like(y))[0]
        return -g.unsqueeze(1)


def normal_diff(model: "OracleNerf", cam, ray, d_src, obj_mask, noise):
    """rendering.py:127-135 (normal_loss branch): surface points cam + ray d at the masked
    rays (rendering.py:76-88), a jittered copy (noise: the injected U[0,1) (N,3) of
    torch.rand_like), normals g / (|g| + 1e-5) of g = gradient() (official_nerf.py:46-58),
    -> |n - n_jitter| per surface point."""
    surface = (cam + ray * d_src.unsqueeze(-1))[obj_mask]
    n = surface.shape[0]
    neighbours = surface + (noise - 0.5) * 0.01
    g = model.gradient(torch.cat([surface, neighbours], 0))[:, 0, :]
    normals = g / (g.norm(2, dim=1).unsqueeze(-1) + 10 ** (-5))
    return torch.norm(normals[:n] - normals[n:], dim=-1)


# ----------------------------------------------------------------------------
# camera helpers  (model/common.py)
# ----------------------------------------------------------------------------
def arange_pixels(h: int, w: int, device="cpu", dtype=torch.float32):
    """common.py:13-40: integer (x=col, y=row) locations and their [-1,1] scaling
    x' = 2 col/(W-1) - 1, y' = 2 row/(H-1) - 1 (row-major over the image)."""
    rows, cols = torch.meshgrid(torch.arange(h, device=device), torch.arange(w, device=device),
                                indexing="ij")
    loc = torch.stack([cols, rows], dim=-1).reshape(1, -1, 2)
    scaled = loc.to(dtype).clone()
    scaled[..., 0] = 2.0 * scaled[..., 0] / (w - 1) - 1.0
    scaled[..., 1] = 2.0 * scaled[..., 1] / (h - 1) - 1.0
    return loc, scaled


def _unproject(pixels: torch.Tensor, depth: torch.Tensor, camera_mat, world_mat, scale_mat):
    """common.py:112-160 (transform_to_world, invert=True): scale^-1 world^-1 K^-1 [x d, y d, d, 1]."""
    B, N, _ = pixels.shape
    hom = torch.cat([pixels * depth, depth, torch.ones_like(depth)], dim=-1).permute(0, 2, 1)
    M = torch.inverse(scale_mat) @ torch.inverse(world_mat) @ torch.inverse(camera_mat)
    return (M @ hom)[:, :3].permute(0, 2, 1)


def transform_to_world(pixels, depth, camera_mat, world_mat=None, scale_mat=None):
    eye = torch.eye(4, dtype=pixels.dtype, device=pixels.device).unsqueeze(0)
    world_mat = eye if world_mat is None else world_mat
    scale_mat = eye if scale_mat is None else scale_mat
    return _unproject(pixels, depth, camera_mat, world_mat, scale_mat)


def origin_to_world(n_points: int, camera_mat, world_mat, scale_mat):
    """common.py:186-215: camera centre, repeated n_points times -> (B, n, 3)."""
    B = camera_mat.shape[0]
    p = torch.zeros(B, 4, n_points, dtype=camera_mat.dtype, device=camera_mat.device)
    p[:, -1] = 1.0
    M = torch.inverse(scale_mat) @ torch.inverse(world_mat) @ torch.inverse(camera_mat)
    return (M @ p)[:, :3].permute(0, 2, 1)


def image_points_to_world(pixels, camera_mat, world_mat, scale_mat):
    """common.py:218-237: unprojection at depth 1."""
    ones = torch.ones(*pixels.shape[:2], 1, dtype=pixels.dtype, device=pixels.device)
    return _unproject(pixels, ones, camera_mat, world_mat, scale_mat)


def get_mask(t: torch.Tensor) -> torch.Tensor:
    """common.py:60-72: finite (not +-inf, not nan)."""
    return (t.abs() != math.inf) & ~torch.isnan(t)


def get_ndc_rays_fxfy(fxfy, near, rays_o, rays_d):
    """common.py:632-675 (NDC warp used by sample_option 'ndc')."""
    t = -(near + rays_o[..., 2]) / rays_d[..., 2]
    rays_o = rays_o + t[..., None] * rays_d
    ox_oz = rays_o[..., 0] / rays_o[..., 2]
    oy_oz = rays_o[..., 1] / rays_o[..., 2]
    o0 = -1.0 / (1 / fxfy[0]) * ox_oz
    o1 = -1.0 / (1 / fxfy[1]) * oy_oz
    o2 = 1.0 + 2.0 * near / rays_o[..., 2]
    d0 = -1.0 / (1 / fxfy[0]) * (rays_d[..., 0] / rays_d[..., 2] - ox_oz)
    d1 = -1.0 / (1 / fxfy[1]) * (rays_d[..., 1] / rays_d[..., 2] - oy_oz)
    d2 = 1 - o2
    return torch.stack([o0, o1, o2], -1), torch.stack([d0, d1, d2], -1)


# ----------------------------------------------------------------------------
# renderer  (model/rendering.py:36-198)
# ----------------------------------------------------------------------------
DEFAULT_RENDER_CFG = dict(num_points=128, depth_range=[0.01, 10.0], dist_alpha=False,
                          sample_option="uniform", use_ray_dir=True, normalise_ray=True,
                          white_background=False, outside_steps=0, n_max_network_queries=64000)


def linspace01(S: int, dtype=torch.float32, device="cpu") -> torch.Tensor:
    """torch.linspace(0, 1, S) as the reference's device computes it (the CUDA kernel of
    aten/src/ATen/native/cuda/RangeFactories.cu, PyTorch 1.7-2.x: float step, element
    i = start + step*i below the halfway point, end - step*(S-1-i) above it).  The CPU
    kernel vectorises with a machine-dependent chunking (base + k*step), so the per-element
    form is the stable definition; products and sums are rounded separately."""
    if S == 1:
        return torch.zeros(1, dtype=dtype, device=device)
    step = torch.tensor(1.0, dtype=dtype) / torch.tensor(float(S - 1), dtype=dtype)
    i = torch.arange(S, dtype=dtype)
    lo = step * i
    hi = torch.tensor(1.0, dtype=dtype) - step * (S - 1 - i)
    return torch.where(torch.arange(S) < S // 2, lo, hi).to(device)


def stratified_z(n_rays: int, S: int, near: float, far: float, noise: Optional[torch.Tensor],
                 dtype=torch.float32, device="cpu"):
    """rendering.py:89-90 + 183-191: z = lerp(near, far, linspace(0,1,S)); with noise,
    z = lo + (hi - lo) U where lo/hi are bin midpoints (ends clamped)."""
    t = linspace01(S, dtype, device).view(1, 1, -1).repeat(1, n_rays, 1)
    z = near * (1.0 - t) + far * t
    if noise is not None:
        mid = 0.5 * (z[:, :, 1:] + z[:, :, :-1])
        hi = torch.cat([mid, z[:, :, -1:]], dim=-1)
        lo = torch.cat([z[:, :, :1], mid], dim=-1)
        z = lo + (hi - lo) * noise.view(1, n_rays, S).to(dtype)
    return z  # (1, R, S)


def rays_from_cameras(pixels, depth, camera_mat, world_mat, scale_mat, normalise_ray=True):
    """rendering.py:52-87: ray origin/direction, d_gt and the depth-loss mask."""
    n = pixels.shape[1]
    cam = origin_to_world(n, camera_mat, world_mat, scale_mat)
    pts_d = transform_to_world(pixels, depth, camera_mat, world_mat, scale_mat)
    d_src = torch.norm(pts_d - cam, p=2, dim=-1)
    pix_w = image_points_to_world(pixels, camera_mat, world_mat, scale_mat)
    ray = pix_w - cam
    ray_norm = ray.norm(2, 2)
    if normalise_ray:
        ray = ray / ray.norm(2, 2).unsqueeze(-1)
    else:
        d_src = d_src / ray_norm
    zero = d_src == 0                               # rendering.py:69
    valid = get_mask(d_src)                         # rendering.py:72
    obj_mask = (valid & ~zero)[0]                   # rendering.py:78-80
    return cam.reshape(-1, 3), ray.reshape(-1, 3), d_src[0], ray_norm[0], obj_mask


def composite(alpha: torch.Tensor, rgb: torch.Tensor, z: torch.Tensor, dist_alpha: bool = False,
              white_background: bool = False):
    """rendering.py:113-141: alpha (R,S) [density when dist_alpha], rgb (R,S,3), z (R,S).
    Returns rgb (R,3), dist (R,), alpha (R,S) as the reference computes them."""
    if dist_alpha:                                  # rendering.py:116-122
        deltas = z[:, 1:] - z[:, :-1]
        far = torch.full((z.shape[0], 1), 1e10, dtype=z.dtype, device=z.device)
        deltas = torch.cat([deltas, far], -1)
        alpha = 1 - torch.exp(-1.0 * alpha * deltas)
        alpha = torch.cat([alpha[:, :-1], torch.ones_like(alpha[:, -1:])], dim=-1)
    ones = torch.ones((alpha.shape[0], 1), dtype=alpha.dtype, device=alpha.device)
    trans = torch.cumprod(torch.cat([ones, 1.0 - alpha + EPS_COMPOSITE], -1), -1)[:, :-1]
    weights = alpha * trans                         # rendering.py:124
    rgb_out = torch.sum(weights.unsqueeze(-1) * rgb, dim=-2)
    dist = torch.sum(weights * z, dim=-1)
    if white_background:                            # rendering.py:139-141
        rgb_out = rgb_out + (1.0 - weights.sum(-1)).unsqueeze(-1)
    return rgb_out, dist, alpha, weights


def render_nope_nerf(model: OracleNerf, pixels, depth, camera_mat, world_mat, scale_mat,
                     cfg: Optional[dict] = None, noise: Optional[torch.Tensor] = None,
                     eval_: bool = False, chunk: Optional[int] = None) -> Dict[str, torch.Tensor]:
    """Renderer.nope_nerf, rendering.py:36-168 (uniform and ndc sampling).
    ``noise`` is the injected U[0,1) (1,R,S) tensor; None == add_noise False.  ``chunk``:
    evaluate the network in chunks of that many samples, as rendering.py:102-111 does with
    n_max_network_queries (a no-op in exact arithmetic; on a GPU it changes the GEMM
    shapes and so their rounding -- the convergence study's reference-vs-reference control)."""
    c = dict(DEFAULT_RENDER_CFG)
    c.update(cfg or {})
    S = c["num_points"] - c["outside_steps"]
    near, far = c["depth_range"]
    cam, ray, d_src, ray_norm, obj_mask = rays_from_cameras(
        pixels, depth, camera_mat, world_mat, scale_mat, c["normalise_ray"])
    R = cam.shape[0]
    if c["sample_option"] == "ndc":                 # rendering.py:169-181 (no noise)
        fxfy = torch.cat([camera_mat[:, 0, 0], camera_mat[:, 1, 1]])
        o_n, d_n = get_ndc_rays_fxfy(fxfy, 1.0, cam, ray)
        z = stratified_z(R, S, 0.0, 1.0, None, pixels.dtype, pixels.device)
        pts = (o_n.unsqueeze(-2) + d_n.unsqueeze(-2) * z.view(R, S, 1)).reshape(-1, 3)
    else:                                           # rendering.py:183-198
        z = stratified_z(R, S, near, far, noise, pixels.dtype, pixels.device)
        pts = (cam.unsqueeze(-2) + ray.unsqueeze(-2) * z.view(R, S, 1)).reshape(-1, 3)
    dirs = -1 * ray.unsqueeze(-2).repeat(1, S, 1).reshape(-1, 3)
    if not c["use_ray_dir"]:
        dirs = torch.ones_like(dirs)
    if chunk:                                       # rendering.py:100-111
        outs = [model(pts[i:i + chunk], dirs[i:i + chunk]) for i in range(0, pts.shape[0], chunk)]
        rgb_s, alpha_s = torch.cat([o[0] for o in outs]), torch.cat([o[1] for o in outs])
    else:
        rgb_s, alpha_s = model(pts, dirs)           # (chunking is a no-op in exact arithmetic)
    rgb_out, dist, alpha, _ = composite(alpha_s.view(R, S), rgb_s.view(R, S, 3), z.view(R, S),
                                        c["dist_alpha"], c["white_background"])
    if eval_ and c["normalise_ray"]:                # rendering.py:144-148
        dist = dist / ray_norm
        d_src = d_src / ray_norm
    if not eval_:                                   # rendering.py:151-156
        dpred, dgt = dist[obj_mask], d_src[obj_mask]
    else:
        dpred, dgt = dist, d_src
    if c["sample_option"] == "ndc":
        dgt = 1 - 1 / dgt
    return {"rgb": rgb_out.reshape(1, -1, 3), "z_vals": z.view(R, S), "normal": None,
            "depth_pred": dpred, "depth_gt": dgt, "alpha": alpha}


# ----------------------------------------------------------------------------
# poses / distortion  (model/common.py:277-330, model/poses.py, model/distortions.py)
# ----------------------------------------------------------------------------
def vec2skew(v):
    z = torch.zeros(1, dtype=v.dtype, device=v.device)
    return torch.stack([torch.cat([z, -v[2:3], v[1:2]]), torch.cat([v[2:3], z, -v[0:1]]),
                        torch.cat([-v[1:2], v[0:1], z])], dim=0)


def Exp(r):
    """common.py:290-299: Rodrigues with theta = |r| + 1e-15 (not an SE(3) exp)."""
    K = vec2skew(r)
    th = r.norm() + 1e-15
    eye = torch.eye(3, dtype=r.dtype, device=r.device)
    return eye + (torch.sin(th) / th) * K + ((1 - torch.cos(th)) / th ** 2) * (K @ K)


def make_c2w(r, t):
    """common.py:301-310 (+ convert3x4_4x4 :312-330)."""
    top = torch.cat([Exp(r), t.unsqueeze(1)], dim=1)
    bottom = torch.tensor([[0, 0, 0, 1]], dtype=r.dtype, device=r.device)
    return torch.cat([top, bottom], dim=0)


def learn_pose_forward(r_all, t_all, init_c2w, cam_id: int):
    """poses.py:23-31: c2w = make_c2w(r, t) @ init_c2w[cam]."""
    c2w = make_c2w(r_all[cam_id], t_all[cam_id])
    if init_c2w is not None:
        c2w = c2w @ init_c2w[cam_id]
    return c2w


def learn_distortion_forward(scales, shifts, cam_id: int, fix_scaleN: bool = True):
    """distortions.py:19-27: scale clamped to >= 0.01, last camera fixed to 1."""
    scale = scales[cam_id]
    if scale < 0.01:
        scale = torch.tensor(0.01, dtype=scales.dtype, device=scales.device)
    if fix_scaleN and cam_id == scales.shape[0] - 1:
        scale = torch.tensor(1.0, dtype=scales.dtype, device=scales.device)
    return scale, shifts[cam_id]


# ----------------------------------------------------------------------------
# losses  (model/losses.py:17-228)
# ----------------------------------------------------------------------------
def rgb_full_loss(rgb, gt, kind="l2"):
    """losses.py:28-33: summed error divided by shape[1] (= number of rays)."""
    d = rgb - gt
    s = (d * d).sum() if kind == "l2" else d.abs().sum()
    return s / float(rgb.shape[1])


def depth_l1_loss(dpred, dgt):
    """losses.py:60-66 (l1): sum |.| / M."""
    return (dpred - dgt).abs().sum() / float(dpred.shape[0])


def closest_idx(src, dst):
    """losses.py:129-144: brute-force argmin of the L2 distance; src (3,S), dst (3,D)."""
    out = []
    for part in torch.split(src, 500000, dim=1):
        diff = part[:, :, None] - dst[:, None, :]
        out.append(torch.argmin(torch.linalg.norm(diff, dim=0), dim=1))
    return torch.cat(out)


def point_point_error(X, Y):
    """losses.py:145-150: mean |X - Y[nn(X)]|; X (3,S), Y (3,D)."""
    idx = closest_idx(X, Y)
    return torch.linalg.norm(X - Y[:, idx], dim=0).mean()


def pc_loss(Xt, Yt):
    """losses.py:116-123 (dense): symmetric chamfer on (1,P,3) clouds."""
    X, Y = Xt[0].permute(1, 0), Yt[0].permute(1, 0)
    return point_point_error(X, Y) + point_point_error(Y, X)


def mean_on_mask(diff, valid_mask):
    """losses.py:79-87."""
    mask = valid_mask.expand_as(diff)
    if mask.sum() > 0:
        return diff[mask].sum() / mask.sum()
    return torch.tensor(0.0, dtype=diff.dtype, device=diff.device)


def rgb_s_loss(rgb1, rgb2, valid_points):
    """losses.py:152-159 without SSIM (with_ssim False in the V_KITTI configs)."""
    return mean_on_mask((rgb1 - rgb2).abs().clamp(0, 1), valid_points)


def weight_dist_loss(t_list):
    """losses.py:105-114."""
    dist = (t_list - t_list.roll(shifts=1, dims=0))[1:].norm(dim=1)
    dd = (dist - dist.roll(shifts=1))[1:]
    return dist.mean(), dd.pow(2.0).mean()


def depth_invariant_loss(pred, gt, weight=None):
    """losses.py:35-58 (depth_loss_type 'invariant', via get_depth_loss :67-68): both depths
    normalised by their median t and mean absolute deviation s, (d - t) / s, then the MSE
    (optionally weighted: sum(w * se) / (sum(w) + 1e-8)).  torch.median of an even count
    is the lower middle value."""
    def norm(d):
        t = torch.median(d)
        return (d - t) / torch.mean(torch.abs(d - t))
    se = (norm(pred) - norm(gt)) ** 2
    if weight is None:
        return se.mean()
    return (se * weight).sum() / (weight.sum() + 1e-8)


def depth_consistency_loss(d1_proj, d2, d2_proj=None, d1=None):
    """losses.py:124-128: sum |d1_proj - d2| / shape[1], averaged with the reverse term when
    d2_proj is given."""
    loss = (d1_proj - d2).abs().sum() / float(d1_proj.shape[1])
    if d2_proj is not None:
        loss = 0.5 * loss + 0.5 * (d2_proj - d1).abs().sum() / float(d2_proj.shape[1])
    return loss


def t_cycle_loss(rt_pred, rt_gt):
    """losses.py:161-162: Frobenius norm of I - inverse(Rt_gt) @ Rt_pred (relative pose of
    the image pair, training.py:329-358)."""
    eye = torch.eye(4, dtype=rt_gt.dtype, device=rt_gt.device)
    return torch.linalg.norm(eye - torch.inverse(rt_gt) @ rt_pred)


def total_loss(rgb_pred, rgb_gt, depth_pred, depth_gt, weights: dict, rgb_loss_type="l2",
               pc=None, rgb_s=None, t_list=None, t_cycle=None, depth_loss_type="l1", d_consistency=None):
    """losses.py:164-228: the weighted sum of every term the trainer can switch on, with
    the reference's output keys; a term is evaluated only when its weight is non-zero."""
    dt = rgb_pred.dtype if rgb_pred is not None else torch.float32
    z = torch.zeros((), dtype=dt, device=rgb_pred.device if rgb_pred is not None else "cpu")
    w = {k: weights.get(k, 0.0) for k in ("rgb_weight", "depth_weight", "pc_weight", "rgb_s_weight",
                                          "weight_dist_1st_loss", "weight_dist_2nd_loss",
                                          "depth_consistency_weight", "t_cycle_weight")}
    l_rgb = rgb_full_loss(rgb_pred, rgb_gt, rgb_loss_type) if w["rgb_weight"] != 0 else z
    if w["depth_weight"] != 0:
        l_depth = (depth_l1_loss(depth_pred, depth_gt) if depth_loss_type == "l1"
                   else depth_invariant_loss(depth_pred, depth_gt))
    else:
        l_depth = z
    if w["weight_dist_1st_loss"] != 0 or w["weight_dist_2nd_loss"] != 0:
        l_d1, l_d2 = weight_dist_loss(t_list)
    else:
        l_d1 = l_d2 = z
    l_pc = pc if (pc is not None and w["pc_weight"] != 0) else z
    l_rgbs = rgb_s if (rgb_s is not None and w["rgb_s_weight"] != 0) else z
    l_dc = d_consistency if (d_consistency is not None and w["depth_consistency_weight"] != 0) else z
    l_tc = t_cycle if (t_cycle is not None and w["t_cycle_weight"] != 0) else z
    l2_mean = F.mse_loss(rgb_pred, rgb_gt) if (w["rgb_weight"] != 0 or w["depth_weight"] != 0) else z
    loss = (w["rgb_weight"] * l_rgb + w["depth_weight"] * l_depth + w["weight_dist_1st_loss"] * l_d1
            + w["weight_dist_2nd_loss"] * l_d2 + w["pc_weight"] * l_pc + w["rgb_s_weight"] * l_rgbs
            + w["depth_consistency_weight"] * l_dc + w["t_cycle_weight"] * l_tc)
    return {"loss": loss, "loss_rgb": l_rgb, "loss_depth": l_depth, "l2_mean": l2_mean,
            "loss_dist_1st": l_d1, "loss_dist_2nd": l_d2, "loss_pc": l_pc, "loss_rgb_s": l_rgbs,
            "loss_depth_consistency": l_dc, "loss_t_cycle": l_tc}


def anneal(start, end, anneal_start_epoch, anneal_epochs, current):
    """training.py:204-212."""
    if current <= anneal_start_epoch:
        return start
    if current >= anneal_start_epoch + anneal_epochs:
        return end
    return start + (end - start) * (current - anneal_start_epoch) / anneal_epochs


def mse2psnr(mse: float) -> float:
    """common.py:623-630."""
    return float(-10.0 * math.log10(max(mse, 1e-10)))


# ----------------------------------------------------------------------------
# one training step of the pure render path (config 2), training.py:70-100 + 214-416
# ----------------------------------------------------------------------------
def camera_K(h: int, w: int, fx: float, fy: float, dtype=torch.float32):
    """dataset.py:83-86."""
    return torch.tensor([[2 * fx / w, 0, 0, 0], [0, -2 * fy / h, 0, 0], [0, 0, -1, 0], [0, 0, 0, 1]],
                        dtype=dtype).unsqueeze(0)


def train_step_render(model: OracleNerf, optimizer, img, depth_img, camera_mat, c2w, scale_mat,
                      ray_idx, noise, cfg_render=None, rgb_weight=1.0, depth_weight=0.04,
                      rgb_loss_type="l2", chunk=None):
    """training.py:70-100 with compute_loss restricted to the render branch
    (training.py:277-303; losses rgb + depth as configured for epoch 0 of straight_d1
    minus the reference-image branch).  ``ray_idx``/``noise`` are injected."""
    optimizer.zero_grad()
    _, _, h, w = img.shape
    world_mat = torch.inverse(c2w).unsqueeze(0)                           # training.py:257
    img_flat = img.view(1, 3, h * w).permute(0, 2, 1)
    rgb_gt = img_flat[:, ray_idx]                                          # training.py:285-286
    p = arange_pixels(h, w, device=img.device, dtype=img.dtype)[1][:, ray_idx]   # training.py:287-288
    depth = F.interpolate(depth_img, (h, w), mode="area").view(1, 1, -1).permute(0, 2, 1)[:, ray_idx]
    out = render_nope_nerf(model, p, depth, camera_mat, world_mat, scale_mat, cfg_render, noise, chunk=chunk)
    ld = total_loss(out["rgb"], rgb_gt, out["depth_pred"], out["depth_gt"],
                    {"rgb_weight": rgb_weight, "depth_weight": depth_weight}, rgb_loss_type)
    ld["loss"].backward()
    optimizer.step()
    return ld, out


# ----------------------------------------------------------------------------
# the full NoPe-NeRF step (config 3): pose + distortion learning, point-cloud and
# reprojection terms of the image pair (training.py:214-416, losses.py:105-228,
# common.py:75-109, 436-457)
# ----------------------------------------------------------------------------
def grid_values(tensor, p, mode="bilinear", align_corners=True):
    """get_tensor_values, common.py:75-109, with scale=False, detach=False, detach_p=False
    (the arguments of training.py:370, 378): grid_sample of [B,C,H,W] at p [B,N,2] -> [B,N,C]."""
    v = F.grid_sample(tensor, p.unsqueeze(1), mode=mode, align_corners=align_corners).squeeze(2)
    return v.permute(0, 2, 1)


def project_to_cam(points, camera_mat):
    """common.py:436-457: K [x, y, z, 1]^T, perspective divide, |xy| <= 1 validity."""
    B, N, _ = points.shape
    hom = torch.cat([points.permute(0, 2, 1), torch.ones(B, 1, N, dtype=points.dtype, device=points.device)], 1)
    xy = (camera_mat @ hom)[:, :3].permute(0, 2, 1)
    xy = xy[..., :2] / xy[..., 2:]
    valid = (xy.abs().max(dim=-1)[0] <= 1).unsqueeze(-1)
    return xy, valid


def rgb_s_loss_ref(rgb1, rgb2, valid_points, with_ssim=False):
    """losses.py:152-159 (+ mean_on_mask :79-87); SSIM (losses.py:232-263) when with_ssim,
    applied to the (B,H,W,3) tensors exactly as the reference passes them."""
    diff = (rgb1 - rgb2).abs().clamp(0, 1)
    if with_ssim:
        diff = 0.15 * diff + 0.85 * ssim_map(rgb1, rgb2)
    return mean_on_mask(diff, valid_points)


def ssim_map(x, y):
    """losses.py:232-263: 3x3 mean-pool SSIM dissimilarity with reflection padding."""
    pad = nn.ReflectionPad2d(1)
    pool = nn.AvgPool2d(3, 1)
    x, y = pad(x), pad(y)
    mu_x, mu_y = pool(x), pool(y)
    sx = pool(x ** 2) - mu_x ** 2
    sy = pool(y ** 2) - mu_y ** 2
    sxy = pool(x * y) - mu_x * mu_y
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    n = (2 * mu_x * mu_y + C1) * (2 * sxy + C2)
    d = (mu_x ** 2 + mu_y ** 2 + C1) * (sx + sy + C2)
    return torch.clamp((1 - n / d) / 2, 0, 1)


def compute_loss_full(model, pose, distortion, data, tcfg, rcfg, epoch, scheduling_start, ray_idx, noise):
    """Trainer.compute_loss (training.py:214-416) with the reference image (the pair
    terms of :305-405) on the CPU.  ``pose`` = {"r", "t", "init_c2w"} (LearnPose
    parameters, poses.py:6-33), ``distortion`` = {"scales", "shifts", "fix_scaleN"}
    (Learn_Distortion, distortions.py:4-27); ``ray_idx`` and ``noise`` are injected
    (training.py:277, rendering.py:189)."""
    names = ["rgb_weight", "depth_weight", "pc_weight", "rgb_s_weight", "depth_consistency_weight",
             "weight_dist_2nd_loss", "weight_dist_1st_loss", "t_cycle_weight"]
    w = {n: anneal(tcfg[n][0], tcfg[n][1], scheduling_start, tcfg["annealing_epochs"], epoch) for n in names}
    rgb_loss_type = "l1" if epoch < tcfg["annealing_epochs"] + scheduling_start else "l2"     # :228
    render_model = w["rgb_weight"] != 0.0 or w["depth_weight"] != 0.0
    use_ref = w["pc_weight"] != 0.0 or w["rgb_s_weight"] != 0.0 or w["t_cycle_weight"] != 0.0
    nl = tcfg["nearest_limit"]
    img = data["img"]
    depth_input = data["img.depth"].unsqueeze(1)
    camera_mat = data["img.camera_mat"]
    scale_mat = data["img.scale_mat"]
    img_idx = int(data["img.idx"])
    pose_gt = data["img.pose_gt"]
    B, _, h, w_ = img.shape
    _, _, h_depth, w_depth = depth_input.shape
    num_cams = pose["r"].shape[0]
    world_mat_gt = torch.inverse(pose_gt).unsqueeze(0)                        # :254
    c2w = learn_pose_forward(pose["r"], pose["t"], pose["init_c2w"], img_idx)   # :257
    world_mat = torch.inverse(c2w).unsqueeze(0)
    scale_input, shift_input = learn_distortion_forward(distortion["scales"], distortion["shifts"], img_idx,
                                                        distortion["fix_scaleN"])                 # :260-264
    depth_input = depth_input * scale_input + shift_input                    # shift_first False
    img_flat = img.view(B, 3, h * w_).permute(0, 2, 1)
    rgb_gt = img_flat[:, ray_idx]                                             # :285-286
    p = arange_pixels(h, w_, device=img.device, dtype=img.dtype)[1][:, ray_idx]   # :287-288
    out = {}
    if render_model:                                                          # :290-303
        depth = F.interpolate(depth_input, (h, w_), mode="area").reshape(1, -1, 1)[:, ray_idx]
        out = render_nope_nerf(model, p, depth, camera_mat, world_mat, scale_mat, rcfg, noise)
    terms = {}
    if use_ref:                                                               # :305-405
        ref_img = data["img.ref_imgs"]
        depth_ref = data["img.ref_depths"].unsqueeze(1)
        ref_idx = int(data["img.ref_idxs"])
        ref_pose_gt = data["img.ref_pose_gt"]
        ref_Rt_gt = torch.inverse(ref_pose_gt).unsqueeze(0)
        c2w_ref = learn_pose_forward(pose["r"], pose["t"], pose["init_c2w"], ref_idx)
        scale_ref, shift_ref = learn_distortion_forward(distortion["scales"], distortion["shifts"], ref_idx,
                                                        distortion["fix_scaleN"])
        depth_ref = scale_ref * depth_ref + shift_ref
        if tcfg["detach_ref_img"]:
            c2w_ref, scale_ref, shift_ref, depth_ref = (c2w_ref.detach(), scale_ref.detach(), shift_ref.detach(),
                                                        depth_ref.detach())
        ref_Rt = torch.inverse(c2w_ref).unsqueeze(0)
        if img_idx < num_cams - 1:                                            # :329-343
            d1, d2, img1, img2 = depth_input, depth_ref, img, ref_img
            Rt_rel_12 = ref_Rt @ torch.inverse(world_mat)
            Rt_rel_12_gt = ref_Rt_gt @ torch.inverse(world_mat_gt)
            scale1 = scale_input
        else:                                                                 # :344-358
            d1, d2, img1, img2 = depth_ref, depth_input, ref_img, img
            Rt_rel_12 = world_mat @ torch.inverse(ref_Rt)
            Rt_rel_12_gt = world_mat_gt @ torch.inverse(ref_Rt_gt)
            scale1 = scale_ref
        R_rel_12, t_rel_12 = Rt_rel_12[:, :3, :3], Rt_rel_12[:, :3, 3]
        res = (int(h_depth / tcfg["pc_ratio"]), int(w_depth / tcfg["pc_ratio"]))   # :360-361
        p_pc = arange_pixels(res[0], res[1], device=img.device, dtype=img.dtype)[1]
        d1 = F.interpolate(d1, res, mode="nearest")
        d2 = F.interpolate(d2, res, mode="nearest")
        d1 = torch.where(d1 < nl, torch.full_like(d1, nl), d1)              # d1[d1 < nl] = nl
        d2 = torch.where(d2 < nl, torch.full_like(d2, nl), d2)
        pc1 = transform_to_world(p_pc, d1.view(1, -1, 1), camera_mat)
        pc2 = transform_to_world(p_pc, d2.view(1, -1, 1), camera_mat)
        if w["rgb_s_weight"] != 0.0:                                         # :367-390
            i1 = F.interpolate(img1, res, mode="bilinear")
            i2 = F.interpolate(img2, res, mode="bilinear")
            rgb_pc1 = grid_values(i1, p_pc)
            src = pc1.detach().clone() if tcfg["detach_rgbs_scale"] else pc1
            pc1_rot = src @ R_rel_12.transpose(1, 2) + t_rel_12
            bad = (-pc1_rot[:, :, 2:] < nl).expand_as(pc1_rot)
            pc1_rot = torch.where(bad, torch.full_like(pc1_rot, nl), pc1_rot)  # pc1_rotated[mask] = nl
            p_re, valid = project_to_cam(pc1_rot, camera_mat)
            rgb_proj = grid_values(i2, p_re)
            terms["rgb_s"] = rgb_s_loss_ref(rgb_pc1.view(B, res[0], res[1], 3), rgb_proj.view(B, res[0], res[1], 3),
                                            valid.view(B, res[0], res[1], 1), tcfg.get("with_ssim", False))
        if tcfg["scale_pcs"]:                                                 # :391-393
            pc1 = pc1 / scale1
            pc2 = pc2 / scale1
        X = pc1 @ R_rel_12.transpose(1, 2) + t_rel_12
        if w["pc_weight"] != 0.0:
            terms["pc"] = pc_loss(X, pc2)
        if w["t_cycle_weight"] != 0.0:                                        # losses.py:161-162
            terms["t_cycle"] = t_cycle_loss(Rt_rel_12, Rt_rel_12_gt)
    rgb_pred = out.get("rgb")
    dgt = out.get("depth_gt")
    if render_model and tcfg["detach_gt_depth"]:
        dgt = dgt.detach()
    ld = total_loss(rgb_pred, rgb_gt, out.get("depth_pred"), dgt, w, rgb_loss_type, pc=terms.get("pc"),
                    rgb_s=terms.get("rgb_s"), t_list=pose["t"], t_cycle=terms.get("t_cycle"),
                    depth_loss_type=tcfg.get("depth_loss_type", "l1"))
    ld["scale"], ld["shift"] = scale_input, shift_input
    return ld


# ----------------------------------------------------------------------------
# geometry visualisation: sphere-bounded ray marching, secant refinement and Phong
# shading of the occupancy surface (rendering.py:199-460)
# ----------------------------------------------------------------------------
def get_sphere_intersection(cam_loc, ray_directions, r=1.0):
    """rendering.py:447-468: near/far distances of the rays to the sphere |x| = r (0 without
    an intersection), clamped at 0.  cam_loc [n_imgs, 3], ray_directions [n_imgs, n_pix, 3]."""
    n_imgs, n_pix, _ = ray_directions.shape
    cam = cam_loc.unsqueeze(-1)
    ray_cam_dot = torch.bmm(ray_directions, cam).squeeze()
    under_sqrt = (ray_cam_dot ** 2 - (cam.norm(2, 1) ** 2 - r ** 2)).reshape(-1)
    mask = under_sqrt > 0
    inter = torch.zeros(n_imgs * n_pix, 2, dtype=ray_directions.dtype)
    inter[mask] = torch.sqrt(under_sqrt[mask]).unsqueeze(-1) * torch.tensor([-1.0, 1.0], dtype=inter.dtype)
    inter[mask] -= ray_cam_dot.reshape(-1)[mask].unsqueeze(-1)
    return inter.reshape(n_imgs, n_pix, 2).clamp_min(0.0), mask.reshape(n_imgs, n_pix)


def secant(model, f_low, f_high, d_low, d_high, n_secant_steps, ray0, ray_dir, tau):
    """rendering.py:405-436."""
    d_pred = -f_low * (d_high - d_low) / (f_high - f_low) + d_low
    for _ in range(n_secant_steps):
        p_mid = ray0 + d_pred.unsqueeze(-1) * ray_dir
        f_mid = model.occupancy(p_mid)[..., 0] - tau
        low = f_mid < 0
        d_low = torch.where(low, d_pred, d_low)
        f_low = torch.where(low, f_mid, f_low)
        d_high = torch.where(low, d_high, d_pred)
        f_high = torch.where(low, f_high, f_mid)
        d_pred = -f_low * (d_high - d_low) / (f_high - f_low) + d_low
    return d_pred


def ray_marching(model, ray0, ray_direction, tau=0.5, n_steps=512, n_secant_steps=8, depth_range=(0.0, 2.4),
                 rad=1.0):
    """rendering.py:262-403: n_steps samples from depth_range[0] to the far sphere
    intersection, first sign change of occupancy - tau from outside to inside, secant
    refinement; inf where none, 0 where the first sample is already occupied."""
    B, n_pts, _ = ray0.shape
    d_int, _ = get_sphere_intersection(ray0[:, 0], ray_direction, r=rad)
    d_far = d_int[..., 1]
    t = torch.linspace(0, 1, steps=n_steps, dtype=ray0.dtype).view(1, 1, n_steps, 1)
    d_prop = depth_range[0] * (1.0 - t) + d_far.view(1, -1, 1, 1) * t
    p_prop = ray0.unsqueeze(2) + ray_direction.unsqueeze(2) * d_prop
    val = (model.occupancy(p_prop.reshape(-1, 3)) - tau).view(B, n_pts, n_steps)
    mask_0_not_occ = val[:, :, 0] < 0
    sign = torch.cat([torch.sign(val[:, :, :-1] * val[:, :, 1:]), torch.ones(B, n_pts, 1, dtype=val.dtype)], -1)
    cost = sign * torch.arange(n_steps, 0, -1, dtype=val.dtype)
    values, idx = torch.min(cost, -1)
    mask_sign_change = values < 0
    mask_neg_to_pos = torch.gather(val, 2, idx.unsqueeze(-1)).squeeze(-1) < 0
    mask = mask_sign_change & mask_neg_to_pos & mask_0_not_occ
    dp = d_prop.expand(B, n_pts, n_steps, 1)[..., 0]
    d_low = torch.gather(dp, 2, idx.unsqueeze(-1)).squeeze(-1)[mask]
    f_low = torch.gather(val, 2, idx.unsqueeze(-1)).squeeze(-1)[mask]
    idx_h = torch.clamp(idx + 1, max=n_steps - 1)
    d_high = torch.gather(dp, 2, idx_h.unsqueeze(-1)).squeeze(-1)[mask]
    f_high = torch.gather(val, 2, idx_h.unsqueeze(-1)).squeeze(-1)[mask]
    d_out = torch.ones(B, n_pts, dtype=ray0.dtype)
    if mask.any():
        d_out[mask] = secant(model, f_low, f_high, d_low, d_high, n_secant_steps, ray0[mask],
                             ray_direction[mask], tau)
    d_out[~mask] = float("inf")
    d_out[~mask_0_not_occ] = 0.0
    return d_out


def phong_renderer(model, pixels, camera_mat, world_mat, scale_mat, rad=4.0, n_steps=512):
    """rendering.py:199-258: surface by ray marching, Phong-lit normals (ambient 0.3,
    diffuse 0.7, headlight from the camera direction), background 1; also the field's
    colour at the surface ('rgb_surf')."""
    B, n, _ = pixels.shape
    pix_w = image_points_to_world(pixels, camera_mat, world_mat, scale_mat)
    cam_w = origin_to_world(n, camera_mat, world_mat, scale_mat)
    ray = pix_w - cam_w
    ray = ray / ray.norm(2, 2).unsqueeze(-1)
    light_src = cam_w[0, 0]
    light = (light_src / light_src.norm(2)).unsqueeze(1)
    diffuse_per = torch.tensor([0.7, 0.7, 0.7], dtype=pixels.dtype)
    ambient = torch.tensor([0.3, 0.3, 0.3], dtype=pixels.dtype)
    with torch.no_grad():
        d_i = ray_marching(model, cam_w, ray, n_steps=n_steps, n_secant_steps=8, rad=rad)
    zero_occ = d_i == 0
    mask_pred = get_mask(d_i)
    dists = torch.ones_like(d_i)
    dists[mask_pred] = d_i[mask_pred]
    dists[zero_occ] = 0.0
    obj = (mask_pred & ~zero_occ)[0]
    dists = dists[0]
    cam_f, ray_f = cam_w.reshape(-1, 3), ray.reshape(-1, 3)
    points = cam_f + ray_f * dists.unsqueeze(-1)
    view = -ray_f
    rgb = torch.ones_like(points)
    surf, surf_view = points[obj], view[obj]
    grad = model.gradient(surf)[:, 0, :]
    normals = grad / grad.norm(2, 1, keepdim=True)
    diffuse = torch.mm(normals, light).clamp_min(0).repeat(1, 3) * diffuse_per.unsqueeze(0)
    rgb[obj] = (ambient.unsqueeze(0) + diffuse).clamp_max(1.0)
    rgb_surf = torch.zeros(B * n, 3, dtype=pixels.dtype)
    with torch.no_grad():
        rgb_surf[obj] = model(surf, surf_view)[0]
    return {"rgb": rgb.reshape(B, -1, 3), "normal": None, "rgb_surf": rgb_surf.reshape(B, -1, 3),
            "d_i": d_i, "mask": obj}

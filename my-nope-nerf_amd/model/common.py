"""Camera / pose helpers of the hot path (drop-in subset of model/common.py).

Device-agnostic (the reference hard-codes ``device=cuda`` defaults, common.py:113); the
three 4x4 inversions of every unprojection (common.py:139-141, 205-208) are composed
once per call into a single camera-to-world matrix.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from . import rays as _rays


def arange_pixels(resolution=(128, 128), batch_size=1, image_range=(-1.0, 1.0), device=torch.device("cpu")):
    """common.py:13-40 -> (integer (x, y) locations [B, H*W, 2], scaled locations)."""
    h, w = resolution
    ys, xs = torch.meshgrid(torch.arange(h, device=device), torch.arange(w, device=device), indexing="ij")
    loc = torch.stack([xs, ys], dim=-1).long().view(1, -1, 2).repeat(batch_size, 1, 1)
    span = image_range[1] - image_range[0]
    scaled = loc.float()
    scaled[:, :, 0] = span * scaled[:, :, 0] / (w - 1) - span / 2
    scaled[:, :, 1] = span * scaled[:, :, 1] / (h - 1) - span / 2
    return loc, scaled


def get_mask(t):
    """common.py:60-72: finite entries."""
    if isinstance(t, np.ndarray):
        return np.isfinite(t)
    return (t.abs() != math.inf) & ~torch.isnan(t)


def inv(m):
    """torch.inverse of [..., 4, 4]: the HIP batched inverse for device tensors (one launch,
    no host-side singularity check or LAPACK info read-back), torch for host tensors."""
    return _rays.inv(m)


def unproject_matrix(camera_mat, world_mat, scale_mat):
    """scale^-1 @ world^-1 @ K^-1 evaluated in the reference's association order
    (common.py:139-141); one camera on the device is a single HIP launch."""
    if camera_mat.is_cuda and camera_mat.numel() == world_mat.numel() == scale_mat.numel() == 16:
        return _rays.unproject_matrix(camera_mat, world_mat, scale_mat)
    return (inv(scale_mat) @ inv(world_mat)) @ inv(camera_mat)


def transform_to_world(pixels, depth, camera_mat, world_mat=None, scale_mat=None, invert=True, device=None):
    """common.py:112-160: world points of pixels [B,N,2] at depth [B,N,1]."""
    eye = torch.eye(4, dtype=camera_mat.dtype, device=camera_mat.device).unsqueeze(0)
    world_mat = eye if world_mat is None else world_mat
    scale_mat = eye if scale_mat is None else scale_mat
    if invert:
        M = unproject_matrix(camera_mat, world_mat, scale_mat)
    else:
        M = scale_mat @ world_mat @ camera_mat
    hom = torch.cat([pixels * depth, depth, torch.ones_like(depth)], dim=-1).transpose(1, 2)
    return (M @ hom)[:, :3].transpose(1, 2)


def origin_to_world(n_points, camera_mat, world_mat, scale_mat, invert=True):
    """common.py:186-215: camera centre repeated n_points times."""
    M = unproject_matrix(camera_mat, world_mat, scale_mat) if invert else scale_mat @ world_mat @ camera_mat
    B = camera_mat.shape[0]
    p = torch.zeros(B, 4, n_points, device=camera_mat.device, dtype=camera_mat.dtype)
    p[:, -1] = 1.0
    return (M @ p)[:, :3].transpose(1, 2)


def image_points_to_world(image_points, camera_mat, world_mat, scale_mat, invert=True):
    """common.py:218-237: unprojection at depth 1."""
    d = torch.ones(*image_points.shape[:2], 1, device=image_points.device, dtype=image_points.dtype)
    return transform_to_world(image_points, d, camera_mat, world_mat, scale_mat, invert)


def get_tensor_values(tensor, p, mode="nearest", scale=True, detach=True, detach_p=True, align_corners=False):
    """common.py:75-109: grid_sample lookup of [B,C,H,W] at p [B,N,2]."""
    _, _, h, w = tensor.shape
    if detach_p:
        p = p.detach()
    if scale:
        p = p.clone()
        p[:, :, 0] = 2.0 * p[:, :, 0] / w - 1
        p[:, :, 1] = 2.0 * p[:, :, 1] / h - 1
    v = torch.nn.functional.grid_sample(tensor, p.unsqueeze(1), mode=mode, align_corners=align_corners)
    v = v.squeeze(2)
    if detach:
        v = v.detach()
    return v.permute(0, 2, 1)


def project_to_cam(points, camera_mat, device=None):
    """common.py:436-457: project [B,N,3] with K; returns xy [B,N,2] and |xy|<=1 mask."""
    B, N, _ = points.shape
    hom = torch.cat([points, torch.ones(B, N, 1, device=points.device, dtype=points.dtype)], -1).transpose(1, 2)
    xyz = (camera_mat @ hom)[:, :3].transpose(1, 2)
    xy = xyz[..., :2] / xyz[..., 2:]
    valid = (xy.abs().max(dim=-1)[0] <= 1).unsqueeze(-1)
    return xy, valid


def vec2skew(v):
    """common.py:277-287."""
    z = torch.zeros_like(v[0:1])
    return torch.stack([torch.cat([z, -v[2:3], v[1:2]]),
                        torch.cat([v[2:3], z, -v[0:1]]),
                        torch.cat([-v[1:2], v[0:1], z])], dim=0)


def Exp(r):
    """common.py:290-299: axis-angle -> SO(3), theta = |r| + 1e-15."""
    K = vec2skew(r)
    th = r.norm() + 1e-15
    I = torch.eye(3, dtype=r.dtype, device=r.device)
    return I + (torch.sin(th) / th) * K + ((1 - torch.cos(th)) / th ** 2) * (K @ K)


def convert3x4_4x4(m):
    """common.py:312-330."""
    if torch.is_tensor(m):
        if m.dim() == 3:
            out = torch.cat([m, torch.zeros_like(m[:, 0:1])], dim=1)
            out[:, 3, 3] = 1.0
            return out
        # [0, 0, 0, 1] built on the device (a host->device copy breaks hipGraph capture)
        bottom = torch.eye(4, dtype=m.dtype, device=m.device)[3:]
        return torch.cat([m, bottom], dim=0)
    if m.ndim == 3:
        out = np.concatenate([m, np.zeros_like(m[:, 0:1])], axis=1)
        out[:, 3, 3] = 1.0
        return out
    out = np.concatenate([m, np.array([[0, 0, 0, 1]], dtype=m.dtype)], axis=0)
    out[3, 3] = 1.0
    return out


def make_c2w(r, t):
    """common.py:301-310: [Exp(r) | t] as 4x4."""
    return convert3x4_4x4(torch.cat([Exp(r), t.unsqueeze(1)], dim=1))


def get_ndc_rays_fxfy(fxfy, near, rays_o, rays_d):
    """common.py:632-675: rays to NDC (LLFF configs)."""
    t = -(near + rays_o[..., 2]) / rays_d[..., 2]
    o = rays_o + t[..., None] * rays_d
    ox, oy = o[..., 0] / o[..., 2], o[..., 1] / o[..., 2]
    fx, fy = fxfy[0], fxfy[1]
    o2 = 1.0 + 2.0 * near / o[..., 2]
    o_ndc = torch.stack([-1.0 / (1 / fx) * ox, -1.0 / (1 / fy) * oy, o2], -1)
    d_ndc = torch.stack([-1.0 / (1 / fx) * (rays_d[..., 0] / rays_d[..., 2] - ox),
                         -1.0 / (1 / fy) * (rays_d[..., 1] / rays_d[..., 2] - oy),
                         1 - o2], -1)
    return o_ndc, d_ndc


def mse2psnr(mse):
    """common.py:623-630."""
    mse = np.maximum(mse, 1e-10)
    return (-10.0 * np.log10(mse)).astype(np.float32)


# ---------------------------------------------------------------------------
# the rest of the reference module's public helpers (host-side utilities the drivers
# import: train.py:17, vis/render.py:12, evaluation/*): not on the hot path
# ---------------------------------------------------------------------------
from .camera_paths import (create_spheric_poses, generate_spiral_nerf, get_poses_at_times,  # noqa: E402,F401
                           interp_poses, interp_poses_bspline, interp_t, normalize, poses_avg,
                           render_path_spiral, scipy_bspline, viewmatrix)


def backup(out_dir, config):
    """common.py:492-508: snapshot the run's config and sources into <out_dir>/backup
    (config.yaml, train.py, configs/default.yaml and the files of ./model and
    ./dataloading, relative to the working directory as the reference resolves them).
    Sources absent from the working directory are skipped instead of raising."""
    import shutil
    dst = os.path.join(out_dir, "backup")
    os.makedirs(dst, exist_ok=True)
    shutil.copyfile(config, os.path.join(dst, "config.yaml"))
    for f in ("train.py", os.path.join("configs", "default.yaml")):
        if os.path.isfile(f):
            shutil.copy(f, dst)
    for d in ("model", "dataloading"):
        if not os.path.isdir(d):
            continue
        sub = os.path.join(dst, d)
        os.makedirs(sub, exist_ok=True)
        for f in sorted(os.listdir(d)):
            if os.path.isfile(os.path.join(d, f)):
                shutil.copy(os.path.join(d, f), sub)


def to_pytorch(tensor, return_type=False):
    """common.py:42-57: numpy -> torch (and whether the input was numpy)."""
    was_np = isinstance(tensor, np.ndarray)
    if was_np:
        tensor = torch.from_numpy(tensor)
    return (tensor, was_np) if return_type else tensor


def transform_to_camera_space(p_world, camera_mat, world_mat, scale_mat):
    """common.py:163-183: K @ world @ scale applied to world points [B,N,3]."""
    hom = torch.cat([p_world, torch.ones_like(p_world[..., :1])], dim=-1).transpose(1, 2)
    return (camera_mat @ world_mat @ scale_mat @ hom)[:, :3].transpose(1, 2)


def check_weights(params):
    """common.py:240-248: warn about NaN parameters."""
    import logging
    for k, v in params.items():
        if torch.isnan(v).any():
            logging.getLogger(__name__).warning("NaN Values detected in model weight %s.", k)


def check_tensor(tensor, tensorname="", input_tensor=None):
    """common.py:251-262."""
    import logging
    if torch.isnan(tensor).any():
        log = logging.getLogger(__name__)
        log.warning("Tensor %s contains nan values.", tensorname)
        if input_tensor is not None:
            log.warning("Input was: %s", input_tensor)


def normalize_tensor(tensor, min_norm=1e-5, feat_dim=-1):
    """common.py:265-275."""
    return tensor / tensor.norm(dim=feat_dim, keepdim=True).clamp_min(min_norm)


def reprojection(pixels, depth, Rt_ref, world_mat, camera_mat):
    """common.py:405-434: pixels [B,N,2] at depth -> the reference camera's image plane;
    returns (xy [B,N,2], valid [B,N,1] float)."""
    pixels, was_np = to_pytorch(pixels, True)
    depth, camera_mat, Rt_ref = to_pytorch(depth), to_pytorch(camera_mat), to_pytorch(Rt_ref)
    d = depth.reshape(1, -1, 1)
    hom = torch.cat([pixels * d, d, torch.ones_like(d)], dim=-1).transpose(1, 2)
    M = camera_mat @ Rt_ref @ torch.inverse(world_mat) @ torch.inverse(camera_mat)
    xyz = (M @ hom)[:, :3].transpose(1, 2)
    xy = xyz[..., :2] / xyz[..., 2:]
    valid = (xy.abs().max(dim=-1)[0] <= 1).unsqueeze(-1).float()
    return (xy.numpy() if was_np else xy), valid


def skew_symmetric(w):
    """common.py:459-465: batched [.., 3] -> [.., 3, 3]."""
    w0, w1, w2 = w.unbind(dim=-1)
    o = torch.zeros_like(w0)
    return torch.stack([torch.stack([o, -w2, w1], -1), torch.stack([w2, o, -w0], -1),
                        torch.stack([-w1, w0, o], -1)], -2)


def _taylor(x, nth, step):
    """sum_i (-1)^i x^(2i) / prod(...) with the reference's running denominators."""
    out = torch.zeros_like(x)
    den = 1.0
    for i in range(nth + 1):
        den = step(i, den)
        out = out + (-1) ** i * x ** (2 * i) / den
    return out


def taylor_A(x, nth=10):
    """common.py:467-473: sin(x)/x."""
    return _taylor(x, nth, lambda i, d: d * (2 * i) * (2 * i + 1) if i > 0 else d)


def taylor_B(x, nth=10):
    """common.py:475-481: (1-cos(x))/x^2."""
    return _taylor(x, nth, lambda i, d: d * (2 * i + 1) * (2 * i + 2))


def taylor_C(x, nth=10):
    """common.py:483-490: (x-sin(x))/x^3."""
    return _taylor(x, nth, lambda i, d: d * (2 * i + 2) * (2 * i + 3))


def convert2mip(pts):
    """common.py:616-621: contract points outside the unit ball to radius < 2."""
    n = pts.norm(dim=-1, keepdim=True)
    return torch.where(n >= 1.0, (2 - 1.0 / n) * (pts / n), pts)


def compute_errors(gt, pred):
    """common.py:676-694: depth error metrics (abs_rel, sq_rel, rmse, rmse_log, a1, a2, a3)."""
    ratio = np.maximum(gt / pred, pred / gt)
    a1, a2, a3 = ((ratio < 1.25 ** k).mean() for k in (1, 2, 3))
    rmse = np.sqrt(((gt - pred) ** 2).mean())
    rmse_log = np.sqrt(((np.log(gt) - np.log(pred)) ** 2).mean())
    abs_rel = np.mean(np.abs(gt - pred) / gt)
    sq_rel = np.mean((gt - pred) ** 2 / gt)
    return abs_rel, sq_rel, rmse, rmse_log, a1, a2, a3

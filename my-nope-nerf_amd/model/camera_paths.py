"""Novel-view camera trajectories of the render caller (drop-in for model/common.py:333-403
and :511-615, imported by vis/render.py:12 through ``model.common``).

Host-side pose arithmetic over a handful of 4x4 matrices per frame: numpy / scipy, no
device work.  The frames these poses produce are rendered by Extract_Images through the
sharded HIP path (extracting_images.py, render_dist.py).
"""
from __future__ import annotations

import numpy as np
import torch
from scipy import interpolate as _si
from scipy.spatial.transform import Rotation, Slerp


def _to_4x4(m):
    """[N,3,4] torch -> [N,4,4] (common.py:312-330 for batched tensors)."""
    bottom = torch.zeros(m.shape[0], 1, 4, dtype=m.dtype)
    bottom[:, 0, 3] = 1.0
    return torch.cat([m, bottom], dim=1)


def normalize(v):
    """common.py:371-373."""
    return v / np.linalg.norm(v)


def viewmatrix(z, up, pos):
    """common.py:374-380: [x | y | z | pos] 3x4 camera frame looking along z."""
    ez = normalize(z)
    ex = normalize(np.cross(up, ez))
    ey = normalize(np.cross(ez, ex))
    return np.stack([ex, ey, ez, pos], axis=1)


def poses_avg(poses):
    """common.py:393-403: mean camera of [N,3,5] poses (hwf in the last column)."""
    hwf = poses[0, :3, 4:5]
    centre = poses[:, :3, 3].mean(axis=0)
    return np.concatenate([viewmatrix(normalize(poses[:, :3, 2].sum(axis=0)), poses[:, :3, 1].sum(axis=0), centre),
                           hwf], axis=1)


def render_path_spiral(c2w, up, rads, focal, zdelta, zrate, rots, N):
    """common.py:381-392: N poses on an ellipse-spiral around c2w ([3,5]) looking at the
    focus point focal in front of it."""
    scale = np.append(np.asarray(rads, dtype=np.float64), 1.0)
    hwf = c2w[:, 4:5]
    target = c2w[:3, :4] @ np.array([0.0, 0.0, -focal, 1.0])
    out = []
    for th in np.linspace(0.0, 2.0 * np.pi * rots, N + 1)[:N]:
        local = np.array([0.2 * np.cos(th), -0.2 * np.sin(th), -0.1 * np.sin(th * zrate), 1.0]) * scale
        c = c2w[:3, :4] @ local
        out.append(np.concatenate([viewmatrix(normalize(c - target), up, c), hwf], axis=1))
    return out


def create_spheric_poses(radius, mean_h, n_poses=120):
    """common.py:333-369: n_poses cameras on a circle about the y axis, pitched by -15 deg."""
    phi = -np.pi / 12
    rot_phi = np.array([[1, 0, 0], [0, np.cos(phi), -np.sin(phi)], [0, np.sin(phi), np.cos(phi)]])
    trans = np.array([[1, 0, 0, 0], [0, 1, 0, 2 * mean_h], [0, 0, 1, -radius]], dtype=np.float64)
    flip = np.array([[-1, 0, 0], [0, 0, 1], [0, 1, 0]])
    poses = []
    for th in np.linspace(0, 2 * np.pi, n_poses + 1)[:n_poses]:
        rot_th = np.array([[np.cos(th), 0, -np.sin(th)], [0, 1, 0], [np.sin(th), 0, np.cos(th)]])
        poses.append(flip @ (rot_th @ rot_phi @ trans))
    return np.stack(poses, 0)


def interp_poses(c2ws, N_views):
    """common.py:511-522: N_views poses, rotations slerped and translations linearly
    interpolated (F.interpolate 'linear', align_corners=False) over the input cameras."""
    n = c2ws.shape[0]
    slerp = Slerp(np.linspace(0, 1, n), Rotation.from_matrix(c2ws[:, :3, :3].numpy()))
    rots = torch.tensor(slerp(np.linspace(0, 1, N_views)).as_matrix().astype(np.float32))
    trans = torch.nn.functional.interpolate(c2ws[:, :3, 3:].permute(2, 1, 0), size=N_views, mode="linear")
    return _to_4x4(torch.cat([rots, trans.permute(2, 1, 0)], dim=2))


def scipy_bspline(cv, n=100, degree=3, periodic=False):
    """common.py:563-589: n samples of the (clamped, or closed) B-spline through the
    control vertices cv."""
    cv = np.asarray(cv)
    count = cv.shape[0]
    if periodic:
        knots = np.arange(-degree, count + degree + 1)
        reps, extra = divmod(count + degree + 1, count)
        cv = np.roll(np.concatenate([cv] * reps + [cv[:extra]]), -1, axis=0)
        degree = int(np.clip(degree, 1, degree))
    else:
        degree = int(np.clip(degree, 1, count - 1))
        knots = np.clip(np.arange(count + degree + 1) - degree, 0, count - degree)
    top = count - (degree * (1 - periodic))
    return _si.BSpline(knots, cv, degree)(np.linspace(0, top, n))


def interp_poses_bspline(c2ws, N_novel_imgs, input_times, degree):
    """common.py:523-532: translations on a B-spline through the camera centres, rotations
    slerped at the input times."""
    trans = torch.tensor(scipy_bspline(c2ws[:, :3, 3].numpy(), n=N_novel_imgs, degree=degree,
                                       periodic=False).astype(np.float32)).unsqueeze(2)
    slerp = Slerp(input_times, Rotation.from_matrix(c2ws[:, :3, :3].numpy()))
    times = np.linspace(input_times[0], input_times[-1], N_novel_imgs)
    rots = torch.tensor(slerp(times).as_matrix().astype(np.float32))
    return _to_4x4(torch.cat([rots, trans], dim=2))


def interp_t(trans, input_times, target_times):
    """common.py:544-559: per target time, blend the translations of the nearest input
    times at or before / at or after it with the reference's weights."""
    out = []
    for t in target_times:
        d = t - input_times
        before = np.argmin(np.where(d < 0, 1000, d))       # smallest non-negative offset
        after = np.argmin(-np.where(d > 0, -1000, d))      # largest non-positive offset
        span = input_times[after] - input_times[before]
        out.append((t - input_times[before]) / span * trans[before] + (input_times[after] - t) / span * trans[after])
    return torch.stack(out, 0)


def get_poses_at_times(c2ws, input_times, target_times):
    """common.py:533-543."""
    slerp = Slerp(input_times, Rotation.from_matrix(c2ws[:, :3, :3].numpy()))
    rots = torch.tensor(slerp(target_times).as_matrix().astype(np.float32))
    return _to_4x4(torch.cat([rots, interp_t(c2ws[:, :3, 3:], input_times, target_times)], dim=2))


def generate_spiral_nerf(learned_poses, bds, N_novel_views, hwf):
    """common.py:591-615: a 2-turn spiral about the average learned camera, radii from the
    90th percentile of |t|, focus depth from the bounds bds; returns [N,3,4]."""
    lp = np.concatenate([learned_poses[:, :3, :4].detach().cpu().numpy(), hwf[:len(learned_poses)]], axis=-1)
    c2w = poses_avg(lp)
    up = normalize(lp[:, :3, 1].sum(0))
    near, far = bds.min() * 0.9, bds.max() * 5.0
    dt = 0.75
    focal = 1.0 / ((1.0 - dt) / near + dt / far)
    rads = np.percentile(np.abs(lp[:, :3, 3]), 90, 0)
    path = render_path_spiral(c2w, up, rads, focal, near * 0.2, zrate=0.5, rots=2, N=N_novel_views)
    return torch.tensor(np.stack(path).astype(np.float32))[:, :3, :4]

"""Shared test fixtures: configs and seeded synthetic V_KITTI-shaped inputs."""
from __future__ import annotations

import copy
import math

import torch

BASE_CFG = {
    "model": {"hidden_dim": 256, "pos_enc_levels": 10, "dir_enc_levels": 4, "occ_activation": "softplus",
              "num_layers": 8},
    "rendering": {"type": "nope_nerf", "n_max_network_queries": 64000, "white_background": False,
                  "radius": 4.0, "num_points": 128, "depth_range": [0.01, 10.0], "dist_alpha": False,
                  "use_ray_dir": True, "normalise_ray": True, "normal_loss": False,
                  "sample_option": "uniform", "outside_steps": 0},
    "depth": {"type": None},
    "distortion": {"learn_distortion": True, "fix_scaleN": True, "learn_scale": True, "learn_shift": True},
    "training": {"type": "nope_nerf", "n_training_points": 1024, "detach_gt_depth": False, "pc_ratio": 4,
                 "match_method": "dense", "shift_first": False, "detach_ref_img": True, "scale_pcs": True,
                 "detach_rgbs_scale": False, "vis_reprojection_every": 5000, "nearest_limit": 0.01,
                 "annealing_epochs": 0, "scheduling_start": 0, "rgb_weight": [1.0, 1.0],
                 "depth_weight": [0.04, 0.0], "weight_dist_2nd_loss": [0.0, 0.0],
                 "weight_dist_1st_loss": [0.0, 0.0], "pc_weight": [1.0, 0.0], "rgb_s_weight": [1.0, 0.0],
                 "depth_consistency_weight": [0.0, 0.0], "t_cycle_weight": [0.0, 0.0],
                 "depth_loss_type": "l1", "with_auto_mask": False, "with_ssim": False, "vis_geo": False,
                 "learning_rate": 0.001},
}


def make_cfg(hidden=256, S=128, **render):
    cfg = copy.deepcopy(BASE_CFG)
    cfg["model"]["hidden_dim"] = hidden
    cfg["rendering"]["num_points"] = S
    cfg["rendering"].update(render)
    return cfg


def camera_K(h, w, fx, fy):
    """dataset.py:83-86."""
    return torch.tensor([[2 * fx / w, 0, 0, 0], [0, -2 * fy / h, 0, 0], [0, 0, -1, 0], [0, 0, 0, 1]],
                        dtype=torch.float32).unsqueeze(0)


def rigid_c2w(seed=0, scale=0.3):
    g = torch.Generator().manual_seed(seed)
    r = (torch.rand(3, generator=g) - 0.5) * scale
    th = r.norm()
    k = r / th
    K = torch.tensor([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    Rm = torch.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * (K @ K)
    c2w = torch.eye(4)
    c2w[:3, :3] = Rm
    c2w[:3, 3] = (torch.rand(3, generator=g) - 0.5)
    return c2w


def synthetic_rays(R=1024, S=128, H=188, W=621, seed=0, zero_frac=0.05, fx=362.5):
    """A V_KITTI-shaped batch: R random pixels of an HxW image, depth prior U[1,8] with
    some zeros (mask exercise), a fixed rigid pose, stratified noise U[0,1)."""
    g = torch.Generator().manual_seed(seed)
    idx = torch.randperm(H * W, generator=g)[:R]
    rows, cols = idx // W, idx % W
    px = 2.0 * cols.float() / (W - 1) - 1.0
    py = 2.0 * rows.float() / (H - 1) - 1.0
    pixels = torch.stack([px, py], -1).unsqueeze(0)
    depth = 1.0 + 7.0 * torch.rand(1, R, 1, generator=g)
    depth[torch.rand(1, R, 1, generator=g) < zero_frac] = 0.0
    c2w = rigid_c2w(seed)
    return {"pixels": pixels, "depth": depth, "K": camera_K(H, W, fx, fx), "c2w": c2w,
            "w2c": torch.inverse(c2w).unsqueeze(0), "scale": torch.eye(4).unsqueeze(0),
            "noise": torch.rand(1, R, S, generator=g), "ray_idx": idx}


# ---- parity bar (BASELINE.json north_star: 1e-4 rel on rendered RGB / depth) -----------
RENDER_RTOL = 1e-4     # elementwise, relative to the oracle value
RENDER_ATOL = 1e-6     # absolute floor for values near zero (dark pixels, masked depths)


def elementwise_excess(a, b, rtol=RENDER_RTOL, atol=RENDER_ATOL):
    """max over elements of |a - b| / (rtol |b| + atol): <= 1 passes the elementwise bar
    |a - b| <= rtol |b| + atol."""
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs() / (rtol * b.abs() + atol)).max().item()


def assert_elementwise(a, b, rtol=RENDER_RTOL, atol=RENDER_ATOL, what=""):
    """|a - b| <= rtol |b| + atol for every element; the message carries the worst element
    and, as a diagnostic, the max-normalised error max|a-b| / max|b|."""
    a_, b_ = a.detach().double().cpu(), b.detach().double().cpu()
    assert a_.shape == b_.shape, (what, a_.shape, b_.shape)
    err = (a_ - b_).abs()
    lim = rtol * b_.abs() + atol
    ratio = err / lim
    if ratio.numel() and ratio.max().item() > 1.0:
        i = int(ratio.argmax())
        raise AssertionError(f"{what}: element {i}: |{a_.flatten()[i].item():.9g} - {b_.flatten()[i].item():.9g}| = "
                             f"{err.flatten()[i].item():.3g} > {rtol:g}*|b| + {atol:g} "
                             f"(max-normalised error {(err.max() / b_.abs().max().clamp_min(1e-30)).item():.3g})")

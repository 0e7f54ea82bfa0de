"""Synthetic V_KITTI-shaped workloads: the default config tree of
configs/default.yaml with the V_KITTI overrides the benchmarks and tests run, the camera
matrix of dataset.py:83-86, rigid poses and a resident data dict with the keys of
dataset.py:281-364.  There is no dataset offline, so every benchmark line says "synthetic"."""
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

# V_KITTI scene-1 shape (configs/V_KITTI/straight_d1.yaml:7,19-21; get_kittivirtual.py:11-13)
VKITTI_H, VKITTI_W, VKITTI_FOCAL = 188, 621, 362.5


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


def vkitti_scene(dev, seed=0, H=VKITTI_H, W=VKITTI_W, focal=VKITTI_FOCAL):
    """A V_KITTI-shaped data dict (dataset.py:281-364 keys) resident on ``dev``: a smooth
    textured image, a depth prior U[1, 8] with ~5 % holes, a fixed rigid camera.  Returns
    (data, c2w)."""
    g = torch.Generator().manual_seed(seed)
    yy, xx = torch.meshgrid(torch.linspace(0, 1, H), torch.linspace(0, 1, W), indexing="ij")
    img = torch.stack([0.5 + 0.4 * torch.sin(6 * xx + 2 * yy), 0.5 + 0.4 * torch.cos(5 * yy),
                       0.3 + 0.3 * xx * yy], 0).unsqueeze(0)
    img = (img + 0.02 * torch.rand(img.shape, generator=g)).clamp(0, 1)
    depth = 1.0 + 7.0 * torch.rand(1, H, W, generator=g)
    holes = torch.rand(1, H, W, generator=g) < 0.05
    depth[holes] = 0.0
    c2w = rigid_c2w(seed)
    data = {"img": img, "img.idx": torch.tensor([0]), "img.depth": depth, "img.depth_mask": ~holes,
            "img.camera_mat": camera_K(H, W, focal, focal), "img.scale_mat": torch.eye(4).unsqueeze(0),
            "img.pose_gt": c2w.unsqueeze(0)}
    for k, v in list(data.items()):
        if k not in ("img.idx", "img.depth_mask"):
            data[k] = v.to(dev)
    return data, c2w


def vkitti_pair_scene(dev, H=VKITTI_H, W=VKITTI_W, focal=VKITTI_FOCAL):
    """Config 3's two-view V_KITTI-shaped scene: two textured images with depth priors
    (U[1, 8], ~5 % holes) and camera 1 offset from camera 0, as two data dicts whose
    reference keys (dataset.py:330-364: img.ref_imgs / ref_depths / ref_idxs / ref_pose_gt)
    point at the other view.  Returns ([data view 0, data view 1], c2w [2, 4, 4])."""
    g = torch.Generator().manual_seed(0)
    yy, xx = torch.meshgrid(torch.linspace(0, 1, H), torch.linspace(0, 1, W), indexing="ij")
    imgs, depths = [], []
    for s in (0, 1):
        img = torch.stack([0.5 + 0.4 * torch.sin(6 * xx + 2 * yy + 0.3 * s), 0.5 + 0.4 * torch.cos(5 * yy),
                           0.3 + 0.3 * xx * yy], 0).unsqueeze(0)
        imgs.append((img + 0.02 * torch.rand(img.shape, generator=g)).clamp(0, 1).to(dev))
        d = 1.0 + 7.0 * torch.rand(1, H, W, generator=g)
        d[torch.rand(1, H, W, generator=g) < 0.05] = 0.0
        depths.append(d.to(dev))
    c2w = torch.stack([rigid_c2w(0), rigid_c2w(0)])
    c2w[1, :3, 3] += torch.tensor([0.1, 0.0, -0.2])
    K = camera_K(H, W, focal, focal).to(dev)
    datas = []
    for cam in (0, 1):
        ref = 1 - cam
        datas.append({"img": imgs[cam], "img.depth": depths[cam], "img.depth_mask": (depths[cam] > 0).cpu(),
                      "img.camera_mat": K, "img.scale_mat": torch.eye(4, device=dev).unsqueeze(0),
                      "img.pose_gt": c2w[cam].unsqueeze(0).to(dev), "img.idx": torch.tensor([cam]),
                      "img.ref_imgs": imgs[ref], "img.ref_depths": depths[ref], "img.ref_idxs": torch.tensor([ref]),
                      "img.ref_pose_gt": c2w[ref].unsqueeze(0).to(dev)})
    return datas, c2w

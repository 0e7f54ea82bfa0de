"""Losses of the training step (drop-in for model/losses.py:17-228).

Same ``Loss`` class, method names, weights dict and output keys.  Differences are
device hygiene only (no ``.cuda()``, no import-time ``SSIM().to('cuda')``,
losses.py:168-264) plus:
  * the dense point-cloud nearest neighbour (losses.py:129-144) runs in the nerf_hip
    chamfer kernel instead of materialising the (3, P, P) difference tensor;
  * the depth term accepts the dense (unmasked) render output + mask, giving the same
    value as the boolean-indexed form without a host sync.
"""
from __future__ import annotations

import torch
from torch import nn
from torch.nn import functional as F

from . import _hip
from .common import inv
from .rays import ray_loss


class Loss_Eval(nn.Module):
    def forward(self, rgb_pred, rgb_gt):
        return {"loss": F.mse_loss(rgb_pred, rgb_gt)}


def nearest_index(src, dst):
    """argmin_j |src[:, i] - dst[:, j]| for src (3,S), dst (3,D) on the HIP chamfer kernel."""
    x = src.detach().t().contiguous().float()
    y = dst.detach().t().contiguous().float()
    idx = torch.empty(x.shape[0], dtype=torch.int64, device=x.device)
    _hip.chamfer_nn(x, y, idx)
    return idx


class SSIM(nn.Module):
    """losses.py:232-263 (3x3 box-filter SSIM dissimilarity)."""

    def __init__(self):
        super().__init__()
        self.pool = nn.AvgPool2d(3, 1)
        self.refl = nn.ReflectionPad2d(1)
        self.C1, self.C2 = 0.01 ** 2, 0.03 ** 2

    def forward(self, x, y):
        x, y = self.refl(x), self.refl(y)
        mx, my = self.pool(x), self.pool(y)
        sx = self.pool(x ** 2) - mx ** 2
        sy = self.pool(y ** 2) - my ** 2
        sxy = self.pool(x * y) - mx * my
        n = (2 * mx * my + self.C1) * (2 * sxy + self.C2)
        d = (mx ** 2 + my ** 2 + self.C1) * (sx + sy + self.C2)
        return torch.clamp((1 - n / d) / 2, 0, 1)


_ssim = None


def compute_ssim_loss(x, y):
    global _ssim
    if _ssim is None:
        _ssim = SSIM()
    return _ssim(x, y)


_zeros = {}


def _zero(dev):
    """The 0-dim zero of skipped terms: one tensor per device (no fill launch per step).
    Callers only read it; it never requires grad."""
    key = str(dev)
    z = _zeros.get(key)
    if z is None:
        z = _zeros[key] = torch.zeros((), device=dev)
    return z


class Loss(nn.Module):
    def __init__(self, cfg=None):
        super().__init__()
        self.depth_loss_type = cfg["depth_loss_type"]
        self.cfg = cfg

    # ---- photometric / depth terms -------------------------------------------------
    def get_rgb_full_loss(self, rgb_values, rgb_gt, rgb_loss_type="l2"):
        """losses.py:28-33: summed error / number of rays."""
        diff = rgb_values - rgb_gt
        err = diff.abs().sum() if rgb_loss_type == "l1" else (diff * diff).sum()
        return err / float(rgb_values.shape[1])

    def depth_loss_dpt(self, pred_depth, gt_depth, weight=None):
        """losses.py:35-58: median/MAD normalised MSE."""
        def norm(d):
            t = torch.median(d)
            return (d - t) / torch.mean(torch.abs(d - t))
        p, g = norm(pred_depth), norm(gt_depth)
        if weight is not None:
            l = F.mse_loss(p, g, reduction="none") * weight
            return l.sum() / (weight.sum() + 1e-8)
        return F.mse_loss(p, g)

    def get_depth_loss(self, depth_pred, depth_gt, depth_mask=None):
        """losses.py:60-66.  With ``depth_mask`` the inputs are dense (R,) and the l1 mean
        runs over the masked rays: sum(|.| [mask]) / count(mask), no host sync."""
        if self.depth_loss_type == "l1":
            if depth_mask is None:
                return (depth_pred - depth_gt).abs().sum() / float(depth_pred.shape[0])
            err = torch.where(depth_mask, (depth_pred - depth_gt).abs(), 0.0)   # scalar 0: no fill launch
            return err.sum() / depth_mask.sum().clamp_min(1)   # 0 (not 0/0) if no ray is valid
        if depth_mask is not None:
            depth_pred, depth_gt = depth_pred[depth_mask], depth_gt[depth_mask]
        return self.depth_loss_dpt(depth_pred, depth_gt)

    def mean_on_mask(self, diff, valid_mask):
        """losses.py:79-87 without the data-dependent branch (0 when the mask is empty)."""
        mask = valid_mask.expand_as(diff)
        cnt = mask.sum()
        total = torch.where(mask, diff, 0.0).sum()        # scalar zeros: no fill launches
        return torch.where(cnt > 0, total / cnt.clamp_min(1), 0.0)

    def get_reprojection_loss(self, rgb, rgb_refs, valid_points, rgb_refs_ori):
        loss = 0
        for rgb_ref, rgb_ref_ori in zip(rgb_refs, rgb_refs_ori):
            diff = (rgb - rgb_ref).abs()
            if self.cfg["with_auto_mask"]:
                valid_points = (diff.mean(dim=-1, keepdim=True)
                                < (rgb - rgb_ref_ori).abs().mean(dim=-1, keepdim=True)).float() * valid_points
            loss = loss + self.mean_on_mask(diff, valid_points.bool())
        return loss / len(rgb_refs)

    def get_DPT_reprojection_loss(self, rgb, rgb_refs, valid_points, rgb_img_refs_ori):
        loss = 0
        for rgb_ref, rgb_ori in zip(rgb_refs, rgb_img_refs_ori):
            diff = (rgb - rgb_ref).abs().clamp(0, 1)
            if self.cfg["with_auto_mask"]:
                valid_points = (diff.mean(dim=1, keepdim=True)
                                < (rgb - rgb_ori).abs().mean(dim=1, keepdim=True)).float() * valid_points
            if self.cfg["with_ssim"]:
                diff = 0.15 * diff + 0.85 * compute_ssim_loss(rgb, rgb_ref)
            loss = loss + self.mean_on_mask(diff, valid_points.bool())
        return loss / len(rgb_refs)

    def get_weight_dist_loss(self, t_list):
        """losses.py:105-114: first / second differences of the camera path."""
        d = (t_list - t_list.roll(shifts=1, dims=0))[1:].norm(dim=1)
        dd = (d - d.roll(shifts=1))[1:]
        return d.mean(), dd.pow(2.0).mean()

    # ---- point clouds -------------------------------------------------------------
    def comp_closest_pts_idx_with_split(self, pts_src, pts_des):
        """losses.py:129-144 on the HIP nearest-neighbour kernel (no split needed)."""
        return nearest_index(pts_src, pts_des)

    def comp_point_point_error(self, Xt, Yt):
        """losses.py:145-150."""
        idx = self.comp_closest_pts_idx_with_split(Xt, Yt)
        return torch.linalg.norm(Xt - Yt[:, idx], dim=0).mean()

    def get_pc_loss(self, Xt, Yt):
        """losses.py:116-123 (dense matching)."""
        if self.cfg["match_method"] != "dense":
            raise NotImplementedError(self.cfg["match_method"])
        X, Y = Xt[0].permute(1, 0), Yt[0].permute(1, 0)
        return self.comp_point_point_error(X, Y) + self.comp_point_point_error(Y, X)

    def get_depth_consistency_loss(self, d1_proj, d2, d2_proj=None, d1=None):
        loss = (d1_proj - d2).abs().sum() / float(d1_proj.shape[1])
        if d2_proj is not None:
            loss = 0.5 * loss + 0.5 * (d2_proj - d1).abs().sum() / float(d2_proj.shape[1])
        return loss

    def get_rgb_s_loss(self, rgb1, rgb2, valid_points):
        """losses.py:152-159."""
        diff = (rgb1 - rgb2).abs().clamp(0, 1)
        if self.cfg["with_ssim"]:
            diff = 0.15 * diff + 0.85 * compute_ssim_loss(rgb1, rgb2)
        return self.mean_on_mask(diff, valid_points.bool())

    def get_t_cycle_loss(self, rt_pred, rt_gt):
        eye = torch.eye(4, device=rt_gt.device, dtype=rt_gt.dtype)
        return torch.norm(eye - inv(rt_gt) @ rt_pred)

    # ---- total ----------------------------------------------------------------------
    def forward(self, rgb_pred, rgb_gt, depth_pred=None, depth_gt=None, t_list=None, X=None, Y=None,
                rgb_pc1=None, rgb_pc1_proj=None, valid_points=None, d1_proj=None, d2=None, d2_proj=None,
                d1=None, weights={}, rgb_loss_type="l2", depth_mask=None, **kwargs):
        """losses.py:164-228: weighted sum + the same output dict."""
        dev = rgb_pred.device if rgb_pred is not None else (X.device if X is not None else "cpu")
        zero = _zero(dev)
        rgb_gt = rgb_gt.to(dev) if rgb_gt is not None else None
        w = weights
        fused = None
        use_depth = w["depth_weight"] != 0.0
        if (rgb_pred is not None and rgb_pred.is_cuda and (w["rgb_weight"] != 0.0 or use_depth)
                and (not use_depth or self.depth_loss_type == "l1")):
            # one launch for l_rgb, l_depth, l2_mean and their weighted sum; one for the backward
            fused = ray_loss(rgb_pred, rgb_gt, depth_pred if use_depth else None,
                             depth_gt if use_depth else None, depth_mask if use_depth else None,
                             rgb_loss_type == "l1", w["rgb_weight"], w["depth_weight"])
            l_rgb = fused[1] if w["rgb_weight"] != 0.0 else zero
            l_depth = fused[2] if use_depth else zero
        else:
            l_rgb = self.get_rgb_full_loss(rgb_pred, rgb_gt, rgb_loss_type) if w["rgb_weight"] != 0.0 else zero
            l_depth = self.get_depth_loss(depth_pred, depth_gt, depth_mask) if use_depth else zero
        if w["weight_dist_2nd_loss"] != 0.0 or w["weight_dist_1st_loss"] != 0.0:
            l_d1, l_d2 = self.get_weight_dist_loss(t_list)
        else:
            l_d1, l_d2 = zero, zero
        pair = kwargs.get("pair_losses")   # (loss_pc, loss_rgb_s) from the fused pair kernels
        if w["pc_weight"] != 0.0:
            l_pc = pair[0] if pair is not None else self.get_pc_loss(X, Y)
        else:
            l_pc = zero
        if w["rgb_s_weight"] != 0.0:
            l_rgbs = pair[1] if pair is not None else self.get_rgb_s_loss(rgb_pc1, rgb_pc1_proj, valid_points)
        else:
            l_rgbs = zero
        l_dc = (self.get_depth_consistency_loss(d1_proj, d2, d2_proj, d1)
                if w["depth_consistency_weight"] != 0.0 else zero)
        l_tc = self.get_t_cycle_loss(kwargs["rt_12"], kwargs["rt_12_gt"]) if w["t_cycle_weight"] != 0.0 else zero
        if fused is not None:
            l2_mean = fused[3]
        elif w["rgb_weight"] != 0.0 or w["depth_weight"] != 0.0:
            l2_mean = F.mse_loss(rgb_pred, rgb_gt)
        else:
            l2_mean = zero
        terms = [("weight_dist_1st_loss", l_d1), ("weight_dist_2nd_loss", l_d2), ("pc_weight", l_pc),
                 ("rgb_s_weight", l_rgbs), ("depth_consistency_weight", l_dc), ("t_cycle_weight", l_tc)]
        if fused is not None:
            loss = fused[0]
        else:
            terms = [("rgb_weight", l_rgb), ("depth_weight", l_depth)] + terms
            loss = zero
        for name, term in terms:        # zero-weight terms add nothing (and launch nothing)
            if w[name] != 0.0:
                loss = loss + w[name] * term
        # losses.py:213-214 drops into breakpoint() on NaN; that forces a host sync every
        # step and is left to the caller here.
        return {"loss": loss, "loss_rgb": l_rgb, "loss_depth": l_depth, "l2_mean": l2_mean,
                "loss_dist_1st": l_d1, "loss_dist_2nd": l_d2, "loss_pc": l_pc, "loss_rgb_s": l_rgbs,
                "loss_depth_consistency": l_dc, "loss_t_cycle": l_tc}

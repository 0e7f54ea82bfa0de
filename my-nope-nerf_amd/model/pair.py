"""Image-pair terms of the full NoPe-NeRF step on the HIP kernels of pair.hip (SURVEY.md
section 8(f) row 3): point clouds of both depth maps, relative pose, dense chamfer loss and
reprojection (rgb_s) loss in four launches forward and four backward, replacing the ~200
ATen launches of training.py:359-405 + losses.py:116-159.

``pair_losses`` keeps the reference inputs (depth maps at the pc resolution after the
``nearest_limit`` clamp, camera matrix, Rt_rel_12, scale1, the bilinearly resized images)
and is differentiable w.r.t. the depths (distortion learning), Rt_rel_12 (pose learning)
and scale1.  A learned camera matrix (focal learning) is not supported here; the Trainer
keeps the torch expressions for that case.
"""
from __future__ import annotations

import torch

from . import _hip


class _PairTerms(torch.autograd.Function):
    @staticmethod
    def forward(ctx, d1, d2, K, Rt, s1, img1, img2, h, w, nl, rgbs_detach_scale):
        ctx.set_materialize_grads(False)
        dev = d1.device
        P = h * w
        c = lambda t: None if t is None else t.detach().float().contiguous()
        d1c, d2c, Kc, Rtc, s1c = c(d1), c(d2), c(K), c(Rt), c(s1)
        i1, i2 = c(img1), c(img2)
        _, nfl = _hip.pair_workspace(P)
        work = torch.empty(nfl, device=dev, dtype=torch.float32)
        nn = torch.empty(2 * P, device=dev, dtype=torch.int32)
        out3 = torch.empty(3, device=dev, dtype=torch.float32)
        _hip.pair_forward(d1c, d2c, h, w, Kc, Rtc, s1c, nl, i1, i2, work, nn, out3)
        ctx.save_for_backward(d1c, d2c, Kc, Rtc, s1c, i1, i2, work, nn, out3)
        ctx.meta = (h, w, nl, int(rgbs_detach_scale), d1.shape, d2.shape, Rt.shape,
                    None if s1 is None else s1.shape)
        l_pc = out3[0].clone()
        l_rgbs = out3[1].clone()
        return l_pc, l_rgbs

    @staticmethod
    def backward(ctx, g_pc, g_rgbs):
        d1c, d2c, Kc, Rtc, s1c, i1, i2, work, nn, out3 = ctx.saved_tensors
        h, w, nl, det, sh1, sh2, shRt, shs = ctx.meta
        if g_pc is None and g_rgbs is None:
            return (None,) * 11
        dev = d1c.device
        P = h * w
        nb = (P + 255) // 256
        c = lambda g: None if g is None else g.detach().float().contiguous()
        gxy = torch.empty(12 * P, device=dev, dtype=torch.float32)   # 6 P int64 fixed-point sums (ABI 14)
        part = torch.empty(13 * nb, device=dev, dtype=torch.float32)
        g13 = torch.empty(13, device=dev, dtype=torch.float32)
        want = ctx.needs_input_grad
        g_d1 = torch.empty(P, device=dev, dtype=torch.float32) if want[0] else None
        g_d2 = torch.empty(P, device=dev, dtype=torch.float32) if want[1] else None
        _hip.pair_backward(d1c, d2c, h, w, Kc, Rtc, s1c, nl, i1 if g_rgbs is not None else None,
                           i2 if g_rgbs is not None else None, det, work, nn, out3, c(g_pc), c(g_rgbs), gxy,
                           g_d1, g_d2, g13, part)
        gRt = None
        if want[3]:
            gRt = torch.zeros(4, 4, device=dev, dtype=torch.float32)
            gRt[:3, :3] = g13[:9].view(3, 3)
            gRt[:3, 3] = g13[9:12]
            gRt = gRt.view(shRt)
        gs = g13[12:13].view(shs) if (want[4] and shs is not None) else None
        return (g_d1.view(sh1) if g_d1 is not None else None, g_d2.view(sh2) if g_d2 is not None else None,
                None, gRt, gs, None, None, None, None, None, None)


def pair_losses(d1, d2, camera_mat, Rt_rel, scale1, img1, img2, res, nl, rgbs_detach_scale=False):
    """(loss_pc, loss_rgb_s) of the image pair.  d1, d2: [1,1,h,w] depths at res (clamped);
    img1, img2: [1,3,h,w] or None (no rgb_s term, returned as 0)."""
    h, w = res
    if camera_mat.requires_grad:
        raise ValueError("pair_losses: a learned camera matrix is not supported")
    return _PairTerms.apply(d1.reshape(-1), d2.reshape(-1), camera_mat.reshape(4, 4), Rt_rel.reshape(4, 4),
                            None if scale1 is None else scale1.reshape(1), img1, img2, int(h), int(w), float(nl),
                            bool(rgbs_detach_scale))

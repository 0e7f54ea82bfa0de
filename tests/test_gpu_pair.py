"""Fused image-pair kernels (pair.hip) against the oracle's restatement of
training.py:359-405 and losses.py:116-159 (GPU only).  Values at 1e-5 relative; gradients
w.r.t. both depth maps, Rt_rel_12 and the point-cloud scale at 1e-3 relative to each
tensor's largest entry (fp32 HIP vs fp64 oracle autograd through the same nearest
neighbours)."""
import pytest
import torch
import torch.nn.functional as F

from model.pair import pair_losses
from oracle import nerf_oracle as orc
from tests.helpers import camera_K

pytestmark = pytest.mark.gpu


def _oracle(d1, d2, K, Rt, s1, img1, img2, res, nl):
    """training.py:359-393 + losses.py:116-159 (with_ssim False), float64."""
    p_pc = orc.arange_pixels(res[0], res[1], dtype=d1.dtype)[1]
    pc1 = orc.transform_to_world(p_pc, d1.reshape(1, -1, 1), K)
    pc2 = orc.transform_to_world(p_pc, d2.reshape(1, -1, 1), K)
    R, t = Rt[:, :3, :3], Rt[:, :3, 3]
    out = {}
    if img1 is not None:
        rgb1 = orc.grid_values(img1, p_pc)
        q = pc1 @ R.transpose(1, 2) + t
        bad = (-q[:, :, 2:] < nl).expand_as(q)
        q = torch.where(bad, torch.full_like(q, nl), q)
        p_re, valid = orc.project_to_cam(q, K)
        rgb2 = orc.grid_values(img2, p_re)
        out["rgb_s"] = orc.rgb_s_loss_ref(rgb1.view(1, res[0], res[1], 3), rgb2.view(1, res[0], res[1], 3),
                                          valid.view(1, res[0], res[1], 1))
        out["n_valid"] = int(valid.sum())
    if s1 is not None:
        pc1, pc2 = pc1 / s1, pc2 / s1
    out["pc"] = orc.pc_loss(pc1 @ R.transpose(1, 2) + t, pc2)
    return out


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("res,with_rgbs,with_scale", [((12, 17), True, True), ((47, 155), True, True),
                                                      ((20, 30), False, False)])
def test_pair_losses_match_oracle(dev, res, with_rgbs, with_scale):
    g = torch.Generator().manual_seed(res[0])
    h, w = res
    K = camera_K(4 * h, 4 * w, 3.0 * w, 3.0 * w)
    d1 = 2.0 + 3.0 * torch.rand(1, 1, h, w, generator=g)
    d2 = 2.0 + 3.0 * torch.rand(1, 1, h, w, generator=g)
    d1[0, 0, 0, :3] = 0.01                                   # the nearest_limit floor
    th = 0.05
    Rt = torch.eye(4).unsqueeze(0)
    Rt[0, :3, :3] = torch.tensor([[1.0, 0, 0], [0, torch.cos(torch.tensor(th)), -torch.sin(torch.tensor(th))],
                                  [0, torch.sin(torch.tensor(th)), torch.cos(torch.tensor(th))]])
    Rt[0, :3, 3] = torch.tensor([0.05, -0.02, 0.1])
    Rt[0, 2, 3] = 0.3                                        # pushes some points behind the camera (-z < nl)
    s1 = torch.tensor([1.3]) if with_scale else None
    img1 = torch.rand(1, 3, h, w, generator=g) if with_rgbs else None
    img2 = torch.rand(1, 3, h, w, generator=g) if with_rgbs else None
    nl = 0.01

    # oracle, float64 with autograd
    o = [x.double().clone().requires_grad_(True) if x is not None else None for x in (d1, d2, Rt, s1)]
    ref = _oracle(o[0], o[1], K.double(), o[2], o[3], None if img1 is None else img1.double(),
                  None if img2 is None else img2.double(), res, nl)
    tot = ref["pc"] + (0.7 * ref["rgb_s"] if with_rgbs else 0.0)
    tot.backward()

    hd = [x.to(dev).requires_grad_(True) if x is not None else None for x in (d1, d2, Rt, s1)]
    l_pc, l_rgbs = pair_losses(hd[0], hd[1], K.to(dev), hd[2], hd[3], None if img1 is None else img1.to(dev),
                               None if img2 is None else img2.to(dev), res, nl)
    assert abs(l_pc.item() - ref["pc"].item()) <= 1e-5 * abs(ref["pc"].item())
    if with_rgbs:
        assert ref["n_valid"] > 0 and ref["n_valid"] < h * w      # both valid and invalid projections
        assert abs(l_rgbs.item() - ref["rgb_s"].item()) <= 1e-5 * abs(ref["rgb_s"].item()) + 1e-7
        (l_pc + 0.7 * l_rgbs).backward()
    else:
        assert l_rgbs.item() == 0.0
        l_pc.backward()
    assert _rel(hd[0].grad, o[0].grad) < 1e-3
    assert _rel(hd[1].grad, o[1].grad) < 1e-3
    assert _rel(hd[2].grad[0, :3], o[2].grad[0, :3]) < 1e-3
    assert hd[2].grad[0, 3].abs().max().item() == 0
    if with_scale:
        assert _rel(hd[3].grad, o[3].grad) < 1e-3

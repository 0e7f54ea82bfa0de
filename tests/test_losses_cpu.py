"""The auxiliary loss terms (losses.py:35-58, 105-114, 124-128, 161-162, 232-263): oracle
known-answer tests, and the drop-in Loss methods against the oracle on CPU tensors (these
terms are small torch expressions in both; the GPU tests run them inside Trainer).

Parity unpinned upstream: the reference ships no fixtures for these terms; the KATs below
are closed forms of the reference's formulas."""
import math

import pytest
import torch

from model.losses import Loss
from oracle import nerf_oracle as orc
from tests.helpers import make_cfg


def _loss(**over):
    t = dict(make_cfg()["training"])
    t.update(over)
    return Loss(t)


def _rigid(seed, scale=0.3):
    from tests.helpers import rigid_c2w
    return rigid_c2w(seed, scale).double()


# ---- t-cycle (losses.py:161-162) --------------------------------------------------
def test_t_cycle_kat():
    gt = _rigid(1).unsqueeze(0)
    assert orc.t_cycle_loss(gt, gt).item() == pytest.approx(0.0, abs=1e-6)
    # a pure translation error d: I - gt^-1 (gt + [0 | d]) = -[0 | R^T d] -> |d|
    pred = gt.clone()
    pred[0, :3, 3] += torch.tensor([0.3, -0.4, 0.0], dtype=torch.float64)
    assert orc.t_cycle_loss(pred, gt).item() == pytest.approx(0.5, rel=1e-6)
    # a rotation error by theta about any axis: |I - R_theta|_F = 2 sqrt(2) sin(theta / 2)
    th = 0.2
    Rz = torch.eye(4, dtype=torch.float64)
    Rz[:2, :2] = torch.tensor([[math.cos(th), -math.sin(th)], [math.sin(th), math.cos(th)]])
    assert orc.t_cycle_loss(gt @ Rz, gt).item() == pytest.approx(2 * math.sqrt(2) * math.sin(th / 2), rel=1e-6)


def test_t_cycle_dropin_matches_oracle():
    a, b = _rigid(2).unsqueeze(0).float(), _rigid(3).unsqueeze(0).float()
    assert _loss().get_t_cycle_loss(a, b).item() == pytest.approx(orc.t_cycle_loss(a, b).item(), rel=1e-6)


# ---- invariant depth (losses.py:35-58) --------------------------------------------
def test_depth_invariant_kat():
    g = torch.Generator().manual_seed(0)
    d = 1 + 5 * torch.rand(101, generator=g, dtype=torch.float64)
    # median / MAD normalisation: invariant to positive scale and shift
    assert orc.depth_invariant_loss(3.0 * d + 2.0, d).item() == pytest.approx(0.0, abs=1e-24)
    # even count: torch.median is the lower middle value
    e = torch.tensor([1.0, 2.0, 3.0, 10.0], dtype=torch.float64)
    t, s = 2.0, (1 + 0 + 1 + 8) / 4
    n = (e - t) / s
    assert orc.depth_invariant_loss(e, torch.zeros(4, dtype=torch.float64) + torch.arange(4.0)).item() == \
        pytest.approx(((n - (torch.arange(4.0) - 1) / 1.0) ** 2).mean().item())
    w = torch.tensor([1.0, 0.0, 1.0, 0.0], dtype=torch.float64)
    full = (n - (torch.arange(4.0) - 1)) ** 2
    assert orc.depth_invariant_loss(e, torch.arange(4.0, dtype=torch.float64), w).item() == \
        pytest.approx(((full * w).sum() / (w.sum() + 1e-8)).item())


def test_depth_invariant_dropin_matches_oracle():
    g = torch.Generator().manual_seed(1)
    p, q = 1 + 4 * torch.rand(64, generator=g), 1 + 4 * torch.rand(64, generator=g)
    L = _loss(depth_loss_type="invariant")
    assert L.get_depth_loss(p, q).item() == pytest.approx(orc.depth_invariant_loss(p, q).item(), rel=1e-6)
    # the dense (mask) form the trainer uses equals the reference's masked vectors
    m = torch.rand(64, generator=g) > 0.3
    assert L.get_depth_loss(p, q, m).item() == pytest.approx(orc.depth_invariant_loss(p[m], q[m]).item(), rel=1e-6)


# ---- camera-path regularisers (losses.py:105-114) ---------------------------------
def test_weight_dist_kat():
    # constant-speed straight path: first differences all |v|, second differences 0
    v = torch.tensor([0.3, 0.0, 0.4], dtype=torch.float64)
    t = torch.arange(5, dtype=torch.float64)[:, None] * v
    d1, d2 = orc.weight_dist_loss(t)
    assert d1.item() == pytest.approx(0.5) and d2.item() == pytest.approx(0.0, abs=1e-24)
    t = torch.tensor([[0.0, 0, 0], [1, 0, 0], [3, 0, 0]], dtype=torch.float64)     # steps 1, 2
    d1, d2 = orc.weight_dist_loss(t)
    assert d1.item() == pytest.approx(1.5) and d2.item() == pytest.approx(1.0)


def test_weight_dist_dropin_matches_oracle():
    t = torch.randn(7, 3, generator=torch.Generator().manual_seed(2))
    a = _loss().get_weight_dist_loss(t)
    b = orc.weight_dist_loss(t)
    assert all(x.item() == pytest.approx(y.item(), rel=1e-6) for x, y in zip(a, b))


# ---- depth consistency (losses.py:124-128) -----------------------------------------
def test_depth_consistency_kat_and_dropin():
    a = torch.tensor([[1.0, 2.0, 3.0]])
    b = torch.tensor([[1.5, 2.0, 1.0]])
    assert orc.depth_consistency_loss(a, b).item() == pytest.approx((0.5 + 0 + 2) / 3)
    assert orc.depth_consistency_loss(a, b, b, a).item() == pytest.approx((0.5 + 0 + 2) / 3)
    assert _loss().get_depth_consistency_loss(a, b, b, a).item() == pytest.approx(
        orc.depth_consistency_loss(a, b, b, a).item())


# ---- SSIM (losses.py:232-263) -------------------------------------------------------
def test_ssim_kat_and_dropin():
    from model.losses import SSIM
    g = torch.Generator().manual_seed(3)
    x = torch.rand(1, 5, 7, 3, generator=g)                  # (B,H,W,3), as get_rgb_s_loss passes it
    assert orc.ssim_map(x, x).abs().max().item() == pytest.approx(0.0, abs=1e-6)
    # constant images a, b: mu = a, b; sigma = 0 -> 1 - (2ab + C1) / (a^2 + b^2 + C1), halved
    a, b = torch.full((1, 1, 4, 4), 0.2), torch.full((1, 1, 4, 4), 0.6)
    C1 = 0.01 ** 2
    want = (1 - (2 * 0.2 * 0.6 + C1) / (0.04 + 0.36 + C1)) / 2
    assert torch.allclose(orc.ssim_map(a, b), torch.full((1, 1, 4, 4), want), atol=2e-5)
    y = torch.rand(1, 5, 7, 3, generator=g)
    assert torch.allclose(SSIM()(x, y), orc.ssim_map(x, y), atol=1e-7)


def test_rgb_s_loss_with_ssim_dropin_matches_oracle():
    g = torch.Generator().manual_seed(4)
    r1, r2 = torch.rand(1, 6, 9, 3, generator=g), torch.rand(1, 6, 9, 3, generator=g)
    valid = torch.rand(1, 6, 9, 1, generator=g) > 0.2
    L = _loss(with_ssim=True)
    assert L.get_rgb_s_loss(r1, r2, valid).item() == pytest.approx(
        orc.rgb_s_loss_ref(r1, r2, valid, with_ssim=True).item(), rel=1e-6)


# ---- the weighted sum (losses.py:164-228) -----------------------------------------
def test_loss_forward_all_terms_matches_oracle():
    g = torch.Generator().manual_seed(5)
    R = 32
    rgb, gt = torch.rand(1, R, 3, generator=g), torch.rand(1, R, 3, generator=g)
    dp, dg = 1 + torch.rand(R, generator=g), 1 + torch.rand(R, generator=g)
    t_list = torch.randn(4, 3, generator=g)
    rt, rt_gt = _rigid(6).float().unsqueeze(0), _rigid(7).float().unsqueeze(0)
    w = {"rgb_weight": 1.0, "depth_weight": 0.04, "pc_weight": 0.0, "rgb_s_weight": 0.0,
         "depth_consistency_weight": 0.0, "weight_dist_2nd_loss": 0.3, "weight_dist_1st_loss": 0.2,
         "t_cycle_weight": 1.0}
    for dtype in ("l1", "invariant"):
        L = _loss(depth_loss_type=dtype)
        a = L(rgb, gt, dp, dg, t_list=t_list, weights=w, rgb_loss_type="l2", rt_12=rt, rt_12_gt=rt_gt)
        b = orc.total_loss(rgb, gt, dp, dg, w, "l2", t_list=t_list, t_cycle=orc.t_cycle_loss(rt, rt_gt),
                           depth_loss_type=dtype)
        for k in b:
            assert a[k].item() == pytest.approx(b[k].item(), rel=1e-6, abs=1e-7), (dtype, k)

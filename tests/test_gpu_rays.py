"""Ray prologue / loss epilogue kernels (rays.hip) against the oracle and torch autograd
(GPU only).  Tolerances: 1e-5 relative for the 4x4 chains and ray geometry (fp32 with a
different but equally stable elimination order), bit-exact for the sampler's gathers."""
import math

import pytest
import torch

from model import _hip, rays
from model.losses import Loss
from oracle import nerf_oracle as orc
from tests.helpers import make_cfg, rigid_c2w, synthetic_rays

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


# ------------------------------------------------------------------ sampler
@pytest.mark.parametrize("H,W,R", [(188, 621, 1024), (40, 50, 1000), (96, 96, 4096), (3, 5, 1), (10, 10, 50)])
def test_sample_rays_distinct_gathers(dev, H, W, R):
    img = torch.rand(3, H, W, device=dev)
    idx, pix, rgb = rays.sample_rays(H * W, R, W, H, img, seed=1234)
    idx_c = idx.cpu()
    assert idx_c.shape == (R,) and idx_c.dtype == torch.int64
    assert idx_c.min() >= 0 and idx_c.max() < H * W
    assert idx_c.unique().numel() == R                        # without replacement
    ref_pix = orc.arange_pixels(H, W)[1][:, idx_c]
    assert torch.equal(pix.cpu(), ref_pix)                    # bit-exact arange_pixels
    assert torch.equal(rgb.cpu(), img.cpu().view(1, 3, H * W).permute(0, 2, 1)[:, idx_c])
    idx2, _, _ = rays.sample_rays(H * W, R, W, H, img, seed=1234)
    assert torch.equal(idx2.cpu(), idx_c)                     # deterministic in the seed
    if R > 1:
        idx3, _, _ = rays.sample_rays(H * W, R, W, H, img, seed=1235)
        assert not torch.equal(idx3.cpu(), idx_c)


def test_sample_rays_uniform(dev):
    """Each pixel's inclusion frequency over many draws is R/n (binomial, 6 sigma), and
    every ray slot's marginal is uniform too (no slot prefers low indices)."""
    n, R, draws = 1000, 400, 400
    counts = torch.zeros(n, dtype=torch.float64)
    first = torch.zeros(10, dtype=torch.float64)
    for s in range(draws):
        c = _sample_idx(n, R, 10 ** 6 + s, dev).cpu()
        counts += torch.bincount(c, minlength=n).double()
        first += torch.bincount(c[:50] // 100, minlength=10).double()
    p = R / n
    sd = math.sqrt(draws * p * (1 - p))
    assert (counts - draws * p).abs().max().item() < 6 * sd
    exp_first = draws * 50 / 10
    assert (first - exp_first).abs().max().item() < 6 * math.sqrt(exp_first)


def _sample_idx(n, R, seed, dev):
    idx = torch.empty(R, device=dev, dtype=torch.int64)
    status = torch.zeros(1, device=dev, dtype=torch.int32)
    _hip.sample_rays(n, R, seed, 0, 0, None, idx, None, None, status)
    assert status.item() >= 1
    return idx


def test_sample_rays_half_density(dev):
    """n = 2R (the densest allowed draw) still converges and stays distinct."""
    idx = _sample_idx(8192, 4096, 7, dev)
    assert idx.cpu().unique().numel() == 4096


# ------------------------------------------------------------------ 4x4 chains
def test_inverse_matches_torch_and_grad(dev):
    g = torch.Generator().manual_seed(0)
    A = torch.randn(37, 4, 4, generator=g, dtype=torch.float64) + 3 * torch.eye(4, dtype=torch.float64)
    A[5] = rigid_c2w(3).double()
    A[6, 0, 0] = 0.0                                           # forces a pivot swap
    ref = torch.linalg.inv(A)
    out = rays.inv(A.float().to(dev))
    assert _rel(out, ref) < 1e-5
    Ad = A.float().to(dev).requires_grad_(True)
    gy = torch.randn(37, 4, 4, generator=g)
    rays.inv(Ad).backward(gy.to(dev))
    A64 = A.clone().requires_grad_(True)
    torch.linalg.inv(A64).backward(gy.double())
    assert _rel(Ad.grad, A64.grad) < 1e-4


def test_pose_c2w_matches_oracle_and_grad(dev):
    g = torch.Generator().manual_seed(1)
    init = rigid_c2w(5)
    for r0 in (torch.zeros(3), 1e-3 * torch.randn(3, generator=g), 0.7 * torch.randn(3, generator=g)):
        t0 = torch.randn(3, generator=g)
        ref = orc.make_c2w(r0.double(), t0.double()) @ init.double()
        r = r0.to(dev).requires_grad_(True)
        t = t0.to(dev).requires_grad_(True)
        out = rays.pose_c2w(r, t, init.to(dev))
        assert _rel(out, ref) < 1e-5
        gy = torch.randn(4, 4, generator=g)
        out.backward(gy.to(dev))
        r64 = r0.double().clone().requires_grad_(True)
        t64 = t0.double().clone().requires_grad_(True)
        (orc.make_c2w(r64, t64) @ init.double()).backward(gy.double())
        assert _rel(t.grad, t64.grad) < 1e-5
        if r0.norm() > 0:          # at r = 0 the reference's own gradient is 0/0 territory
            assert _rel(r.grad, r64.grad) < 1e-4


def test_pose_c2w_grad_at_zero_rotation(dev):
    """r = 0 (LearnPose's initial value): the closed-form backward equals torch autograd of the
    reference expression in fp32 (the |r| subgradient is 0, the [r]x terms carry the gradient)."""
    g = torch.Generator().manual_seed(2)
    init = rigid_c2w(4)
    gy = torch.randn(4, 4, generator=g)
    r = torch.zeros(3, device=dev, requires_grad=True)
    t = torch.randn(3, generator=g).to(dev).requires_grad_(True)
    rays.pose_c2w(r, t, init.to(dev)).backward(gy.to(dev))
    rc = torch.zeros(3, requires_grad=True)
    tc = t.detach().cpu().clone().requires_grad_(True)
    rays._pose_torch(rc, tc, init).backward(gy)
    assert torch.isfinite(r.grad).all()
    assert _rel(r.grad, rc.grad) < 1e-5 and _rel(t.grad, tc.grad) < 1e-6


def test_mat4_mul_and_grad(dev):
    g = torch.Generator().manual_seed(5)
    A = torch.randn(1, 4, 4, generator=g, dtype=torch.float64)
    B = torch.randn(1, 4, 4, generator=g, dtype=torch.float64)
    gy = torch.randn(1, 4, 4, generator=g, dtype=torch.float64)
    a = A.float().to(dev).requires_grad_(True)
    b = B.float().to(dev).requires_grad_(True)
    c = rays.mat4_mul(a, b)
    assert _rel(c, A @ B) < 1e-6
    c.backward(gy.float().to(dev))
    a64, b64 = A.clone().requires_grad_(True), B.clone().requires_grad_(True)
    (a64 @ b64).backward(gy)
    assert _rel(a.grad, a64.grad) < 1e-5 and _rel(b.grad, b64.grad) < 1e-5


def test_unproject_matrix_grad_all_inputs(dev):
    """Gradients of inv(S) inv(W) inv(K) w.r.t. all three matrices (focal, pose and scale
    learning) against fp64 autograd."""
    b = synthetic_rays(R=8, seed=6)
    K, w2c, S = b["K"].double(), b["w2c"].double(), b["scale"].double().clone()
    S[0, :3, :3] *= 1.3
    gy = torch.randn(1, 4, 4, generator=torch.Generator().manual_seed(7), dtype=torch.float64)
    ins64 = [x.clone().requires_grad_(True) for x in (K, w2c, S)]
    iv = torch.linalg.inv
    ((iv(ins64[2]) @ iv(ins64[1])) @ iv(ins64[0])).backward(gy)
    ins = [x.float().to(dev).requires_grad_(True) for x in (K, w2c, S)]
    M = rays.unproject_matrix(*ins)
    assert _rel(M, (iv(S) @ iv(w2c)) @ iv(K)) < 1e-5
    M.backward(gy.float().to(dev))
    for h, r in zip(ins, ins64):
        assert _rel(h.grad, r.grad) < 1e-4


@pytest.mark.parametrize("shift_first,lo", [(False, float("-inf")), (True, float("-inf")), (False, 0.5),
                                            (True, 0.5)])
def test_depth_affine_matches_torch(dev, shift_first, lo):
    """rays.depth_affine (distortion + nearest_limit clamp, one launch each way) vs the torch
    expressions of training.py:259-264 / 346-347 and their autograd, incl. clamped entries."""
    g = torch.Generator().manual_seed(8)
    d = torch.rand(1, 1, 47, 155, generator=g) * 8
    d[0, 0, :3, :5] = 0.0                                    # below the clamp after the affine
    gy = torch.randn(1, 1, 47, 155, generator=g)
    s0, t0 = torch.tensor([1.3]), torch.tensor([-0.2])
    pre = (d + t0) * s0 if shift_first else d * s0 + t0
    ref = pre.clamp_min(lo) if lo != float("-inf") else pre
    sd, td = s0.to(dev).requires_grad_(True), t0.to(dev).requires_grad_(True)
    y = rays.depth_affine(d.to(dev), sd, td, shift_first, lo)
    assert torch.equal(y.cpu(), ref)                         # same fp32 expression, bit-exact
    y.backward(gy.to(dev))
    # gradients: fp64 sums over the unclamped entries; the bar is relative to sum |term|
    # (g sums over ~7 000 entries cancel, so fp32 order differences show against the result)
    keep = (pre >= lo).double()                              # torch's clamp_min passes x >= lo
    g64 = gy.double() * keep
    ts = g64 * ((d.double() + t0.double()) if shift_first else d.double())
    tt = g64 * (s0.double() if shift_first else 1.0)
    for h, terms in ((sd.grad, ts), (td.grad, tt)):
        assert abs(h.item() - terms.sum().item()) <= 1e-6 * terms.abs().sum().item()


def test_learnpose_forward_device(dev):
    import model as mdl
    init = torch.stack([rigid_c2w(1), rigid_c2w(2)])
    lp = mdl.LearnPose(2, True, True, None, init_c2w=init)
    with torch.no_grad():
        lp.r.copy_(0.01 * torch.arange(6.0).view(2, 3))
        lp.t.copy_(0.1 * torch.arange(6.0).view(2, 3))
    ref = orc.learn_pose_forward(lp.r.detach().double(), lp.t.detach().double(), init.double(), 1)
    lp = lp.to(dev)
    out = lp(1)
    assert _rel(out, ref) < 1e-5
    out.sum().backward()
    assert lp.r.grad is not None and lp.r.grad[0].abs().sum().item() == 0.0
    assert lp.r.grad[1].abs().sum().item() > 0 and lp.t.grad[1].abs().sum().item() > 0


# ------------------------------------------------------------------ camera rays
@pytest.mark.parametrize("normalise", [True, False])
def test_camera_rays_match_oracle(dev, normalise):
    b = synthetic_rays(R=1024, seed=3)
    K, w2c, S = b["K"], b["w2c"], b["scale"].clone()
    S[0, :3, :3] *= 1.7                                        # non-trivial scale matrix
    cam_r, ray_r, ds_r, rn_r, m_r = orc.rays_from_cameras(b["pixels"].double(), b["depth"].double(), K.double(),
                                                          w2c.double(), S.double(), normalise)
    M = rays.unproject_matrix(K.to(dev), w2c.to(dev), S.to(dev))
    cam, ray, view, rn, ds, m = rays.camera_rays_hip(M, b["pixels"].to(dev), b["depth"].to(dev), normalise)
    assert _rel(cam, cam_r) < 1e-5 and _rel(ray, ray_r) < 1e-5 and _rel(rn, rn_r) < 1e-5
    assert _rel(ds, ds_r) < 1e-5
    assert torch.equal(m.cpu(), m_r)
    assert torch.equal(view.cpu(), -ray.cpu())
    _, _, view1, _, ds1, _ = rays.camera_rays_hip(M, b["pixels"].to(dev), None, normalise, view_ones=True)
    assert bool((view1 == 1).all()) and (bool((ds1 == 1).all()) if normalise else True)


@pytest.mark.parametrize("normalise", [True, False])
def test_camera_rays_backward(dev, normalise):
    """Gradients w.r.t. the world matrix (pose learning) and the depth prior (distortion
    learning) equal torch autograd through the oracle's unprojection in fp64."""
    b = synthetic_rays(R=700, seed=4)
    K, w2c, S = b["K"], b["w2c"], b["scale"]
    g = torch.Generator().manual_seed(9)
    gc, gr, gv, gn, gd = (torch.randn(700, 3, generator=g), torch.randn(700, 3, generator=g),
                          torch.randn(700, 3, generator=g), torch.randn(700, generator=g),
                          torch.randn(700, generator=g))
    w64 = w2c.double().clone().requires_grad_(True)
    d64 = b["depth"].double().clone().requires_grad_(True)
    cam_r, ray_r, ds_r, rn_r, _ = orc.rays_from_cameras(b["pixels"].double(), d64, K.double(), w64, S.double(),
                                                        normalise)
    loss = ((cam_r * gc.double()).sum() + (ray_r * gr.double()).sum() + (-ray_r * gv.double()).sum()
            + (rn_r * gn.double()).sum() + (ds_r * gd.double()).sum())
    loss.backward()
    wd = w2c.to(dev).requires_grad_(True)
    dd = b["depth"].to(dev).requires_grad_(True)
    M = rays.unproject_matrix(K.to(dev), wd, S.to(dev))
    cam, ray, view, rn, ds, _ = rays.camera_rays_hip(M, b["pixels"].to(dev), dd, normalise)
    lh = ((cam * gc.to(dev)).sum() + (ray * gr.to(dev)).sum() + (view * gv.to(dev)).sum()
          + (rn * gn.to(dev)).sum() + (ds * gd.to(dev)).sum())
    lh.backward()
    assert _rel(wd.grad, w64.grad) < 1e-4
    assert _rel(dd.grad, d64.grad) < 1e-4


# ------------------------------------------------------------------ loss
@pytest.mark.parametrize("kind", ["l2", "l1"])
@pytest.mark.parametrize("mask_kind", ["some", "none_valid", "no_mask"])
def test_ray_loss_matches_torch(dev, kind, mask_kind):
    g = torch.Generator().manual_seed(2)
    R = 1024
    rgb = torch.rand(1, R, 3, generator=g)
    gt = torch.rand(1, R, 3, generator=g)
    dp = 5 * torch.rand(R, generator=g)
    dg = 5 * torch.rand(R, generator=g)
    mask = {"some": torch.rand(R, generator=g) > 0.1, "none_valid": torch.zeros(R, dtype=torch.bool),
            "no_mask": None}[mask_kind]
    cfg = make_cfg()["training"]
    weights = {"rgb_weight": 1.0, "depth_weight": 0.04, "pc_weight": 0.0, "rgb_s_weight": 0.0,
               "depth_consistency_weight": 0.0, "weight_dist_2nd_loss": 0.0, "weight_dist_1st_loss": 0.0,
               "t_cycle_weight": 0.0}
    lf = Loss(cfg)
    # reference (host tensors take the unfused torch expressions)
    r_c = rgb.clone().requires_grad_(True)
    dp_c = dp.clone().requires_grad_(True)
    dg_c = dg.clone().requires_grad_(True)
    ref = lf(r_c, gt, dp_c, dg_c, weights=weights, rgb_loss_type=kind, depth_mask=mask)
    (ref["loss"] + 0.3 * ref["l2_mean"]).backward()
    r_d = rgb.to(dev).requires_grad_(True)
    dp_d = dp.to(dev).requires_grad_(True)
    dg_d = dg.to(dev).requires_grad_(True)
    out = lf(r_d, gt.to(dev), dp_d, dg_d, weights=weights, rgb_loss_type=kind,
             depth_mask=None if mask is None else mask.to(dev))
    (out["loss"] + 0.3 * out["l2_mean"]).backward()
    for k in ("loss", "loss_rgb", "loss_depth", "l2_mean"):
        assert math.isclose(out[k].item(), ref[k].item(), rel_tol=1e-5, abs_tol=1e-7), (k, out[k], ref[k])
    assert _rel(r_d.grad, r_c.grad) < 1e-5
    assert _rel(dp_d.grad, dp_c.grad) < 1e-5 if mask_kind != "none_valid" else dp_d.grad.abs().max() == 0
    assert _rel(dg_d.grad, dg_c.grad) < 1e-5 if mask_kind != "none_valid" else dg_d.grad.abs().max() == 0


def test_sample_rays_device_counter(dev):
    """seed_counter: each launch advances the device counter by one and keys the draw on
    it, so identical launches (a replayed hipGraph) draw different, still distinct, sets."""
    H, W, R = 40, 50, 512
    img = torch.rand(3, H, W, device=dev)
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    draws = [rays.sample_rays(H * W, R, W, H, img, seed=99, seed_counter=ctr)[0].cpu() for _ in range(3)]
    assert ctr.item() == 3
    for d in draws:
        assert d.unique().numel() == R
    assert not torch.equal(draws[0], draws[1]) and not torch.equal(draws[1], draws[2])
    ctr.zero_()
    again = rays.sample_rays(H * W, R, W, H, img, seed=99, seed_counter=ctr)[0].cpu()
    assert torch.equal(again, draws[0])                       # deterministic in (seed, counter)

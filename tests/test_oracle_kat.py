"""Analytic known-answer tests pinning the oracle to the reference text (CPU)."""
import math

import pytest
import torch
import torch.nn.functional as F

from oracle import nerf_oracle as orc


def test_encoding_channel_order():
    """official_nerf.py:112-118: [x, sin(2^0 x), cos(2^0 x), sin(2^1 x), ...] per 3-vector."""
    x = torch.tensor([[0.1, -0.2, 0.3]], dtype=torch.float64)
    e = orc.encode_position(x, 2)
    want = torch.cat([x, torch.sin(x), torch.cos(x), torch.sin(2 * x), torch.cos(2 * x)], -1)
    assert e.shape == (1, 15) and torch.equal(e, want)
    assert orc.encode_position(torch.zeros(5, 3), 10).shape == (5, 63)
    assert orc.encode_position(torch.zeros(5, 3), 4).shape == (5, 27)


def test_init_bias_overrides():
    """official_nerf.py:39-44."""
    m = orc.OracleNerf(hidden_dim=64)
    assert m.fc_density.bias.item() == pytest.approx(0.1)
    assert torch.allclose(m.fc_rgb.bias, torch.full((3,), 0.02))
    assert torch.allclose(orc.OracleNerf(hidden_dim=64, white_background=True).fc_rgb.bias, torch.full((3,), 0.8))
    assert sum(p.numel() for p in orc.OracleNerf(256).parameters()) == 595844
    assert sum(p.numel() for p in orc.OracleNerf(64).parameters()) == 44516


def test_softplus_threshold():
    """F.softplus(beta=1, threshold=20): identity above 20 (official_nerf.py:78)."""
    x = torch.tensor([19.0, 20.0, 20.5, 30.0, -5.0], dtype=torch.float64)
    y = F.softplus(x)
    assert y[2] == 20.5 and y[3] == 30.0
    assert y[0] == pytest.approx(math.log1p(math.exp(19.0)))


def test_composite_constant_alpha_closed_form():
    """w_i = a (1 - a + eps)^i for constant alpha (rendering.py:124)."""
    R, S, a = 2, 16, 0.3
    alpha = torch.full((R, S), a, dtype=torch.float64)
    rgb = torch.rand(R, S, 3, dtype=torch.float64)
    z = torch.linspace(1, 2, S, dtype=torch.float64).repeat(R, 1)
    out, dist, _, w = orc.composite(alpha, rgb, z)
    f = 1 - a + orc.EPS_COMPOSITE
    want_w = a * f ** torch.arange(S, dtype=torch.float64)
    assert torch.allclose(w[0], want_w, rtol=0, atol=1e-15)
    assert torch.allclose(out, (want_w[None, :, None] * rgb).sum(1), atol=1e-14)
    assert torch.allclose(dist, (want_w * z[0]).sum().expand(R), atol=1e-13)


def test_composite_zero_alpha_gives_zero():
    alpha = torch.zeros(3, 8)
    rgb = torch.rand(3, 8, 3)
    z = torch.rand(3, 8)
    out, dist, _, w = orc.composite(alpha, rgb, z)
    assert out.abs().max() == 0 and dist.abs().max() == 0
    out_w, _, _, _ = orc.composite(alpha, rgb, z, white_background=True)
    assert torch.allclose(out_w, torch.ones(3, 3))        # rendering.py:139-141


def test_composite_dist_alpha_last_sample_opaque():
    """dist_alpha: delta_last = 1e10 and alpha_last forced to 1 (rendering.py:116-122)."""
    sigma = torch.zeros(2, 5)
    z = torch.linspace(0, 1, 5).repeat(2, 1)
    rgb = torch.rand(2, 5, 3)
    out, dist, alpha, w = orc.composite(sigma, rgb, z, dist_alpha=True)
    assert torch.equal(alpha[:, -1], torch.ones(2))
    assert torch.allclose(out, rgb[:, -1] * (1 + orc.EPS_COMPOSITE) ** 4)


def test_exp_rotation():
    """common.py:290-299."""
    I = orc.Exp(torch.zeros(3))
    assert torch.allclose(I, torch.eye(3))
    Rz = orc.Exp(torch.tensor([0.0, 0.0, math.pi / 2], dtype=torch.float64))
    want = torch.tensor([[0.0, -1.0, 0.0], [1.0, 0.0, 0.0], [0.0, 0.0, 1.0]], dtype=torch.float64)
    assert torch.allclose(Rz, want, atol=1e-12)
    r = torch.tensor([0.3, -0.2, 0.5], dtype=torch.float64)
    Rm = orc.Exp(r)
    assert torch.allclose(Rm @ Rm.t(), torch.eye(3, dtype=torch.float64), atol=1e-12)
    assert torch.det(Rm).item() == pytest.approx(1.0)


def test_pose_composition_left_multiplied():
    """poses.py:27-30: c2w = make_c2w(r, t) @ init_c2w (translation not rotated by r)."""
    init = torch.eye(4, dtype=torch.float64)
    init[:3, 3] = torch.tensor([1.0, 2.0, 3.0])
    r = torch.zeros(1, 3, dtype=torch.float64)
    t = torch.tensor([[0.5, 0.0, 0.0]], dtype=torch.float64)
    c2w = orc.learn_pose_forward(r, t, init.unsqueeze(0), 0)
    assert torch.allclose(c2w[:3, 3], torch.tensor([1.5, 2.0, 3.0], dtype=torch.float64))


def test_distortion_clamp_and_fixed_last():
    scales = torch.tensor([[0.001], [2.0], [5.0]])
    shifts = torch.tensor([[0.1], [0.2], [0.3]])
    s0, _ = orc.learn_distortion_forward(scales, shifts, 0)
    s2, sh2 = orc.learn_distortion_forward(scales, shifts, 2)
    assert s0.item() == pytest.approx(0.01) and s2.item() == 1.0 and sh2.item() == pytest.approx(0.3)


def test_pixel_grid_and_camera():
    """common.py:36-39 (no +0.5 offset, W-1 normalisation) and dataset.py:83-86."""
    loc, sc = orc.arange_pixels(3, 5)
    assert torch.equal(loc[0, :6], torch.tensor([[0, 0], [1, 0], [2, 0], [3, 0], [4, 0], [0, 1]]))
    assert sc[0, 0].tolist() == [-1.0, -1.0] and sc[0, -1].tolist() == [1.0, 1.0]
    K = orc.camera_K(188, 621, 362.5, 362.5)
    assert K[0, 1, 1].item() == pytest.approx(-2 * 362.5 / 188)


def test_ray_generation_identity_camera():
    """With world = scale = I, the ray of pixel (0,0) is K^-1 [0,0,1] - 0 = (0,0,-1):
    the camera looks down -z; d_gt = depth * |ray|."""
    K = orc.camera_K(100, 100, 50.0, 50.0)
    px = torch.tensor([[[0.0, 0.0], [0.5, -0.5]]])
    depth = torch.tensor([[[2.0], [3.0]]])
    cam, ray, d_src, ray_norm, mask = orc.rays_from_cameras(px, depth, K, torch.eye(4)[None], torch.eye(4)[None])
    assert torch.allclose(cam, torch.zeros(2, 3))
    assert torch.allclose(ray[0], torch.tensor([0.0, 0.0, -1.0]))
    assert torch.allclose(d_src, depth[0, :, 0] * ray_norm)
    assert mask.all()
    d0 = torch.tensor([[[0.0], [3.0]]])
    assert orc.rays_from_cameras(px, d0, K, torch.eye(4)[None], torch.eye(4)[None])[4].tolist() == [False, True]


def test_stratified_samples_stay_in_bins():
    R, S = 4, 32
    noise = torch.rand(1, R, S)
    z = orc.stratified_z(R, S, 0.01, 10.0, noise)[0]
    base = orc.stratified_z(R, S, 0.01, 10.0, None)[0]
    mid = 0.5 * (base[:, 1:] + base[:, :-1])
    assert (z[:, 1:] >= mid - 1e-6).all() and (z[:, :-1] <= mid + 1e-6).all()
    assert (z[:, 0] >= 0.01).all() and (z[:, -1] <= 10.0 + 1e-6).all()
    assert torch.allclose(orc.stratified_z(1, S, 0.01, 10.0, torch.zeros(1, 1, S))[0, 0, 1:],
                          mid[0], atol=1e-6)


def test_losses_reference_normalisation():
    """losses.py:28-33 / 60-66: rgb sum over rays divided by R; depth l1 divided by M."""
    rgb = torch.zeros(1, 4, 3)
    gt = torch.ones(1, 4, 3)
    assert orc.rgb_full_loss(rgb, gt, "l2").item() == 3.0
    assert orc.rgb_full_loss(rgb, 2 * gt, "l1").item() == 6.0
    assert orc.depth_l1_loss(torch.tensor([1.0, 2.0]), torch.tensor([0.0, 0.0])).item() == 1.5
    assert orc.mse2psnr(0.01) == pytest.approx(20.0)
    assert orc.mse2psnr(0.0) == pytest.approx(100.0)


def test_chamfer_bruteforce():
    X = torch.tensor([[0.0, 0, 0], [10.0, 0, 0]]).t()
    Y = torch.tensor([[1.0, 0, 0], [9.0, 0, 0], [9.5, 0, 0]]).t()
    assert orc.closest_idx(X, Y).tolist() == [0, 2]
    assert orc.point_point_error(X, Y).item() == pytest.approx(0.75)


def test_anneal_schedule():
    """training.py:204-212 and the straight_d1 quirk."""
    assert orc.anneal(0.04, 0.0, 0, 0, 0) == 0.04
    assert orc.anneal(0.04, 0.0, 0, 0, 1) == 0.0
    assert orc.anneal(1.0, 0.0, 10, 10, 15) == pytest.approx(0.5)


def test_pair_terms_vanish_for_identical_views():
    """training.py:305-405: two cameras with the same pose, image and depth reproject every
    point onto itself, so the chamfer (pc) and reprojection (rgb_s) terms are 0 while the
    render terms are not; the loss dict carries the distortion scale / shift."""
    from tests.helpers import camera_K, make_cfg, rigid_c2w
    H, W = 24, 32
    cfg = make_cfg(hidden=16, S=8)
    tcfg = dict(cfg["training"])
    yy, xx = torch.meshgrid(torch.linspace(0, 1, H), torch.linspace(0, 1, W), indexing="ij")
    img = torch.stack([xx, yy, xx * yy], 0).unsqueeze(0)
    depth = (2.0 + xx).unsqueeze(0)
    c2w = rigid_c2w(1)
    data = {"img": img, "img.depth": depth, "img.camera_mat": camera_K(H, W, 30.0, 30.0),
            "img.scale_mat": torch.eye(4).unsqueeze(0), "img.pose_gt": c2w.unsqueeze(0), "img.idx": torch.tensor([0]),
            "img.ref_imgs": img.clone(), "img.ref_depths": depth.clone(), "img.ref_idxs": torch.tensor([1]),
            "img.ref_pose_gt": c2w.unsqueeze(0)}
    torch.manual_seed(0)
    model = orc.OracleNerf(hidden_dim=16)
    pose = {"r": torch.zeros(2, 3), "t": torch.zeros(2, 3), "init_c2w": torch.stack([c2w, c2w])}
    dist = {"scales": torch.ones(2, 1), "shifts": torch.zeros(2, 1), "fix_scaleN": True}
    g = torch.Generator().manual_seed(1)
    ld = orc.compute_loss_full(model, pose, dist, data, tcfg, cfg["rendering"], 0, 0,
                               torch.randperm(H * W, generator=g)[:64], torch.rand(1, 64, 8, generator=g))
    assert ld["loss_pc"].item() < 1e-5
    assert ld["loss_rgb_s"].item() < 1e-6
    assert ld["loss_rgb"].item() > 0 and ld["loss_depth"].item() > 0
    assert ld["scale"].item() == 1.0 and ld["shift"].item() == 0.0

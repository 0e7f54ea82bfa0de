"""Host-side logic of the drop-in package, checked against the oracle on the CPU
(no compute call reaches the HIP library here)."""
import pytest
import torch

import model as mdl
from model import field
from model.losses import Loss
from model.rendering import camera_rays
from oracle import nerf_oracle as orc
from tests.helpers import make_cfg, synthetic_rays


def test_state_dict_interop_with_reference_layout():
    cfg = make_cfg(hidden=256)
    torch.manual_seed(42)
    net = mdl.OfficialStaticNerf(cfg)
    torch.manual_seed(42)
    ref = orc.OracleNerf(256)
    sd, sr = net.state_dict(), ref.state_dict()
    assert list(sd) == list(sr)                      # reference key names, same order
    for k in sd:
        assert torch.equal(sd[k], sr[k]), k          # same init under the same seed (train.py:23-24)


def test_encoding_levels_are_hard_wired():
    cfg = make_cfg()
    cfg["model"]["pos_enc_levels"] = 6
    with pytest.raises(ValueError, match="hard-codes"):
        mdl.OfficialStaticNerf(cfg)


def test_no_cpu_fallback():
    net = mdl.OfficialStaticNerf(make_cfg(hidden=64))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        net(torch.rand(4, 3), torch.rand(4, 3))


def test_camera_rays_match_oracle():
    b = synthetic_rays(R=300, S=8, seed=1)
    cam, ray, rn, d_src, mask = camera_rays(b["pixels"], b["depth"], b["K"], b["w2c"], b["scale"])
    oc, orr, od, orn, om = orc.rays_from_cameras(b["pixels"], b["depth"], b["K"], b["w2c"], b["scale"])
    assert torch.allclose(cam, oc, atol=1e-6) and torch.allclose(ray, orr, atol=1e-6)
    assert torch.allclose(d_src, od, rtol=1e-6) and torch.allclose(rn, orn, rtol=1e-6)
    assert torch.equal(mask, om) and (~mask).any()


def test_dense_depth_loss_equals_masked_loss():
    """the sync-free dense form gives the reference's masked l1 value (losses.py:60-66)."""
    L = Loss(make_cfg()["training"])
    dp = torch.rand(50)
    dg = torch.rand(50)
    dg[::7] = float("inf")
    mask = torch.isfinite(dg)
    dense = L.get_depth_loss(dp, dg, mask)
    masked = orc.depth_l1_loss(dp[mask], dg[mask])
    assert torch.allclose(dense, masked)


def test_loss_dict_keys_and_values():
    cfg = make_cfg()["training"]
    L = Loss(cfg)
    w = {"rgb_weight": 1.0, "depth_weight": 0.04, "pc_weight": 0.0, "rgb_s_weight": 0.0,
         "depth_consistency_weight": 0.0, "weight_dist_2nd_loss": 0.0, "weight_dist_1st_loss": 0.0,
         "t_cycle_weight": 0.0}
    rgb, gt = torch.rand(1, 64, 3), torch.rand(1, 64, 3)
    dp, dg = torch.rand(60), torch.rand(60)
    out = L(rgb, gt, dp, dg, weights=w, rgb_loss_type="l2", t_list=torch.zeros(3, 3))
    ref = orc.total_loss(rgb, gt, dp, dg, w, "l2")
    assert set(out) == {"loss", "loss_rgb", "loss_depth", "l2_mean", "loss_dist_1st", "loss_dist_2nd",
                        "loss_pc", "loss_rgb_s", "loss_depth_consistency", "loss_t_cycle"}
    for k in ("loss", "loss_rgb", "loss_depth", "l2_mean"):
        assert torch.allclose(out[k], ref[k])


def test_rgb_s_mask_mean_and_empty_mask():
    L = Loss(make_cfg()["training"])
    a, b = torch.rand(1, 5, 6, 3), torch.rand(1, 5, 6, 3)
    v = torch.rand(1, 5, 6, 1) > 0.5
    assert torch.allclose(L.get_rgb_s_loss(a, b, v), orc.rgb_s_loss(a, b, v))
    assert L.get_rgb_s_loss(a, b, torch.zeros_like(v)).item() == 0.0


def test_pose_and_distortion_modules_match_oracle():
    cfg = make_cfg()
    init = torch.stack([torch.eye(4), torch.eye(4)])
    init[1, :3, 3] = torch.tensor([0.1, 0.2, 0.3])
    lp = mdl.LearnPose(2, True, True, cfg, init_c2w=init)
    with torch.no_grad():
        lp.r.copy_(torch.tensor([[0.01, 0.02, -0.03], [0.2, -0.1, 0.05]]))
        lp.t.copy_(torch.tensor([[0.5, 0.0, 0.1], [0.0, -0.4, 0.2]]))
    for cam in (0, 1):
        assert torch.allclose(lp(torch.tensor(cam)), orc.learn_pose_forward(lp.r, lp.t, init, cam), atol=1e-7)
    ld = mdl.Learn_Distortion(3, True, True, cfg)
    with torch.no_grad():
        ld.global_scales.copy_(torch.tensor([[0.001], [2.0], [3.0]]))
    for cam in range(3):
        s, sh = ld(cam)
        so, sho = orc.learn_distortion_forward(ld.global_scales, ld.global_shifts, cam)
        assert torch.allclose(s.reshape(()), so.reshape(()).float()) and torch.allclose(sh, sho)


def test_library_default_is_benchmarked_path():
    """The library's default GEMM arithmetic is the one bench.py headlines (the fp16 pair,
    mode 2), so a drop-in caller of the reference API gets the benchmarked kernels and the
    fused per-ray eval kernel without any set-up call."""
    import bench
    from model import _hip
    lib = _hip.load_library()
    assert lib.nerf_gemm_get_precision() == 2
    assert bench.PRECISION[bench.DEFAULT_GEMM] == lib.nerf_gemm_get_precision()


def test_dw_split_policy():
    from model import _hip
    _hip.load_library()
    prev = _hip.gemm_get_precision()
    _hip.gemm_set_precision(0)
    try:
        assert _hip.bwd_weight_splits(256, 256, 131072) == 256     # exact f32: 256 x 256 tiles
        assert _hip.bwd_weight_splits(128, 256, 131072) == 256
        # split modes, default TN policy 8 (7's tiles on the 4-wave kernels): XCD-paired
        # 256 x 128 column tiles, 2 blocks per split; the colour layer's 128 x 256 tile, one per split
        _hip.gemm_set_precision(2)
        assert _hip.bwd_weight_splits(256, 256, 131072) == 128
        assert _hip.bwd_weight_splits(256, 64, 131072) == 256
        assert _hip.bwd_weight_splits(128, 256, 131072) == 256
        for pol in (7, 8):
            _hip.gemm_set_policy(0, pol)
            assert _hip.bwd_weight_splits(256, 256, 131072) == 128
        _hip.gemm_set_policy(0, 3)
        assert _hip.bwd_weight_splits(256, 256, 131072) == 256
        for bad in (1, 4, 5, 6, 9, -1):
            with pytest.raises(RuntimeError):
                _hip.gemm_set_policy(0, bad)
    finally:
        _hip.gemm_set_policy(0, 0)
        _hip.gemm_set_precision(prev)
    for m in (128, 1024, 16384, 131072, 131072 + 128):
        for nout, kin in ((256, 256), (128, 256), (256, 64), (64, 64)):
            s = _hip.bwd_weight_splits(nout, kin, m)
            assert s >= 1 and m % s == 0 and (m // s) % 32 == 0
    assert field._pad_rows(1) == 128 and field._pad_rows(131072) == 131072


def test_trainer_anneal_and_pixel_cache():
    cfg = make_cfg()
    tr = mdl.Trainer(None, None, cfg["training"], device=torch.device("cpu"))
    assert tr.anneal(0.04, 0.0, 0, 0, 0) == 0.04 and tr.anneal(0.04, 0.0, 0, 0, 1) == 0.0
    p = tr._pixels(4, 6, torch.device("cpu"))
    assert torch.equal(p, orc.arange_pixels(4, 6)[1])


def test_ray_resampling_guarantee():
    """training.py:280-283 resampling only triggers when the valid count can't guarantee a hit."""
    cfg = make_cfg()
    cfg["training"]["n_training_points"] = 4
    tr = mdl.Trainer(None, None, cfg["training"], device=torch.device("cpu"))
    mask = torch.zeros(1, 10, 10, dtype=torch.bool)
    mask[0, 9, 9] = True                  # one valid pixel: must resample until it is drawn
    torch.manual_seed(0)
    img = torch.rand(1, 3, 10, 10)
    idx, pix, rgb = tr.sample_rays(100, mask, True, img=img, hw=(10, 10))
    assert mask.flatten()[idx].any()
    assert torch.equal(pix, tr._pixels(10, 10, torch.device("cpu"))[:, idx])
    assert torch.equal(rgb, img.view(1, 3, 100).permute(0, 2, 1)[:, idx])
    # a mostly valid mask skips the (sync) check: the all-invalid draw is impossible
    cfg["training"]["n_training_points"] = 64
    tr2 = mdl.Trainer(None, None, cfg["training"], device=torch.device("cpu"))
    mask2 = torch.ones(1, 100, 100, dtype=torch.bool)
    mask2[0, :5] = False
    assert tr2.sample_rays(10000, mask2, True, img=torch.rand(1, 3, 100, 100), hw=(100, 100))[0].shape == (64,)


def test_hip_adam_hyper_block():
    """HipAdam's device hyper-parameter block (k_adam reads it): slot 6 is 1 - beta2 formed in
    double on the host and rounded once, as torch's Adam forms it -- not 1 - f32(beta2) -- and an
    edited param_group (an LR scheduler) is pushed on the next sync (checked on the GPU against
    torch's Adam in tests/test_gpu_checkpoint.py)."""
    from model.optim import HipAdam
    p = torch.nn.Parameter(torch.zeros(10))
    opt = HipAdam([p], lr=1e-3, betas=(0.9, 0.999), eps=1e-8)
    h = opt._hyper
    assert h[1].item() == torch.tensor(1e-3).item() and h[2].item() == torch.tensor(0.9).item()
    assert h[6].item() == torch.tensor(1.0 - 0.999, dtype=torch.float32).item()
    assert h[6].item() != (1.0 - torch.tensor(0.999, dtype=torch.float32)).item()
    # ABI 13: 1 - beta1 from the double too, and lr / beta1 / beta2 as doubles for the bias
    # corrections (slots 8-13), flagged valid by slot 15
    assert h[14].item() == torch.tensor(1.0 - 0.9, dtype=torch.float32).item()
    assert h[14].item() != (1.0 - torch.tensor(0.9, dtype=torch.float32)).item()
    assert h.cpu()[8:14].numpy().view("float64").tolist() == [1e-3, 0.9, 0.999] and h[15].item() == 1.0
    opt.param_groups[0]["lr"] = 5e-4
    opt.sync_hyper()
    assert opt._hyper[1].item() == torch.tensor(5e-4).item()
    assert opt._hyper.cpu()[8:10].numpy().view("float64")[0] == 5e-4
    assert p.data.data_ptr() == opt._flat.data_ptr()     # parameters are views of the flat buffer

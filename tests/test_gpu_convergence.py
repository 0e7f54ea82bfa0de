"""PSNR parity of training (BASELINE.json metric: "PSNR parity (±0.1 dB) vs ref") (GPU only).

The HIP path (Renderer.nope_nerf -> fused render fwd/bwd, Loss, HipAdam) and the oracle
(CPU restatement of training.py:70-100 with torch.optim.Adam) train the same
initial field on the same synthetic scene, with identical ray draws and stratified
noise each step.  After the run both render every pixel without noise and the PSNRs
(common.py:623-630) must agree within 0.1 dB; training must also have improved PSNR,
so the comparison is not between two untrained fields.  Tolerance: 0.1 dB (metric)."""
import math

import pytest
import torch

from model.losses import Loss
from model.official_nerf import OfficialStaticNerf
from model.optim import HipAdam
from model.rendering import Renderer
from oracle import nerf_oracle as orc
from tests.helpers import camera_K, make_cfg, rigid_c2w

pytestmark = pytest.mark.gpu

H, W, FX = 48, 72, 60.0


def _scene(seed=0):
    g = torch.Generator().manual_seed(seed)
    yy, xx = torch.meshgrid(torch.linspace(0, 1, H), torch.linspace(0, 1, W), indexing="ij")
    img = torch.stack([0.5 + 0.4 * torch.sin(7 * xx + 3 * yy), 0.5 + 0.4 * torch.cos(6 * yy - 2 * xx),
                       0.3 + 0.5 * xx * yy], 0).unsqueeze(0)
    depth = 2.0 + 3.0 * xx.unsqueeze(0).unsqueeze(0) + 0.1 * torch.rand(1, 1, H, W, generator=g)
    depth[torch.rand(1, 1, H, W, generator=g) < 0.05] = 0.0
    return img, depth


def _psnr_hip(rnd, pix, depth_flat, K, w2c, scale, img_flat, dev):
    with torch.no_grad():
        out = rnd.nope_nerf(pix.to(dev), depth_flat.to(dev), K.to(dev), w2c.to(dev), scale.to(dev),
                            add_noise=False, dense_depth=True)
    return orc.mse2psnr(((out["rgb"].cpu() - img_flat) ** 2).mean().item())


def _psnr_oracle(ref, pix, depth_flat, K, w2c, scale, img_flat, cfg):
    with torch.no_grad():
        out = orc.render_nope_nerf(ref, pix, depth_flat, K, w2c, scale, cfg, noise=None)
    return orc.mse2psnr(((out["rgb"] - img_flat) ** 2).mean().item())


@pytest.mark.parametrize("hidden,S,R,steps", [
    (64, 64, 256, 80),          # config 1 shape
    (256, 128, 1024, 25),       # the bench shape (config 2: D = 256, 1024 rays x 128 samples)
])
def test_training_psnr_parity(dev, gemm_precision, hidden, S, R, steps):
    cfg = make_cfg(hidden=hidden, S=S)
    r = cfg["rendering"]
    torch.manual_seed(42)                                            # train.py:23-24
    net = OfficialStaticNerf(cfg)
    ref = orc.OracleNerf(hidden_dim=hidden, white_background=r["white_background"], dist_alpha=r["dist_alpha"],
                         occ_activation=cfg["model"]["occ_activation"])
    ref.load_state_dict(net.state_dict())
    net = net.to(dev)
    rnd = Renderer(net, r, device=dev)
    loss_fn = Loss(cfg["training"])
    opt_h = HipAdam(net.parameters(), lr=1e-3)
    opt_o = torch.optim.Adam(ref.parameters(), lr=1e-3)

    img, depth_img = _scene()
    K = camera_K(H, W, FX, FX)
    c2w = rigid_c2w(3)
    w2c = torch.inverse(c2w).unsqueeze(0)
    scale = torch.eye(4).unsqueeze(0)
    pix = orc.arange_pixels(H, W)[1]                                 # (1, H*W, 2)
    img_flat = img.view(1, 3, -1).permute(0, 2, 1)
    depth_flat = depth_img.view(1, 1, -1).permute(0, 2, 1)
    weights = {"rgb_weight": 1.0, "depth_weight": 0.04, "pc_weight": 0.0, "rgb_s_weight": 0.0,
               "depth_consistency_weight": 0.0, "weight_dist_2nd_loss": 0.0, "weight_dist_1st_loss": 0.0,
               "t_cycle_weight": 0.0}

    p0_h = _psnr_hip(rnd, pix, depth_flat, K, w2c, scale, img_flat, dev)
    p0_o = _psnr_oracle(ref, pix, depth_flat, K, w2c, scale, img_flat, r)
    g = torch.Generator().manual_seed(7)
    loss_h, loss_o = [], []
    for _ in range(steps):
        ray_idx = torch.randperm(H * W, generator=g)[:R]
        noise = torch.rand(1, R, S, generator=g)
        ld, _ = orc.train_step_render(ref, opt_o, img, depth_img, K, c2w, scale, ray_idx, noise, r)
        loss_o.append(ld["loss"].item())
        opt_h.zero_grad()
        out = rnd.nope_nerf(pix[:, ray_idx].to(dev), depth_flat[:, ray_idx].to(dev), K.to(dev), w2c.to(dev),
                            scale.to(dev), add_noise=True, noise=noise.to(dev), dense_depth=True)
        lh = loss_fn(out["rgb"], img_flat[:, ray_idx].to(dev), out["depth_pred"], out["depth_gt"],
                     depth_mask=out["depth_mask"], weights=weights, rgb_loss_type="l2")
        lh["loss"].backward()
        opt_h.step()
        loss_h.append(lh["loss"].item())
    p1_h = _psnr_hip(rnd, pix, depth_flat, K, w2c, scale, img_flat, dev)
    p1_o = _psnr_oracle(ref, pix, depth_flat, K, w2c, scale, img_flat, r)

    assert abs(p0_h - p0_o) < 1e-3, (p0_h, p0_o)                   # same initial field
    assert p1_o > p0_o + 0.5, (p0_o, p1_o)                          # training did something
    print(f"PSNR init {p0_h:.4f}/{p0_o:.4f} dB, after {steps} steps HIP {p1_h:.4f} dB, oracle {p1_o:.4f} dB")
    assert abs(p1_h - p1_o) < 0.1, f"PSNR after {steps} steps: HIP {p1_h:.4f} dB vs oracle {p1_o:.4f} dB"
    assert math.isclose(loss_h[0], loss_o[0], rel_tol=1e-4)
    assert abs(loss_h[-1] - loss_o[-1]) < 0.02 * abs(loss_o[-1]) + 1e-4

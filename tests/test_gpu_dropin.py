"""The drop-in callers of the render path on the GPU: OfficialStaticNerf.infer_occ
(official_nerf.py:60-67) and Extract_Images.generate_images (extracting_images.py:40-133,
the cfg4 caller of vis/render.py) against the oracle."""
import numpy as np
import pytest
import torch

from model.official_nerf import OfficialStaticNerf
from model.rendering import Renderer
from oracle import nerf_oracle as orc
from tests.helpers import assert_elementwise, camera_K, make_cfg, rigid_c2w

pytestmark = pytest.mark.gpu


def _pair(cfg, seed=0):
    torch.manual_seed(seed)
    net = OfficialStaticNerf(cfg)
    ref = orc.OracleNerf(hidden_dim=cfg["model"]["hidden_dim"])
    ref.load_state_dict(net.state_dict())
    return net, ref


def _trunk(ref, p):
    enc = orc.encode_position(p, 10)
    x = ref.layers0(enc)
    return ref.layers1(torch.cat([x, enc], -1))


@pytest.mark.parametrize("hidden,n", [(64, 1000), (256, 4096)])
def test_infer_occ_matches_oracle(dev, gemm_precision, hidden, n):
    cfg = make_cfg(hidden=hidden)
    net, ref = _pair(cfg)
    net = net.to(dev)
    g = torch.Generator().manual_seed(1)
    p = (torch.rand(2, n // 2, 3, generator=g) - 0.5) * 4
    x, dens = net.infer_occ(p.to(dev))
    assert x.shape == (2, n // 2, hidden) and dens.shape == (2, n // 2, 1)
    with torch.no_grad():
        xr = _trunk(ref, p)
        dr = ref.fc_density(xr)
    # post-ReLU trunk activations: relative to the tensor scale (exact zeros on both sides)
    assert (x.cpu() - xr).abs().max().item() <= 1e-4 * xr.abs().max().item()
    assert_elementwise(dens.cpu(), dr, rtol=1e-4, atol=1e-5 * dr.abs().max().item(), what="density")
    # density is differentiable w.r.t. the points (gradient(), official_nerf.py:46-58)
    pg = p.to(dev).requires_grad_(True)
    _, d2 = net.infer_occ(pg)
    (gp,) = torch.autograd.grad(d2.sum(), pg)
    pr = p.clone().requires_grad_(True)
    (gr,) = torch.autograd.grad(ref.fc_density(_trunk(ref, pr)).sum(), pr)
    assert ((gp.cpu() - gr).norm() / gr.norm()).item() < 2e-3


def test_extract_images_matches_oracle(dev, gemm_precision, tmp_path):
    from model.extracting_images import Extract_Images
    h, w, S, hidden = 24, 40, 32, 64
    cfg = make_cfg(hidden=hidden, S=S)
    cfg["extract_images"] = {"resolution": [h, w]}
    net, ref = _pair(cfg, seed=3)
    rnd = Renderer(net.to(dev), cfg["rendering"], device=dev)
    K = camera_K(h, w, 30.0, 30.0)
    c2ws = torch.stack([rigid_c2w(5, 0.2), rigid_c2w(6, 0.2)])
    ex = Extract_Images(rnd, cfg, use_learnt_poses=True, use_learnt_focal=False, device=dev, render_type="nope_nerf")
    data = {"img.idx": torch.tensor([1]), "img.camera_mat": K, "img.scale_mat": torch.eye(4).unsqueeze(0)}
    out = ex.generate_images(data, str(tmp_path), c2ws.to(dev), None, 1000, False)
    # oracle: the same eval render of every pixel with a depth prior of ones
    pix = orc.arange_pixels(h, w)[1]
    with torch.no_grad():
        o = orc.render_nope_nerf(ref, pix, torch.ones(1, h * w, 1), K, torch.inverse(c2ws[1]).unsqueeze(0),
                                 torch.eye(4).unsqueeze(0), cfg["rendering"], noise=None, eval_=True)
    depth = np.load(tmp_path / "depth_out" / "1.npy")
    assert_elementwise(torch.from_numpy(depth).reshape(-1), o["depth_pred"].reshape(-1), what="depth")
    img_ref = (o["rgb"].reshape(h, w, 3).numpy() * 255).astype(np.uint8)
    # uint8 quantisation of the rendered colour: off by one only where the float sits on an edge
    assert np.abs(out["img"].astype(int) - img_ref.astype(int)).max() <= 1
    for sub in ("img_out/0001.png", "depth_out/0001.png", "disp_out/0001.png"):
        assert (tmp_path / sub).exists()
    assert out["disp"].shape == (h, w, 3) and out["depth"].dtype == np.uint8

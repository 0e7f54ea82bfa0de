"""Gradients of the HIP field outside the render path (GPU only): infer_occ's trunk output x
and the normal_loss branch (rendering.py:127-137) against the oracle, and the loud failure
of the second derivatives the HIP backward does not provide."""
import pytest
import torch

import model as mdl
from oracle import nerf_oracle as orc
from tests.helpers import assert_elementwise, make_cfg, synthetic_rays

pytestmark = pytest.mark.gpu


def _pair(D, seed=0):
    cfg = make_cfg(hidden=D, S=32)
    torch.manual_seed(seed)
    net = mdl.OfficialStaticNerf(cfg)
    ref = orc.OracleNerf(hidden_dim=D)
    ref.load_state_dict(net.state_dict())
    return cfg, net, ref


def _nrel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("D", [64, 256])
def test_infer_occ_x_and_density_gradients_match_oracle(dev, gemm_precision, D):
    """official_nerf.py:60-67: a loss on BOTH outputs of infer_occ (the trunk output x and
    fc_density(x)) backpropagates to the points and every parameter as the oracle's autograd."""
    cfg, net, ref = _pair(D)
    net = net.to(dev)
    g = torch.Generator().manual_seed(1)
    p = (torch.rand(1000, 3, generator=g) - 0.5) * 2.0
    wx = torch.randn(1000, D, generator=g)
    ph = p.to(dev).requires_grad_(True)
    x, dens = net.infer_occ(ph)
    loss = (x * wx.to(dev)).sum() + dens.square().sum()
    loss.backward()
    po = p.clone().requires_grad_(True)
    enc = orc.encode_position(po, 10)
    xo = ref.layers1(torch.cat([ref.layers0(enc), enc], -1))
    lo = (xo * wx).sum() + ref.fc_density(xo).square().sum()
    lo.backward()
    assert_elementwise(x, xo, rtol=1e-4, atol=1e-5, what="x")
    assert _nrel(ph.grad, po.grad) < 2e-3
    for (n1, p1), (n2, p2) in zip(net.named_parameters(), ref.named_parameters()):
        if p2.grad is None:                      # the colour branch: no path from infer_occ
            assert p1.grad is None or float(p1.grad.abs().max()) == 0.0, n1
            continue
        assert _nrel(p1.grad, p2.grad) < 2e-3, (n1, _nrel(p1.grad, p2.grad))


def test_normal_loss_branch_matches_oracle_and_refuses_second_order(dev):
    """rendering.py:127-137: with normal_loss on, the training render returns 'normal' =
    |n(x) - n(x + jitter)| at the depth-prior surface points, as the oracle computes it from
    its autograd gradient(); a loss on it (a second derivative through the field) raises."""
    D, S, R = 64, 32, 256
    cfg, net, ref = _pair(D, seed=4)
    cfg["rendering"]["normal_loss"] = True
    b = synthetic_rays(R=R, S=S, H=40, W=50, seed=2)
    rnd = mdl.Renderer(net.to(dev), cfg["rendering"], device=dev)
    cam, ray, d_src, _, mask = orc.rays_from_cameras(b["pixels"], b["depth"], b["K"], b["w2c"], b["scale"])
    n_surf = int(mask.sum())
    assert 0 < n_surf < R
    jitter = torch.rand(n_surf, 3, generator=torch.Generator().manual_seed(8))
    out = rnd.nope_nerf(b["pixels"].to(dev), b["depth"].to(dev), b["K"].to(dev), b["w2c"].to(dev),
                        b["scale"].to(dev), add_noise=True, noise=b["noise"].to(dev), dense_depth=True,
                        normal_noise=jitter.to(dev))
    want = orc.normal_diff(ref, cam, ray, d_src, mask, jitter)
    assert out["normal"].shape == want.shape
    assert (out["normal"].detach().cpu() - want).abs().max().item() < 2e-3
    assert out["normal"].requires_grad          # anchored: a loss on it reaches _FirstOrderOnly
    (out["rgb"].square().sum()).backward(retain_graph=True)       # the first-order path still trains
    # a combined loss (rgb + w * normal) must fail loudly, not drop the normal term
    with pytest.raises(RuntimeError, match="second derivatives"):
        (out["rgb"].square().sum() + 0.1 * out["normal"].sum()).backward()
    # eval renders carry no normal term (rendering.py:127: `not eval_`)
    with torch.no_grad():
        ev = rnd.nope_nerf(b["pixels"].to(dev), b["depth"].to(dev), b["K"].to(dev), b["w2c"].to(dev),
                           b["scale"].to(dev), add_noise=False, eval_=True)
    assert ev["normal"] is None

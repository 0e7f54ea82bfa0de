"""Golden fixtures (tests/golden/make_golden.py): the oracle must keep reproducing them
(CPU), and the HIP path must match them within the north-star tolerance (GPU)."""
import glob
import os

import pytest
import torch

from oracle import nerf_oracle as orc

FILES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "render_*.pt")))


def _load(f):
    return torch.load(f, weights_only=True)


def _net(fx, cls):
    c = fx["cfg"]
    return cls(hidden_dim=fx["hidden"], white_background=c.get("white_background", False),
               dist_alpha=c.get("dist_alpha", False))


@pytest.mark.parametrize("f", FILES, ids=[os.path.basename(f) for f in FILES])
def test_oracle_reproduces_fixture(f):
    fx = _load(f)
    net = _net(fx, orc.OracleNerf)
    net.load_state_dict(fx["state_dict"])
    i = fx["inputs"]
    out = orc.render_nope_nerf(net, i["pixels"], i["depth"], i["K"], i["w2c"], i["scale"], fx["cfg"], noise=fx["noise"])
    assert torch.allclose(out["rgb"], fx["rgb"], rtol=1e-6, atol=1e-7)
    assert torch.allclose(out["depth_pred"], fx["depth_pred"], rtol=1e-6, atol=1e-6)
    assert torch.equal(out["depth_gt"], fx["depth_gt"])


@pytest.mark.gpu
@pytest.mark.parametrize("f", FILES, ids=[os.path.basename(f) for f in FILES])
def test_hip_matches_fixture(dev, f):
    from model.official_nerf import OfficialStaticNerf
    from model.rendering import Renderer
    from tests.helpers import make_cfg
    fx = _load(f)
    c = fx["cfg"]
    cfg = make_cfg(hidden=fx["hidden"], S=c["num_points"], **{k: v for k, v in c.items() if k != "num_points"})
    net = OfficialStaticNerf(cfg)
    net.load_state_dict(fx["state_dict"])
    net = net.to(dev)
    rnd = Renderer(net, cfg["rendering"], device=dev)
    i = {k: v.to(dev) for k, v in fx["inputs"].items()}
    noise = fx["noise"].to(dev) if fx["noise"] is not None else None
    out = rnd.nope_nerf(i["pixels"], i["depth"], i["K"], i["w2c"], i["scale"], add_noise=noise is not None,
                        noise=noise)
    from tests.helpers import assert_elementwise
    assert_elementwise(out["rgb"], fx["rgb"], what="rgb")                  # |a-b| <= 1e-4 |b| + 1e-6
    assert_elementwise(out["depth_pred"], fx["depth_pred"], what="depth")
    loss = orc.rgb_full_loss(out["rgb"], fx["gt"].to(dev)) + 0.04 * orc.depth_l1_loss(out["depth_pred"], out["depth_gt"])
    assert abs(loss.item() - fx["loss"].item()) < 1e-4 * abs(fx["loss"].item())
    loss.backward()
    params = dict(net.named_parameters())
    for n, g in fx["grads"].items():
        err = ((params[n].grad.cpu() - g).norm() / g.norm().clamp_min(1e-12)).item()
        assert err < 2e-3, f"{n}: {err:.2e}"

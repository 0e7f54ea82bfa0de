"""fp64 finite-difference gradient checks of the oracle (CPU).  The HIP backward is
checked against the oracle's autograd on the GPU; these tests pin that autograd."""
import torch

from oracle import nerf_oracle as orc


def test_composite_gradcheck():
    torch.manual_seed(0)
    alpha = (torch.rand(3, 10, dtype=torch.float64) * 0.9).requires_grad_(True)
    rgb = torch.rand(3, 10, 3, dtype=torch.float64, requires_grad=True)
    z = torch.sort(torch.rand(3, 10, dtype=torch.float64), 1)[0]

    def f(a, c):
        o, d, _, _ = orc.composite(a, c, z)
        return o, d
    assert torch.autograd.gradcheck(f, (alpha, rgb), eps=1e-6, atol=1e-7)


def test_composite_dist_alpha_gradcheck():
    torch.manual_seed(1)
    sig = (torch.rand(2, 8, dtype=torch.float64) * 3).requires_grad_(True)
    rgb = torch.rand(2, 8, 3, dtype=torch.float64)
    z = torch.sort(torch.rand(2, 8, dtype=torch.float64), 1)[0]
    assert torch.autograd.gradcheck(lambda s: orc.composite(s, rgb, z, dist_alpha=True)[:2], (sig,),
                                    eps=1e-6, atol=1e-7)


def test_render_gradcheck_small_field():
    """rays -> samples -> MLP -> composite, w.r.t. the pose (r, t) and the field weights."""
    torch.manual_seed(2)
    net = orc.OracleNerf(hidden_dim=8).double()
    R, S = 4, 6
    px = torch.rand(1, R, 2, dtype=torch.float64) * 2 - 1
    depth = 1 + torch.rand(1, R, 1, dtype=torch.float64)
    K = orc.camera_K(20, 30, 15.0, 15.0, torch.float64)
    noise = torch.rand(1, R, S, dtype=torch.float64)
    cfg = {"num_points": S, "depth_range": [0.5, 3.0]}

    def f(r, t):
        c2w = orc.make_c2w(r, t)
        w2c = torch.inverse(c2w).unsqueeze(0)
        o = orc.render_nope_nerf(net, px, depth, K, w2c, torch.eye(4, dtype=torch.float64)[None], cfg, noise)
        return o["rgb"], o["depth_pred"]

    r = (torch.rand(3, dtype=torch.float64) * 0.1).requires_grad_(True)
    t = (torch.rand(3, dtype=torch.float64) * 0.1).requires_grad_(True)
    assert torch.autograd.gradcheck(f, (r, t), eps=1e-6, atol=1e-6)

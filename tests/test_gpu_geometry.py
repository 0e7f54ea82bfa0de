"""Geometry visualisation path (rendering.py:199-468): ray
marching of the occupancy surface, secant refinement and Phong shading, HIP field vs the
oracle (GPU only).

The field is built by hand so the surface is known: the trunk passes |x|, |y|, |z| (as
ReLU(+-x)) through identity layers and the density head gives sigma_raw = 3 - 5 |x|_1, so
occupancy = 1 - exp(-softplus(sigma_raw)) crosses tau = 0.5 on the octahedron |x|_1 = 0.6.
Checked: the surface distances d_i (1e-4 absolute; the analytic value too), the hit mask,
the shaded colours (1e-4) and the field colour at the surface (1e-4)."""
import math

import pytest
import torch

import model as mdl
from oracle import nerf_oracle as orc
from tests.helpers import make_cfg

pytestmark = pytest.mark.gpu

D = 64


def _octahedron_field(cfg):
    torch.manual_seed(3)
    net = mdl.OfficialStaticNerf(cfg)
    with torch.no_grad():
        for lin in list(net.layers0)[::2] + list(net.layers1)[::2]:
            lin.weight.zero_()
            lin.bias.zero_()
        w0 = net.layers0[0].weight                       # encoding channels 0-2 are x itself
        for c in range(3):
            w0[2 * c, c], w0[2 * c + 1, c] = 1.0, -1.0
        for lin in list(net.layers0)[2::2] + list(net.layers1)[::2]:
            for i in range(6):
                lin.weight[i, i] = 1.0
        net.fc_density.weight.zero_()
        net.fc_density.weight[0, :6] = -5.0
        net.fc_density.bias.fill_(3.0)
    return net


def _camera(H, W):
    c2w = torch.eye(4)
    c2w[:3, 3] = torch.tensor([0.15, -0.1, 2.0])           # off-axis: faces and edges both hit
    K = torch.tensor([[4.0, 0, 0, 0], [0, -4.0, 0, 0], [0, 0, -1, 0], [0, 0, 0, 1]]).unsqueeze(0)
    return K, torch.inverse(c2w).unsqueeze(0), torch.eye(4).unsqueeze(0)


def test_phong_renderer_matches_oracle(dev):
    cfg = make_cfg(hidden=D, S=32)
    net = _octahedron_field(cfg)
    ref = orc.OracleNerf(hidden_dim=D)
    ref.load_state_dict(net.state_dict())
    H, W = 16, 24
    pix = orc.arange_pixels(H, W)[1]
    K, w2c, S = _camera(H, W)
    out_o = orc.phong_renderer(ref, pix, K, w2c, S, rad=cfg["rendering"]["radius"])
    rnd = mdl.Renderer(net, cfg["rendering"], device=dev)
    out_h = rnd.phong_renderer(pix.to(dev), K.to(dev), w2c.to(dev), S.to(dev), it=0)
    mask = out_o["mask"]
    assert 0.2 * H * W < mask.sum() < 0.9 * H * W          # the surface covers part of the frame
    # the hit points lie on the analytic surface |x|_1 = 0.6
    cam = torch.tensor([0.15, -0.1, 2.0])
    ray = orc.image_points_to_world(pix, K, w2c, S)[0] - cam
    ray = ray / ray.norm(dim=-1, keepdim=True)
    d_o = out_o["d_i"][0]
    hit = cam + ray[mask] * d_o[mask].unsqueeze(-1)
    assert (hit.abs().sum(-1) - 0.6).abs().max().item() < 1e-4
    # HIP vs oracle: hit mask, shading, surface colour
    rgb_h, rgb_o = out_h["rgb"].cpu()[0], out_o["rgb"][0]
    bg_h = (rgb_h == 1).all(-1)
    assert (bg_h != ~mask).sum().item() <= 2
    same = (bg_h == ~mask)
    assert (rgb_h[same] - rgb_o[same]).abs().max().item() < 1e-4
    surf_h, surf_o = out_h["rgb_surf"].cpu()[0], out_o["rgb_surf"][0]
    assert (surf_h[same & mask] - surf_o[same & mask]).abs().max().item() < 1e-4


def test_sphere_intersection_and_ray_marching_edges(dev):
    """get_sphere_intersection near/far distances (clamped at 0, 0 without a hit) and the
    two special ray-marching outcomes: inf (no surface) and 0 (start inside)."""
    from model.rendering import get_sphere_intersection
    cam = torch.tensor([[0.0, 0.0, 3.0]])
    dirs = torch.tensor([[[0.0, 0.0, -1.0], [1.0, 0.0, 0.0], [0.0, 0.0, 1.0]]])
    i_h, m_h = get_sphere_intersection(cam.to(dev), dirs.to(dev), r=1.0)
    i_o, m_o = orc.get_sphere_intersection(cam, dirs, r=1.0)
    assert torch.equal(m_h.cpu(), m_o) and torch.allclose(i_h.cpu(), i_o)
    assert torch.allclose(i_o[0, 0], torch.tensor([2.0, 4.0]))
    cfg = make_cfg(hidden=D, S=32)
    net = _octahedron_field(cfg)
    rnd = mdl.Renderer(net, cfg["rendering"], device=dev)
    ray0 = torch.tensor([[[0.0, 0.0, 3.0], [0.0, 0.0, 3.0], [0.1, 0.0, 0.0]]])
    rdir = torch.tensor([[[0.0, 0.0, -1.0], [1.0, 0.0, 0.0], [0.0, 0.0, -1.0]]])
    with torch.no_grad():
        d = rnd.ray_marching(ray0.to(dev), rdir.to(dev), net, n_steps=[512, 513], rad=4.0).cpu()[0]
    assert abs(d[0].item() - 2.4) < 1e-4                    # hits z = 0.6
    assert math.isinf(d[1].item())                          # misses the octahedron
    assert d[2].item() == 0.0                               # starts inside

"""The fused layer chain (chain.hip, GEMM precision mode 2) against one launch per layer
(gemm_x6.hip, same mode): every saved activation, ReLU bit, column maximum, the rendered
outputs and the parameter gradients (GPU only)."""
import os

import pytest
import torch

from model import _hip
from model.field import render_field, render_field_eval
from model.official_nerf import OfficialStaticNerf
from tests.helpers import make_cfg, synthetic_rays

pytestmark = pytest.mark.gpu


def _run(net, b, dev, chain: bool, keep=True):
    os.environ["NERF_CHAIN"] = "1" if chain else "0"
    try:
        runner = net.hip_runner()
        assert runner.use_chain(keep) == chain
        R, S = b["R"], b["S"]
        o, d = b["o"].to(dev), b["d"].to(dev)
        rgb, dist, alpha, z, st = runner.forward(o, d, -d, b["noise"].to(dev), 0.01, 10.0, S, 0, keep=keep)
        torch.cuda.synchronize()
        return rgb, dist, st
    finally:
        os.environ.pop("NERF_CHAIN", None)


@pytest.fixture
def h16(dev):
    old = _hip.gemm_get_precision()
    _hip.gemm_set_precision(2)
    yield
    _hip.gemm_set_precision(old)


def _net(dev, seed=0, spread=True):
    torch.manual_seed(seed)
    net = OfficialStaticNerf(make_cfg(hidden=256, S=64)).to(dev)
    if not spread:
        return net
    with torch.no_grad():   # spread the weights' scales over layers and rows
        for i, p in enumerate(net.parameters()):
            if p.dim() == 2:
                p.mul_(torch.logspace(-1, 1, p.shape[0], device=dev).unsqueeze(1) * (0.5 + 0.1 * i))
    return net


def _rays(R, S, seed):
    g = torch.Generator().manual_seed(seed)
    o = (torch.rand(R, 3, generator=g) - 0.5) * 4
    d = torch.nn.functional.normalize(torch.rand(R, 3, generator=g) - 0.5, dim=-1)
    return {"R": R, "S": S, "o": o, "d": d, "noise": torch.rand(R, S, generator=g)}


@pytest.mark.parametrize("R,S", [(64, 64), (300, 32), (1024, 128)])
def test_chain_matches_per_layer(dev, h16, R, S):
    net = _net(dev)
    b = _rays(R, S, seed=R + S)
    rgb1, dist1, st1 = _run(net, b, dev, chain=True)
    rgb0, dist0, st0 = _run(net, b, dev, chain=False)
    rel = lambda a, r: ((a - r).abs().max() / r.abs().max().clamp_min(1e-30)).item()
    for i, (a1, a0) in enumerate(zip(st1["acts"], st0["acts"])):
        assert rel(a1, a0) < 2e-6, f"activation {i}: {rel(a1, a0)}"
    for k, m0 in st0["masks"].items():
        m1 = st1["masks"][k]
        act = st0["acts"][[l.name for l in net.hip_runner().layers].index(k)]
        # ReLU bits agree wherever the activation is not within rounding of zero
        bits = lambda m: ((m.long() & 0xffffffff).unsqueeze(-1) >> torch.arange(32, device=dev)) & 1
        differ = (bits(m1) != bits(m0)).view(act.shape)
        assert (act[differ].abs() < 1e-5).all(), k
    for k, c0 in st0["cmaxes"].items():
        if c0 is None or k.startswith("enc"):
            continue
        assert rel(st1["cmaxes"][k], c0) < 2e-6, k
    assert rel(rgb1, rgb0) < 1e-5 and rel(dist1, dist0) < 1e-5


def test_chain_eval_skips_intermediate_stores(dev, h16):
    """keep=False (eval renders): only the trunk output and the colour hidden are stored."""
    net = _net(dev, seed=1)
    b = _rays(512, 64, seed=3)
    o, d = b["o"].to(dev), b["d"].to(dev)
    os.environ["NERF_CHAIN"] = "1"
    try:
        rgb1, dist1, _, _ = render_field_eval(net, o, d, -d, 0.01, 10.0, 64, 0, ray_chunk=200)
    finally:
        os.environ.pop("NERF_CHAIN", None)
    os.environ["NERF_CHAIN"] = "0"
    try:
        rgb0, dist0, _, z0 = render_field_eval(net, o, d, -d, 0.01, 10.0, 64, 0, ray_chunk=200)
    finally:
        os.environ.pop("NERF_CHAIN", None)
    torch.cuda.synchronize()
    # chain (the fused per-ray kernel at S = 64) and per-layer launches sum the K products in
    # different orders (16x16x32 tiles in chain_perm order vs 32x32x16), so with the row-spread
    # weights a ReLU decision near zero can move a ray by ~1e-5: the arbiter is the fp64 oracle,
    # which the chain must track as closely as the per-layer path does
    from oracle import nerf_oracle as orc
    ref = orc.OracleNerf(hidden_dim=256).double()
    ref.load_state_dict({k: v.detach().cpu().double() for k, v in net.state_dict().items()})
    z = z0.cpu().double()
    pts = b["o"].double()[:, None, :] + b["d"].double()[:, None, :] * z[..., None]
    with torch.no_grad():
        rgb_s, a_s = ref(pts.reshape(-1, 3), (-b["d"].double())[:, None, :].expand(512, 64, 3).reshape(-1, 3))
        ro = orc.composite(a_s.reshape(512, 64), rgb_s.reshape(512, 64, 3), z)
    for a1, a0, r in ((rgb1, rgb0, ro[0]), (dist1, dist0, ro[1])):
        e1 = (a1.cpu().double() - r).abs().max().item()
        e0 = (a0.cpu().double() - r).abs().max().item()
        assert e1 <= 1.5 * e0 + 1e-6, (e1, e0)
        # the oracle check above is the main one; the cross-path bound is what is measured
        # (round 6: tightened from 5e-5, the value is in the message when it fails)
        rel = ((a1 - a0).abs().max() / a0.abs().max()).item()
        assert rel < 2e-5, rel


def test_chain_gradients_match_per_layer(dev, h16):
    net = _net(dev, seed=2)
    b = _rays(256, 64, seed=5)
    grads = []
    for chain in (True, False):
        os.environ["NERF_CHAIN"] = "1" if chain else "0"
        try:
            net.zero_grad()
            o, d = b["o"].to(dev).requires_grad_(), b["d"].to(dev)
            rgb, dist, _, _ = render_field(net, o, d, -d, b["noise"].to(dev), 0.01, 10.0, 64, 0)
            (rgb.square().sum() + 0.1 * dist.sum()).backward()
            torch.cuda.synchronize()
            grads.append([p.grad.clone() for p in net.parameters()] + [o.grad.clone()])
        finally:
            os.environ.pop("NERF_CHAIN", None)
    for g1, g0 in zip(*grads):
        assert ((g1 - g0).norm() / g0.norm().clamp_min(1e-30)).item() < 1e-5


# ---- the fused per-ray eval kernel (nerf_render_eval_fused) ----------------------------
@pytest.mark.parametrize("R,S,flags", [(1024, 128, 0), (333, 64, 0), (257, 32, 2), (130, 16, 1), (97, 128, 4),
                                       (5, 2, 0)],
                         ids=["cfg4-S128", "S64-ragged", "S32-white", "S16-distalpha", "S128-relu", "S2-tiny"])
def test_fused_eval_matches_unfused_and_oracle(dev, h16, R, S, flags):
    """One launch (in-kernel samples + encodings, ten linears, heads, composite) against the
    unfused eval path (encode, chain, heads, composite launches) and the fp32 oracle."""
    from oracle import nerf_oracle as orc
    from tests.helpers import assert_elementwise
    # the reference initialisation: the chain-vs-per-layer tests stress the split with
    # row-spread weights; against the oracle the bar is the north-star 1e-4 on a normal field
    net = _net(dev, seed=S, spread=False)
    b = _rays(R, S, seed=R * 7 + S)
    o, d = b["o"].to(dev), b["d"].to(dev)
    view = -d
    runner = net.hip_runner()
    assert runner.use_fused_eval(S)
    rgb_f, dist_f, alpha_f, z_f = render_field_eval(net, o, d, view, 0.01, 10.0, S, flags)
    os.environ["NERF_FUSED"] = "0"
    try:
        assert not runner.use_fused_eval(S)
        rgb_u, dist_u, alpha_u, z_u = render_field_eval(net, o, d, view, 0.01, 10.0, S, flags)
    finally:
        os.environ.pop("NERF_FUSED", None)
    torch.cuda.synchronize()
    assert torch.equal(z_f, z_u)                                   # the same sample positions, bit for bit
    # against the oracle (fp32 CPU restatement of official_nerf.py + rendering.py:113-141)
    ref = orc.OracleNerf(hidden_dim=256, white_background=bool(flags & 2), dist_alpha=bool(flags & 1),
                         occ_activation="relu" if flags & 4 else "softplus")
    ref.load_state_dict({k: v.cpu() for k, v in net.state_dict().items()})
    z = z_u.cpu()
    pts = b["o"][:, None, :] + b["d"][:, None, :] * z[..., None]
    with torch.no_grad():
        rgb_s, a_s = ref(pts.reshape(-1, 3), (-b["d"])[:, None, :].expand(R, S, 3).reshape(-1, 3))
        ro = orc.composite(a_s.reshape(R, S), rgb_s.reshape(R, S, 3), z, dist_alpha=bool(flags & 1),
                           white_background=bool(flags & 2))
    assert_elementwise(rgb_f, ro[0], what="rgb vs oracle")
    assert_elementwise(dist_f, ro[1], what="dist vs oracle")
    assert_elementwise(rgb_u, ro[0], what="rgb (unfused) vs oracle")
    # fused vs unfused: the same chain arithmetic; the head dot products and the
    # composite's summation order differ (dist_alpha amplifies sigma differences by the bin
    # width), so the bar is the oracle's
    assert_elementwise(rgb_f, rgb_u, what="rgb fused vs unfused")
    assert_elementwise(dist_f, dist_u, what="dist fused vs unfused")
    assert (alpha_f - alpha_u).abs().max().item() < 1e-4


def test_fused_eval_falls_back_when_samples_do_not_tile(dev, h16):
    net = _net(dev)
    assert not net.hip_runner().use_fused_eval(96)          # 96 does not divide the 128-row block
    assert not net.hip_runner().use_fused_eval(256)
    b = _rays(40, 96, seed=3)
    o, d = b["o"].to(dev), b["d"].to(dev)
    rgb, dist, alpha, z = render_field_eval(net, o, d, -d, 0.01, 10.0, 96, 0)
    assert rgb.shape == (40, 3) and torch.isfinite(rgb).all()

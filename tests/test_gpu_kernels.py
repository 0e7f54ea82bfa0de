"""Per-kernel parity of the nerf_hip C-ABI against fp64 CPU references (GPU only).

Tolerances: FP32 MFMA GEMMs are exact-f32 fma chains, so against an fp64 reference the
error is ~1e-7 * sqrt(K) * |a||b|; we require max |err| <= 2e-5 * scale (rel 2e-5)."""
import pytest
import torch

from model import _hip
from oracle import nerf_oracle as orc

pytestmark = pytest.mark.gpu


def _rand(*s, g=None):
    return torch.rand(*s, generator=g) * 2 - 1


@pytest.mark.parametrize("m,n,k1,k2,relu", [(256, 256, 256, 0, 1), (384, 256, 64, 0, 1), (128, 256, 256, 64, 1),
                                            (256, 128, 256, 64, 1), (128, 64, 64, 0, 0), (512, 256, 256, 0, 0)])
def test_linear_fwd(dev, m, n, k1, k2, relu):
    g = torch.Generator().manual_seed(m + n + k1 + k2)
    x1 = _rand(m, k1, g=g)
    x2 = _rand(m, k2, g=g) if k2 else None
    W = _rand(n, k1 + k2, g=g) * 0.1
    b = _rand(n, g=g)
    y = torch.empty(m, n, device=dev)
    mo = torch.empty(m, n // 32, device=dev, dtype=torch.int32)
    _hip.linear_fwd(x1.to(dev), k1, x2.to(dev) if x2 is not None else None, k2, W.to(dev), b.to(dev), y, m, n, relu,
                    mask_out=mo)
    xc = torch.cat([x1, x2], 1) if x2 is not None else x1
    ref = xc.double() @ W.double().t() + b.double()
    if relu:
        ref = ref.clamp_min(0)
    torch.cuda.synchronize()
    assert (y.cpu().double() - ref).abs().max().item() < 2e-5 * max(1.0, ref.abs().max().item())
    bits = ((mo.cpu().long() & 0xffffffff).unsqueeze(-1) >> torch.arange(32)) & 1
    assert torch.equal(bits.view(m, n).bool(), y.cpu() > 0)          # ReLU bits agree with y


def test_linear_fwd_asymmetric_identity(dev):
    """A = I against an asymmetric B catches a transposed C write (guide section 3)."""
    m = n = k = 128
    x = torch.eye(m, k)
    W = torch.arange(n * k, dtype=torch.float32).view(n, k) / (n * k)
    y = torch.empty(m, n, device=dev)
    _hip.linear_fwd(x.to(dev), k, None, 0, W.to(dev), None, y, m, n, 0)
    assert torch.equal(y.cpu(), W.t().contiguous())


def test_linear_bwd_data(dev):
    g = torch.Generator().manual_seed(3)
    m, k, n = 256, 256, 128
    dy = _rand(m, k, g=g)
    Wt = _rand(n, k, g=g) * 0.1
    mask = _rand(m, n, g=g)
    u = _rand(m, 4, g=g)
    v = _rand(n, g=g)
    dx = torch.empty(m, n, device=dev)
    bits = (mask > 0).view(m, n // 32, 32).long() << torch.arange(32)
    words = bits.sum(-1)
    words = torch.where(words >= 2 ** 31, words - 2 ** 32, words).to(torch.int32)
    _hip.linear_bwd_data(dy.to(dev), k, Wt.to(dev), dx, m, n, mask=words.to(dev), u=u.to(dev), ldu=4, v=v.to(dev))
    ref = dy.double() @ Wt.double().t() + u[:, 0:1].double() * v.double()
    ref = torch.where(mask > 0, ref, torch.zeros_like(ref))
    torch.cuda.synchronize()
    assert (dx.cpu().double() - ref).abs().max().item() < 2e-5 * ref.abs().max().item()


@pytest.mark.parametrize("nout,kin,m,splits", [(256, 256, 4096, 8), (128, 320, 2048, 4), (256, 64, 1024, 1),
                                               (64, 128, 2048, 2)])
def test_linear_bwd_weight_and_reduce(dev, nout, kin, m, splits):
    g = torch.Generator().manual_seed(nout + kin)
    dy = _rand(m, nout, g=g)
    x = _rand(m, kin, g=g)
    k_main = kin - 64 if (kin % 128 and kin > 64) else kin
    slab = torch.empty(splits * nout * kin, device=dev)
    bslab = torch.empty(splits * nout, device=dev)
    dyd, xd = dy.to(dev), x.to(dev)
    _hip.linear_bwd_weight(dyd, nout, xd[:, :k_main], k_main, m, splits, slab, kin, 0, bslab)
    if k_main < kin:
        _hip.linear_bwd_weight(dyd, nout, xd[:, k_main:], kin - k_main, m, splits, slab, kin, k_main, None)
    kin_ref = kin - 1
    gw = torch.empty(nout, kin_ref, device=dev)
    gb = torch.empty(nout, device=dev)
    _hip.slab_reduce(slab, splits, nout, kin, nout, kin_ref, bslab, gw, gb)
    ref = dy.double().t() @ x.double()
    torch.cuda.synchronize()
    scale = ref.abs().max().item()
    assert (gw.cpu().double() - ref[:, :kin_ref]).abs().max().item() < 2e-5 * scale
    assert (gb.cpu().double() - dy.double().sum(0)).abs().max().item() < 1e-4 * max(1, dy.abs().sum(0).max().item())


@pytest.mark.parametrize("S,flags", [(128, 0), (64, 0), (128, 1), (100, 0), (128, 2), (128, 4), (200, 1)])
def test_composite_fwd_bwd(dev, S, flags):
    R = 37
    g = torch.Generator().manual_seed(S + flags)
    raw = torch.randn(R * S, 4, generator=g) * 2
    raw[:, 0] += 0.5
    z = torch.sort(torch.rand(R, S, generator=g) * 9 + 0.01, dim=1)[0].reshape(-1)
    Np = ((R * S + 127) // 128) * 128
    raw_p = torch.zeros(Np, 4)
    raw_p[:R * S] = raw
    z_p = torch.zeros(Np)
    z_p[:R * S] = z
    rgb = torch.empty(R, 3, device=dev)
    dist = torch.empty(R, device=dev)
    alpha = torch.empty(R, S, device=dev)
    _hip.composite_fwd(raw_p.to(dev), z_p.to(dev), R, S, flags, rgb, dist, alpha)
    # oracle: activations as official_nerf.py:77-92, compositing as rendering.py:113-141
    rr = raw.double().clone().requires_grad_(True)
    sig = torch.relu(rr[:, 0]) if flags & 4 else torch.nn.functional.softplus(rr[:, 0])
    if not flags & 1:
        sig = 1 - torch.exp(-sig)
    c = torch.sigmoid(rr[:, 1:])
    o_rgb, o_dist, o_alpha, _ = orc.composite(sig.view(R, S), c.view(R, S, 3), z.double().view(R, S),
                                              dist_alpha=bool(flags & 1), white_background=bool(flags & 2))
    torch.cuda.synchronize()
    assert (rgb.cpu().double() - o_rgb).abs().max().item() < 1e-5
    assert (dist.cpu().double() - o_dist).abs().max().item() < 1e-4
    assert (alpha.cpu().double() - o_alpha).abs().max().item() < 1e-5
    g_rgb = torch.randn(R, 3, generator=g)
    g_dist = torch.randn(R, generator=g) * 0.1
    graw = torch.empty(Np, 4, device=dev)
    _hip.composite_bwd(raw_p.to(dev), z_p.to(dev), R, S, flags, g_rgb.to(dev), g_dist.to(dev), graw, Np)
    (o_rgb * g_rgb.double()).sum().add((o_dist * g_dist.double()).sum()).backward()
    torch.cuda.synchronize()
    ref = rr.grad
    got = graw.cpu().double()
    assert (got[:R * S] - ref).abs().max().item() < 2e-4 * max(1.0, ref.abs().max().item())
    if Np > R * S:
        assert got[R * S:].abs().max().item() == 0.0


@pytest.mark.parametrize("hidden", [256, 64])
def test_heads_fwd_bwd(dev, hidden):
    Np = 512
    HR = max(64, hidden // 2)
    g = torch.Generator().manual_seed(hidden)
    h8 = torch.rand(Np, hidden, generator=g)
    hr = _rand(Np, HR, g=g).clamp_min(0)
    wd = _rand(1, hidden, g=g)
    bd = _rand(1, g=g)
    wc = _rand(3, HR, g=g)
    bc = _rand(3, g=g)
    raw4 = torch.empty(Np, 4, device=dev)
    _hip.heads_fwd(h8.to(dev), hr.to(dev), hidden, wd.to(dev), bd.to(dev), wc.to(dev), bc.to(dev), raw4, Np)
    ref = torch.cat([h8.double() @ wd.double().t() + bd.double(), hr.double() @ wc.double().t() + bc.double()], 1)
    torch.cuda.synchronize()
    assert (raw4.cpu().double() - ref).abs().max().item() < 2e-5 * ref.abs().max().item()
    graw = torch.randn(Np, 4, generator=g)
    dyr = torch.empty(Np, HR, device=dev)
    part = torch.empty(_hip.heads_part_size(hidden, Np), device=dev)
    _hip.heads_bwd(graw.to(dev), h8.to(dev), hr.to(dev), hidden, wc.to(dev), dyr, part, Np)
    gwd, gbd = torch.empty(hidden, device=dev), torch.empty(1, device=dev)
    gwc, gbc = torch.empty(3, HR, device=dev), torch.empty(3, device=dev)
    _hip.heads_reduce(part, hidden, Np, gwd, gbd, gwc, gbc)
    G = graw.double()
    r_dyr = torch.where(hr > 0, G[:, 1:] @ wc.double(), torch.zeros(Np, HR, dtype=torch.float64))
    torch.cuda.synchronize()
    assert (dyr.cpu().double() - r_dyr).abs().max().item() < 1e-5 * max(1, r_dyr.abs().max().item())
    assert (gwd.cpu().double() - G[:, 0] @ h8.double()).abs().max().item() < 1e-4 * Np
    assert (gwc.cpu().double() - G[:, 1:].t() @ hr.double()).abs().max().item() < 1e-4 * Np
    assert (gbd.cpu().double() - G[:, 0].sum()).abs().item() < 1e-3
    assert (gbc.cpu().double() - G[:, 1:].sum(0)).abs().max().item() < 1e-3


def test_encode_samples(dev):
    R, S = 33, 64
    g = torch.Generator().manual_seed(7)
    o = _rand(R, 3, g=g) * 3
    d = torch.nn.functional.normalize(_rand(R, 3, g=g), dim=-1)
    view = -d
    noise = torch.rand(R, S, generator=g)
    Np = ((R * S + 127) // 128) * 128
    z = torch.empty(Np, device=dev)
    ep = torch.empty(Np, 64, device=dev)
    ed = torch.empty(Np, 64, device=dev)
    _hip.encode_samples(o.to(dev), d.to(dev), view.to(dev), noise.to(dev), R, S, Np, 0.01, 10.0, z, ep, ed)
    oz = orc.stratified_z(R, S, 0.01, 10.0, noise.view(1, R, S))[0]
    pts = (o.unsqueeze(1) + d.unsqueeze(1) * oz.unsqueeze(-1)).reshape(-1, 3)
    ref_p = orc.encode_position(pts, 10)
    ref_d = orc.encode_position(view.unsqueeze(1).expand(R, S, 3).reshape(-1, 3), 4)
    torch.cuda.synchronize()
    zc, zr = z.cpu()[:R * S], oz.reshape(-1)
    bad = (zc != zr).nonzero().flatten()
    assert bad.numel() == 0, (f"{bad.numel()} z mismatches, first {bad[:8].tolist()}: "
                              f"{zc[bad[:4]].tolist()} vs {zr[bad[:4]].tolist()}")   # bit-exact samples
    assert (ep.cpu()[:R * S, :63] - ref_p).abs().max().item() < 2e-6
    assert (ed.cpu()[:R * S, :27] - ref_d).abs().max().item() < 2e-6
    assert ep.cpu()[:, 63].abs().max().item() == 0 and ed.cpu()[:, 27:].abs().max().item() == 0
    assert ep.cpu()[R * S:].abs().max().item() == 0


def test_chamfer_nn(dev):
    g = torch.Generator().manual_seed(11)
    X = torch.rand(3, 1000, generator=g) * 4
    Y = torch.rand(3, 1733, generator=g) * 4
    idx = torch.empty(1000, dtype=torch.int64, device=dev)
    _hip.chamfer_nn(X.t().contiguous().to(dev), Y.t().contiguous().to(dev), idx)
    torch.cuda.synchronize()
    assert torch.equal(idx.cpu(), orc.closest_idx(X, Y))
    # exact ties resolve to the first index like torch.argmin
    Xi = torch.tensor([[0.0, 0.0, 0.0]]).t()
    Yi = torch.tensor([[1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [-1.0, 0.0, 0.0]]).t()
    idx1 = torch.empty(1, dtype=torch.int64, device=dev)
    _hip.chamfer_nn(Xi.t().contiguous().to(dev), Yi.t().contiguous().to(dev), idx1)
    torch.cuda.synchronize()
    assert idx1.item() == 0 == orc.closest_idx(Xi, Yi).item()


def test_adam_matches_torch(dev):
    g = torch.Generator().manual_seed(5)
    p0 = torch.randn(10007, generator=g)
    p = p0.clone().to(dev)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    hyper = torch.tensor([0.0, 1e-3, 0.9, 0.999, 1e-8, 0.0], device=dev)
    tp = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([tp], lr=1e-3)
    for step in range(1, 6):
        gr = torch.randn(10007, generator=g)
        tp.grad = gr.clone()
        opt.step()
        _hip.adam_step(p, gr.to(dev), m, v, hyper)
    torch.cuda.synchronize()
    assert hyper[0].item() == 5.0
    assert (p.cpu() - tp.detach()).abs().max().item() < 2e-6


def test_bad_arguments_raise(dev):
    y = torch.empty(100, 256, device=dev)
    x = torch.empty(100, 256, device=dev)
    W = torch.empty(256, 256, device=dev)
    with pytest.raises(RuntimeError, match="multiple of 128"):
        _hip.linear_fwd(x, 256, None, 0, W, None, y, 100, 256, 1)
    with pytest.raises(RuntimeError, match="GPU"):
        _hip.linear_fwd(x.cpu(), 256, None, 0, W, None, y, 128, 256, 1)

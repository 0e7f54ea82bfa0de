"""Per-kernel parity of the nerf_hip C-ABI against fp64 CPU references (GPU only).

Tolerances: FP32 MFMA GEMMs are exact-f32 fma chains, so against an fp64 reference the
error is ~1e-7 * sqrt(K) * |a||b|; we require max |err| <= 2e-5 * scale (rel 2e-5).  The
GEMM tests run under every arithmetic mode (conftest.gemm_precision); the split-bf16 and
fp16-pair emulations must also be about as accurate as the exact-f32 MFMA
(test_split_accuracy)."""
import pytest
import torch

from model import _hip
from oracle import nerf_oracle as orc

pytestmark = pytest.mark.gpu


def _rand(*s, g=None):
    return torch.rand(*s, generator=g) * 2 - 1


def _rm(x):
    """Row max |x| (the A-operand row scales of precision mode 2), None in other modes."""
    if _hip.gemm_get_precision() != 2 or x is None:
        return None
    return x.abs().amax(1).contiguous()


def _cm(x):
    """Column max |x| per 128-row group ([m/128][cols], the dW column scales of mode 2)."""
    if _hip.gemm_get_precision() != 2 or x is None or x.shape[0] % 128:
        return None
    return x.abs().view(x.shape[0] // 128, 128, x.shape[1]).amax(1).contiguous()


def _images(W, dev):
    """W [n][k] (device) -> (split image of W, image of W^T) via nerf_pack_weights, in the
    form of the current precision mode (bf16x3, or the fp16 pair in mode 2)."""
    n, k = W.shape
    Wp, Wt = torch.zeros(n, k, device=dev), torch.zeros(k, n, device=dev)
    ws, wts = _hip.split_image(n, k, dev), _hip.split_image(k, n, dev)
    _hip.pack_weights([_hip.PackDesc(W.data_ptr(), Wp.data_ptr(), Wt.data_ptr(), n, k, k, k, n, ws.data_ptr(),
                                     wts.data_ptr())])
    return ws, wts


@pytest.mark.parametrize("m,n,k1,k2,relu", [(256, 256, 256, 0, 1), (384, 256, 64, 0, 1), (128, 256, 256, 64, 1),
                                            (256, 128, 256, 64, 1), (128, 64, 64, 0, 0), (512, 256, 256, 0, 0)])
def test_linear_fwd(dev, gemm_precision, m, n, k1, k2, relu):
    g = torch.Generator().manual_seed(m + n + k1 + k2)
    x1 = _rand(m, k1, g=g)
    x2 = _rand(m, k2, g=g) if k2 else None
    W = _rand(n, k1 + k2, g=g) * 0.1
    b = _rand(n, g=g)
    y = torch.empty(m, n, device=dev)
    mo = torch.empty(m, n // 32, device=dev, dtype=torch.int32)
    Wd = W.to(dev)
    ws = _images(Wd, dev)[0] if gemm_precision >= 1 else None
    x1d, x2d = x1.to(dev), (x2.to(dev) if x2 is not None else None)
    y_rm = torch.full((m,), -1.0, device=dev) if gemm_precision == 2 else None
    y_cm = torch.full((m // 128, n), -1.0, device=dev) if gemm_precision == 2 else None
    _hip.linear_fwd(x1d, k1, x2d, k2, Wd, b.to(dev), y, m, n, relu, mask_out=mo, w_split=ws, x1_rmax=_rm(x1d),
                    x2_rmax=_rm(x2d), y_rmax=y_rm, y_cmax=y_cm)
    xc = torch.cat([x1, x2], 1) if x2 is not None else x1
    ref = xc.double() @ W.double().t() + b.double()
    if relu:
        ref = ref.clamp_min(0)
    torch.cuda.synchronize()
    assert (y.cpu().double() - ref).abs().max().item() < 2e-5 * max(1.0, ref.abs().max().item())
    if y_rm is not None:                                              # exact row / column maxima of y
        assert torch.equal(y_rm, y.abs().amax(1))
        assert torch.equal(y_cm, y.abs().view(m // 128, 128, n).amax(1))
    bits = ((mo.cpu().long() & 0xffffffff).unsqueeze(-1) >> torch.arange(32)) & 1
    assert torch.equal(bits.view(m, n).bool(), y.cpu() > 0)          # ReLU bits agree with y


@pytest.mark.parametrize("nt_policy", [0, 1, 2])
@pytest.mark.parametrize("n,k1,k2,nh,col", [(256, 256, 0, 1, 0), (128, 256, 64, 3, 1)])
def test_linear_fwd_fused_heads(dev, n, k1, k2, nh, col, nt_policy):
    """nerf_linear_fwd_heads (precision mode 2): the layer output as nerf_linear_fwd's, plus
    raw4[:, col:col+nh] = relu(x W^T + b) head_w^T + head_b (the density head on the trunk,
    the colour head on the colour layer) vs fp64, the other raw4 columns untouched.  Under
    every NT tile policy: policy 1 would split a 256-wide output over two column blocks,
    whose partial head dots would overwrite each other; the heads launch keeps one block."""
    prev = _hip.gemm_get_precision()
    _hip.gemm_set_precision(2)
    _hip.gemm_set_policy(nt_policy, 0)
    try:
        m = 4096
        g = torch.Generator().manual_seed(n + nh)
        x1 = _rand(m, k1, g=g)
        x2 = _rand(m, k2, g=g) if k2 else None
        W = _rand(n, k1 + k2, g=g) * 0.1
        b = _rand(n, g=g)
        hw = _rand(nh, n, g=g)
        hb = _rand(nh, g=g)
        x1d, x2d = x1.to(dev), (x2.to(dev) if k2 else None)
        Wd = W.to(dev)
        ws = _images(Wd, dev)[0]
        y = torch.empty(m, n, device=dev)
        raw4 = torch.full((m, 4), 7.0, device=dev)
        _hip.linear_fwd(x1d, k1, x2d, k2, Wd, b.to(dev), y, m, n, True, w_split=ws, x1_rmax=_rm(x1d),
                        x2_rmax=_rm(x2d) if k2 else None, heads=(hw.to(dev).contiguous(), hb.to(dev), raw4, col))
        xx = torch.cat([x1, x2], 1) if k2 else x1
        ref_y = torch.relu(xx.double() @ W.double().t() + b.double())
        ref_h = ref_y @ hw.double().t() + hb.double()
        torch.cuda.synchronize()
        assert (y.cpu().double() - ref_y).abs().max().item() < 2e-5 * ref_y.abs().max().item()
        r = raw4.cpu().double()
        assert (r[:, col:col + nh] - ref_h).abs().max().item() < 2e-5 * ref_h.abs().max().item()
        others = [c for c in range(4) if not col <= c < col + nh]
        assert bool((r[:, others] == 7.0).all())
    finally:
        _hip.gemm_set_precision(prev)
        _hip.gemm_set_policy(0, 0)


def test_linear_fwd_asymmetric_identity(dev, gemm_precision):
    """A = I against an asymmetric B catches a transposed C write (guide section 3)."""
    m = n = k = 128
    x = torch.eye(m, k)
    W = torch.arange(n * k, dtype=torch.float32).view(n, k) / (n * k)
    y = torch.empty(m, n, device=dev)
    Wd = W.to(dev)
    ws = _images(Wd, dev)[0] if gemm_precision >= 1 else None
    xd = x.to(dev)
    _hip.linear_fwd(xd, k, None, 0, Wd, None, y, m, n, 0, w_split=ws, x1_rmax=_rm(xd))
    assert torch.equal(y.cpu(), W.t().contiguous())


def test_linear_bwd_data(dev, gemm_precision):
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
    Wtd = Wt.to(dev)
    ws = _images(Wtd, dev)[0] if gemm_precision >= 1 else None     # image of wt itself ([n][k])
    dyd = dy.to(dev)
    dx_rm = torch.full((m,), -1.0, device=dev) if gemm_precision == 2 else None
    dx_cm = torch.full((m // 128, n), -1.0, device=dev) if gemm_precision == 2 else None
    _hip.linear_bwd_data(dyd, k, Wtd, dx, m, n, mask=words.to(dev), u=u.to(dev), ldu=4, v=v.to(dev),
                         wt_split=ws, dy_rmax=_rm(dyd), dx_rmax=dx_rm, dx_cmax=dx_cm)
    ref = dy.double() @ Wt.double().t() + u[:, 0:1].double() * v.double()
    ref = torch.where(mask > 0, ref, torch.zeros_like(ref))
    torch.cuda.synchronize()
    assert (dx.cpu().double() - ref).abs().max().item() < 2e-5 * ref.abs().max().item()
    if dx_rm is not None:
        assert torch.equal(dx_rm, dx.abs().amax(1))
        assert torch.equal(dx_cm, dx.abs().view(m // 128, 128, n).amax(1))


@pytest.mark.parametrize("nout,kin,m,splits", [(256, 256, 4096, 8), (128, 320, 2048, 4), (256, 64, 1024, 1),
                                               (256, 320, 32768, 64), (128, 256, 12288, 48),
                                               (64, 128, 2048, 2)])
@pytest.mark.parametrize("tn_policy", [3, 7, 8])
def test_linear_bwd_weight_and_reduce(dev, gemm_precision, nout, kin, m, splits, tn_policy):
    """Weight gradient + slab reduce vs fp64; TN policies 7 and 8 (8 the default) run the
    256 x 256 cases (the 256-wide segment of the 320-wide one too) as XCD-paired 256 x 128
    column tiles and the 128-output ones with 256-wide segments as one 128 x 256 column tile
    (8: on the 4-wave kernels of wgrad.hip in mode 2)."""
    _hip.gemm_set_policy(0, tn_policy)
    try:
        _bwd_weight_case(dev, nout, kin, m, splits)
    finally:
        _hip.gemm_set_policy(0, 0)


def _bwd_weight_case(dev, nout, kin, m, splits):
    g = torch.Generator().manual_seed(nout + kin)
    dy = _rand(m, nout, g=g)
    x = _rand(m, kin, g=g)
    k_main = kin - 64 if (kin % 128 and kin > 64) else kin
    slab = torch.empty(splits * nout * kin, device=dev)
    bslab = torch.empty(splits * nout, device=dev)
    dyd, xd = dy.to(dev), x.to(dev)
    x1, x2 = xd[:, :k_main].contiguous(), xd[:, k_main:].contiguous()
    _hip.linear_bwd_weight(dyd, nout, x1, k_main, m, splits, slab, kin, 0, bslab, dy_cmax=_cm(dyd),
                           x_cmax=_cm(x1))
    if k_main < kin:
        _hip.linear_bwd_weight(dyd, nout, x2, kin - k_main, m, splits, slab, kin, k_main, None,
                               dy_cmax=_cm(dyd), x_cmax=_cm(x2))
    kin_ref = kin - 1
    gw = torch.empty(nout, kin_ref, device=dev)
    gb = torch.empty(nout, device=dev)
    _hip.slab_reduce(slab, splits, nout, kin, nout, kin_ref, bslab, gw, gb)
    ref = dy.double().t() @ x.double()
    torch.cuda.synchronize()
    scale = ref.abs().max().item()
    assert (gw.cpu().double() - ref[:, :kin_ref]).abs().max().item() < 2e-5 * scale
    assert (gb.cpu().double() - dy.double().sum(0)).abs().max().item() < 1e-4 * max(1, dy.abs().sum(0).max().item())


@pytest.mark.parametrize("nout,m,splits", [(256, 131072, 128), (128, 131072, 256), (256, 8192, 16), (128, 4096, 8),
                                           (256, 4096, 4)])
def test_linear_bwd_weight_seg(dev, gemm_precision, nout, m, splits):
    """The two-segment weight gradient (l4's [h3 | enc_p], the colour layer's [f | enc_d]):
    one launch in mode 2 (TN policy 7, splits % 8 == 0), two otherwise -- bit-identical to
    the two nerf_linear_bwd_weight calls it replaces (the same tiles, splits and k order),
    and within 2e-5 of fp64 after the slab reduce; (256, 4096, 4) takes the two-call path."""
    g = torch.Generator().manual_seed(nout + splits)
    k1, k2 = 256, 64
    dy = _rand(m, nout, g=g).to(dev)
    x1 = _rand(m, k1, g=g).to(dev)
    x2 = _rand(m, k2, g=g).to(dev)
    slab_a = torch.full((splits * nout * (k1 + k2),), float("nan"), device=dev)
    slab_b = torch.full_like(slab_a, float("nan"))
    bslab_a = torch.full((splits * nout,), float("nan"), device=dev)
    bslab_b = torch.full_like(bslab_a, float("nan"))
    _hip.linear_bwd_weight_seg(dy, nout, x1, k1, x2, k2, m, splits, slab_a, k1 + k2, bslab_a, dy_cmax=_cm(dy),
                               x1_cmax=_cm(x1), x2_cmax=_cm(x2))
    _hip.linear_bwd_weight(dy, nout, x1, k1, m, splits, slab_b, k1 + k2, 0, bslab_b, dy_cmax=_cm(dy), x_cmax=_cm(x1))
    _hip.linear_bwd_weight(dy, nout, x2, k2, m, splits, slab_b, k1 + k2, k1, None, dy_cmax=_cm(dy), x_cmax=_cm(x2))
    torch.cuda.synchronize()
    assert torch.equal(slab_a, slab_b)
    assert torch.equal(bslab_a, bslab_b)
    gw = torch.empty(nout, k1 + k2, device=dev)
    gb = torch.empty(nout, device=dev)
    _hip.slab_reduce(slab_a, splits, nout, k1 + k2, nout, k1 + k2, bslab_a, gw, gb)
    ref = dy.double().t() @ torch.cat([x1, x2], 1).double()
    torch.cuda.synchronize()
    assert (gw.double() - ref).abs().max().item() < 2e-5 * ref.abs().max().item()
    assert (gb.double() - dy.double().sum(0)).abs().max().item() < 1e-4 * max(1, dy.abs().sum(0).max().item())


@pytest.mark.parametrize("nout,kin,m,splits", [(256, 256, 131072, 128), (256, 64, 131072, 256),
                                               (128, 256, 131072, 256), (128, 64, 131072, 256),
                                               (256, 256, 4096, 8), (128, 256, 3072, 8), (256, 64, 1024, 8)])
def test_wgrad_4wave_matches_8wave(dev, nout, kin, m, splits):
    """The 4-wave weight-gradient kernels (TN policy 8, wgrad.hip) against the 8-wave ones
    (policy 7) on the same operands, mode 2: the same column scales, fp16 pairs, products and
    16-row k-step order, so every slab entry is bit-identical; the bias partials (a different
    summation order of the same dy columns) within f32 rounding.  Covers the training shapes
    (131 072 rows) and short splits (96-384 rows: the 3-stage pipeline's tail)."""
    prev = _hip.gemm_get_precision()
    _hip.gemm_set_precision(2)
    g = torch.Generator().manual_seed(nout * 7 + kin)
    dy = _rand(m, nout, g=g).to(dev)
    x = _rand(m, kin, g=g).to(dev)
    dy[:, 3] *= 1e-6                       # columns of very different magnitude: the per-column scales
    x[:, 5] *= 1e5
    out = {}
    for pol in (7, 8):
        _hip.gemm_set_policy(0, pol)
        try:
            slab = torch.full((splits * nout * kin,), float("nan"), device=dev)
            bslab = torch.full((splits * nout,), float("nan"), device=dev)
            _hip.linear_bwd_weight(dy, nout, x, kin, m, splits, slab, kin, 0, bslab, dy_cmax=_cm(dy), x_cmax=_cm(x))
            torch.cuda.synchronize()
            out[pol] = (slab, bslab)
        finally:
            _hip.gemm_set_policy(0, 0)
    _hip.gemm_set_precision(prev)
    assert torch.equal(out[7][0], out[8][0])
    b7, b8 = out[7][1].view(splits, nout).double(), out[8][1].view(splits, nout).double()
    ref = dy.double().view(splits, m // splits, nout).sum(1)
    assert (b8 - ref).abs().max().item() <= 2 * (b7 - ref).abs().max().item() + 1e-6 * ref.abs().max().item()


@pytest.mark.parametrize("n,m,splits", [(8, 32768, 32), (4, 131072, 128), (3, 131072, 128), (2, 4096, 8),
                                          (1, 131072, 128)])
def test_wgrad_multi_matches_single(dev, n, m, splits):
    """nerf_linear_bwd_weight_multi (k_wgrad_pairs: a block walks n layers, the exponent sets
    alternating, a layer's first loads beside the previous layer's slab stores) against one
    nerf_linear_bwd_weight per layer: every slab and bias partial bit-identical."""
    prev = _hip.gemm_get_precision()
    _hip.gemm_set_precision(2)
    try:
        g = torch.Generator().manual_seed(n * 31 + m)
        layers, want = [], []
        for i in range(n):
            dy = _rand(m, 256, g=g).to(dev)
            x = _rand(m, 256, g=g).clamp_min(0).to(dev)
            dy[:, i] *= 1e-5
            slab = torch.full((splits * 256 * 256,), float("nan"), device=dev)
            bslab = torch.full((splits * 256,), float("nan"), device=dev)
            layers.append((dy, x, slab, bslab, _cm(dy), _cm(x)))
            s1, b1 = torch.full_like(slab, float("nan")), torch.full_like(bslab, float("nan"))
            _hip.linear_bwd_weight(dy, 256, x, 256, m, splits, s1, 256, 0, b1, dy_cmax=_cm(dy), x_cmax=_cm(x))
            want.append((s1, b1))
        _hip.linear_bwd_weight_multi(layers, m, splits)
        torch.cuda.synchronize()
        for (dy, x, slab, bslab, _, _), (s1, b1) in zip(layers, want):
            assert torch.equal(slab, s1)
            assert torch.equal(bslab, b1)
    finally:
        _hip.gemm_set_precision(prev)


@pytest.mark.parametrize("which,m,S,grouped", [("colour+trunk", 131072, 128, False), ("l4+trunk+l0", 131072, 128, False),
                                                ("colour+trunk", 32768, 32, False), ("l4+trunk+l0", 32768, 32, False),
                                                ("l4+trunk+l0", 131072, 64, True), ("l4+trunk+l0", 32768, 16, True)])
def test_wgrad_jobs_matches_single(dev, which, m, S, grouped):
    """nerf_linear_bwd_weight_jobs (k_wgrad_jobs: 2 S blocks walk tiles of four shapes -- the
    TN schedule 3 launches of the field backward) against one nerf_linear_bwd_weight per job
    with the same splits and slab columns: every slab and bias partial bit-identical."""
    prev = _hip.gemm_get_precision()
    _hip.gemm_set_precision(2)
    try:
        g = torch.Generator().manual_seed(m + len(which))
        jobs = []

        def layer(nout, kin, sp, x2=None, sp2=None, bias=True):
            dy = _rand(m, nout, g=g).to(dev)
            x = _rand(m, kin, g=g).clamp_min(0).to(dev)
            dy[:, 3] *= 1e-5
            ld = kin + (64 if x2 is not None else 0)
            slab = torch.full((sp * nout * ld,), float("nan"), device=dev)
            bslab = torch.full((sp * nout,), float("nan"), device=dev) if bias else None
            jobs.append((dy, nout, x, kin, sp, slab, ld, 0, bslab, _cm(dy), _cm(x)))
            if x2 is not None:
                e = _rand(m, 64, g=g).to(dev)
                jobs.append((dy, nout, e, 64, sp, slab, ld, kin, None, _cm(dy), _cm(e)))

        if which == "colour+trunk":
            layer(128, 256, 2 * S, x2=True)          # the colour layer over [f | enc_d]
            for _ in range(4):
                layer(256, 256, S)                   # l_f .. l5
        else:
            layer(256, 256, S, x2=True)              # l4 over [h3 | enc_p]: the enc_p tile per output half
            for _ in range(3):
                layer(256, 256, S)                   # l3 .. l1
            layer(256, 64, 2 * S)                    # l0 over enc_p
        want = []
        for dy, nout, x, kin, sp, slab, ld, col0, bslab, dcm, xcm in jobs:
            if col0 == 0:
                want.append((torch.full_like(slab, float("nan")),
                             None if bslab is None else torch.full_like(bslab, float("nan"))))
            s1, b1 = want[-1]
            _hip.linear_bwd_weight(dy, nout, x, kin, m, sp, s1, ld, col0, b1 if col0 == 0 else None,
                                   dy_cmax=dcm, x_cmax=xcm)
        if grouped:
            # TN schedule 3's second launch in two block groups (field_bwd.cpp): l4 (both
            # segments) + l3 | l2 + l1 + l0, each group at S splits on its own 2 S blocks
            grp = [0, 0, 0, 1, 1, 1]
            _hip.linear_bwd_weight_jobs(jobs, m, S, groups=grp)
        else:
            _hip.linear_bwd_weight_jobs(jobs, m, S)
        torch.cuda.synchronize()
        got = [(slab, bslab) for (_, _, _, _, _, slab, _, col0, bslab, _, _) in jobs if col0 == 0]
        assert len(got) == len(want)
        for (slab, bslab), (s1, b1) in zip(got, want):
            assert torch.equal(slab, s1)
            assert (bslab is None and b1 is None) or torch.equal(bslab, b1)
    finally:
        _hip.gemm_set_precision(prev)


def test_slab_reduce_accumulate(dev):
    """nerf_slab_reduce with accumulate=1 adds onto the existing gradient (train.py's
    gradient accumulation across render calls); split sums in a fixed order."""
    g = torch.Generator().manual_seed(9)
    splits, nout, ld, kin_ref = 37, 64, 136, 130
    slab = _rand(splits * nout * ld, g=g).to(dev)
    bslab = _rand(splits * nout, g=g).to(dev)
    gw0 = _rand(nout, kin_ref, g=g).to(dev)
    gb0 = _rand(nout, g=g).to(dev)
    gw, gb = gw0.clone(), gb0.clone()
    _hip.slab_reduce(slab, splits, nout, ld, nout, kin_ref, bslab, gw, gb, accumulate=True)
    gw2, gb2 = torch.empty_like(gw), torch.empty_like(gb)
    _hip.slab_reduce(slab, splits, nout, ld, nout, kin_ref, bslab, gw2, gb2)
    _hip.slab_reduce(slab, splits, nout, ld, nout, kin_ref, bslab, gw2, gb2, accumulate=True)
    torch.cuda.synchronize()
    ref = slab.view(splits, nout, ld)[:, :, :kin_ref].double().sum(0)
    assert (gw.double() - gw0.double() - ref).abs().max().item() < 1e-4
    assert (gb.double() - gb0.double() - bslab.view(splits, nout).double().sum(0)).abs().max().item() < 1e-4
    assert torch.equal(gw2, 2 * (gw2 / 2))      # finite
    assert torch.allclose(gw2, 2 * (gw - gw0), atol=1e-4)


@pytest.mark.parametrize("scale_a,scale_b,spread",[(1.0, 0.1, 0), (1e-3, 1e3, 0), (1e-20, 1.0, 0), (1.0, 0.1, 8),
                                                    (1e-7, 1.0, 12), (1e4, 1e-6, 0)])
def test_split_accuracy(dev, scale_a, scale_b, spread):
    """The split-bf16 GEMM (mode 1) and the fp16-pair GEMM (mode 2) against fp64: their
    errors must stay within 1.5x (+ a few ulps) of the exact-f32 MFMA's on the same operands,
    over K = 320 (two segments), including operands far from 1 (bf16 words share f32's
    exponent range; the fp16 pair carries per-row power-of-two scales) and rows whose
    magnitudes differ by up to 2^spread (row-scale independence)."""
    g = torch.Generator().manual_seed(11)
    m, n, k1, k2 = 512, 256, 256, 64
    rs = 2.0 ** (torch.randint(-spread, spread + 1, (m, 1), generator=g).float()) if spread else 1.0
    x1, x2 = _rand(m, k1, g=g) * scale_a * rs, _rand(m, k2, g=g) * scale_a * rs
    W = _rand(n, k1 + k2, g=g) * scale_b
    ref = torch.cat([x1, x2], 1).double() @ W.double().t()
    errs = []
    Wd = W.to(dev)
    x1d, x2d = x1.to(dev), x2.to(dev)
    for mode in (0, 1, 2):
        _hip.gemm_set_precision(mode)
        try:
            ws = _images(Wd, dev)[0]
            y = torch.empty(m, n, device=dev)
            _hip.linear_fwd(x1d, k1, x2d, k2, Wd, None, y, m, n, 0, w_split=ws, x1_rmax=_rm(x1d), x2_rmax=_rm(x2d))
            torch.cuda.synchronize()
        finally:
            _hip.gemm_set_precision(0)
        # per-row error relative to the row's scale (rows differ by 2^spread)
        rowscale = ref.abs().amax(1, keepdim=True).clamp_min(1e-300)
        errs.append(((y.cpu().double() - ref).abs() / rowscale).max().item())
    tiny = 4 * 2.0 ** -24
    assert errs[1] <= 1.5 * errs[0] + tiny, errs
    assert errs[2] <= 1.5 * errs[0] + tiny, errs


@pytest.mark.parametrize("spread", [0, 10])
def test_split_accuracy_weight_gradient(dev, spread):
    """Weight-gradient GEMM (sum over 32768 samples in 64 splits) in every mode against fp64:
    the fp16 pair kernel (column scales per split) within 1.5x (+ulps) of the exact-f32 MFMA,
    also with columns whose magnitudes differ by up to 2^spread."""
    g = torch.Generator().manual_seed(21)
    m, nout, kin, splits = 32768, 256, 256, 64
    cs = 2.0 ** torch.randint(-spread, spread + 1, (1, nout), generator=g).float() if spread else 1.0
    dy = _rand(m, nout, g=g) * cs
    x = _rand(m, kin, g=g)
    ref = dy.double().t() @ x.double()
    rowscale = (dy.double().abs().t() @ x.double().abs()).amax(1, keepdim=True)
    dyd, xd = dy.to(dev), x.to(dev)
    errs = []
    for mode in (0, 1, 2):
        _hip.gemm_set_precision(mode)
        try:
            slab = torch.empty(splits * nout * kin, device=dev)
            gw = torch.empty(nout, kin, device=dev)
            _hip.linear_bwd_weight(dyd, nout, xd, kin, m, splits, slab, kin, 0, None, dy_cmax=_cm(dyd),
                                   x_cmax=_cm(xd))
            _hip.slab_reduce(slab, splits, nout, kin, nout, kin, None, gw, None)
            torch.cuda.synchronize()
        finally:
            _hip.gemm_set_precision(0)
        errs.append(((gw.cpu().double() - ref).abs() / rowscale).max().item())
    tiny = 4 * 2.0 ** -24
    assert errs[1] <= 1.5 * errs[0] + tiny, errs
    assert errs[2] <= 1.5 * errs[0] + tiny, errs


def _split3_ref(x):
    """x -> (hi, mid, lo) bf16 words, each round-to-nearest-even (torch .bfloat16())."""
    h = x.bfloat16()
    r = x - h.float()
    m = r.bfloat16()
    lo = (r - m.float()).bfloat16()
    return [t.view(torch.int16) for t in (h, m, lo)]


def _image_ref(mat):
    """[N][K] f32 -> bf16x3 image [3][K/8][N][8] (nerf_pack_desc.dst_s layout)."""
    N, K = mat.shape
    return torch.stack([p.view(N, K // 8, 8).permute(1, 0, 2) for p in _split3_ref(mat)])


def test_pack_split_images(dev):
    """nerf_pack_weights dst_s / dst_ts are the exact bf16x3 images of the padded packed
    weight and its transpose; hi + mid + lo reconstructs every f32 exactly."""
    g = torch.Generator().manual_seed(5)
    rows, cols, ld, rows_t, ld_t, rows_s = 200, 300, 320, 320, 256, 256   # rows padded 200 -> 256 in the image
    W = (_rand(rows, cols, g=g) * torch.logspace(-6, 2, cols)).to(dev)
    dst = torch.zeros(rows, ld, device=dev)
    dst_t = torch.zeros(rows_t, ld_t, device=dev)
    ws = _hip.split_image(rows_s, ld, dev) - 1        # poisoned: every element must be written
    wts = _hip.split_image(rows_t, ld_t, dev) - 1
    _hip.gemm_set_precision(1)                        # the bf16x3 form (mode 2 writes the fp16 pair)
    _hip.pack_weights([_hip.PackDesc(W.data_ptr(), dst.data_ptr(), dst_t.data_ptr(), rows, cols, ld, rows_t, ld_t,
                                     ws.data_ptr(), wts.data_ptr(), rows_s)])
    torch.cuda.synchronize()
    assert torch.equal(ws.cpu(), _image_ref(torch.cat([dst.cpu(), torch.zeros(rows_s - rows, ld)])))
    assert torch.equal(wts.cpu(), _image_ref(dst_t.cpu()))
    h, m, lo = (ws.cpu()[p].permute(1, 0, 2).reshape(rows_s, ld)[:rows].view(torch.bfloat16).double()
                for p in range(3))
    assert torch.equal((h + m + lo).float(), dst.cpu())


def test_pack_f16_pair_images(dev):
    """Mode 2 images: per row r an exponent e_r with max|row| 2^e_r in [2^14, 2^15), fp16
    hi / lo planes with hi = fp16(x 2^e_r) and lo = fp16(x 2^e_r - hi) (RNE), so that
    (hi + lo) 2^-e_r is x to 2^-22 of the row max; zero rows get e = 0."""
    g = torch.Generator().manual_seed(6)
    rows, cols, ld, rows_t, ld_t, rows_s = 200, 300, 320, 320, 256, 256
    W = (_rand(rows, cols, g=g) * torch.logspace(-6, 2, rows).unsqueeze(1)).to(dev)
    dst = torch.zeros(rows, ld, device=dev)
    dst_t = torch.zeros(rows_t, ld_t, device=dev)
    ws = _hip.split_image(rows_s, ld, dev) - 1
    wts = _hip.split_image(rows_t, ld_t, dev) - 1
    _hip.gemm_set_precision(2)
    try:
        _hip.pack_weights([_hip.PackDesc(W.data_ptr(), dst.data_ptr(), dst_t.data_ptr(), rows, cols, ld, rows_t,
                                         ld_t, ws.data_ptr(), wts.data_ptr(), rows_s)])
        torch.cuda.synchronize()
    finally:
        _hip.gemm_set_precision(0)
    for img, mat in ((ws.cpu(), torch.cat([dst.cpu(), torch.zeros(rows_s - rows, ld)])), (wts.cpu(), dst_t.cpu())):
        N, K = mat.shape
        e = img[2, 0, :, 0:2].contiguous().view(torch.int32).view(N).long()
        rmax = mat.abs().amax(1)
        e_ref = torch.where(rmax > 0, 14 - torch.floor(torch.log2(rmax.double().clamp_min(1e-300))).long(),
                            torch.zeros_like(e))
        assert torch.equal(e, e_ref)
        xs = mat.double() * torch.pow(2.0, e.double()).unsqueeze(1)
        h = img[0].permute(1, 0, 2).reshape(N, K).view(torch.float16)
        lo = img[1].permute(1, 0, 2).reshape(N, K).view(torch.float16)
        assert torch.equal(h, xs.float().half())
        assert torch.equal(lo, (xs.float() - h.float()).half())
        rec = (h.double() + lo.double()) * torch.pow(2.0, -e.double()).unsqueeze(1)
        assert ((rec - mat.double()).abs() <= 2.0 ** -22 * rmax.double().unsqueeze(1) + 1e-45).all()


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("m,n,k1,k2", [(256, 256, 256, 64), (128, 64, 64, 0), (384, 128, 256, 0), (512, 256, 64, 64)])
def test_split_weight_operand(dev, mode, m, n, k1, k2):
    """Modes 1 / 2 with the pre-split weight images: forward (two K segments) and
    backward-data through a row slice of the transposed image, against fp64."""
    g = torch.Generator().manual_seed(m + k2)
    x1 = _rand(m, k1, g=g).to(dev)
    x2 = _rand(m, k2, g=g).to(dev) if k2 else None
    W = (_rand(n, k1 + k2, g=g) * 0.1).to(dev)
    b = _rand(n, g=g).to(dev)
    Wt = W.t().contiguous()
    dy = torch.rand(m, n, device=dev) - 0.5
    lo, hi = (k1, k1 + k2) if k2 else (0, k1)
    _hip.gemm_set_precision(mode)
    try:
        ws, wts = _images(W, dev)
        y = torch.empty(m, n, device=dev)
        _hip.linear_fwd(x1, k1, x2, k2, W, b, y, m, n, 1, w_split=ws, x1_rmax=_rm(x1), x2_rmax=_rm(x2))
        d = torch.empty(m, hi - lo, device=dev)
        _hip.linear_bwd_data(dy, n, Wt[lo:hi], d, m, hi - lo, wt_split=wts[:, :, lo:hi], dy_rmax=_rm(dy))
        torch.cuda.synchronize()
    finally:
        _hip.gemm_set_precision(0)
    xc = torch.cat([x1, x2], 1) if x2 is not None else x1
    ref = (xc.double() @ W.double().t() + b.double()).clamp_min(0)
    assert (y.double() - ref).abs().max().item() < 2e-5 * ref.abs().max().item()
    refd = dy.double() @ Wt[lo:hi].double().t()
    assert (d.double() - refd).abs().max().item() < 2e-5 * refd.abs().max().item()


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
    dyr_rm = torch.full((Np,), -1.0, device=dev)
    dyr_cm = torch.full((Np // 128, HR), -1.0, device=dev)
    _hip.heads_bwd(graw.to(dev), h8.to(dev), hr.to(dev), hidden, wc.to(dev), dyr, part, Np, dyr_rmax=dyr_rm,
                   dyr_cmax=dyr_cm)
    gwd, gbd = torch.empty(hidden, device=dev), torch.empty(1, device=dev)
    gwc, gbc = torch.empty(3, HR, device=dev), torch.empty(3, device=dev)
    _hip.heads_reduce(part, hidden, Np, gwd, gbd, gwc, gbc)
    G = graw.double()
    r_dyr = torch.where(hr > 0, G[:, 1:] @ wc.double(), torch.zeros(Np, HR, dtype=torch.float64))
    torch.cuda.synchronize()
    assert (dyr.cpu().double() - r_dyr).abs().max().item() < 1e-5 * max(1, r_dyr.abs().max().item())
    assert torch.equal(dyr_rm, dyr.abs().amax(1))                    # row scales of precision mode 2
    assert torch.equal(dyr_cm, dyr.abs().view(Np // 128, 128, HR).amax(1))   # its column scales
    assert (gwd.cpu().double() - G[:, 0] @ h8.double()).abs().max().item() < 1e-4 * Np
    assert (gwc.cpu().double() - G[:, 1:].t() @ hr.double()).abs().max().item() < 1e-4 * Np
    assert (gbd.cpu().double() - G[:, 0].sum()).abs().item() < 1e-3
    assert (gbc.cpu().double() - G[:, 1:].sum(0)).abs().max().item() < 1e-3
    # the split form the training backward uses (mode 1: dyr + maxima, mode 2: head-weight
    # partials, h8 / dyr not passed where unused) reproduces mode 3 bit for bit
    dyr1 = torch.full_like(dyr, 7.0)
    rm1, cm1 = torch.full_like(dyr_rm, -1.0), torch.full_like(dyr_cm, -1.0)
    _hip.heads_bwd(graw.to(dev), None, hr.to(dev), hidden, wc.to(dev), dyr1, None, Np, dyr_rmax=rm1, dyr_cmax=cm1,
                   mode=1)
    part2 = torch.full_like(part, 3.0)
    _hip.heads_bwd(graw.to(dev), h8.to(dev), hr.to(dev), hidden, wc.to(dev), None, part2, Np, mode=2)
    torch.cuda.synchronize()
    assert torch.equal(dyr1, dyr) and torch.equal(rm1, dyr_rm) and torch.equal(cm1, dyr_cm)
    assert torch.equal(part2, part)
    # mode 1 gated by the colour layer's ReLU bits (bit = hr > 0, the forward's mask_out layout)
    hb = (hr > 0).to(torch.int64).view(Np, HR // 32, 32) << torch.arange(32)
    bits = hb.sum(-1).to(torch.int64)
    bits = torch.where(bits >= 2 ** 31, bits - 2 ** 32, bits).to(torch.int32)
    dyr3 = torch.full_like(dyr, 7.0)
    rm3, cm3 = torch.full_like(dyr_rm, -1.0), torch.full_like(dyr_cm, -1.0)
    _hip.heads_bwd(graw.to(dev), None, None, hidden, wc.to(dev), dyr3, None, Np, dyr_rmax=rm3, dyr_cmax=cm3, mode=1,
                   hr_mask=bits.to(dev))
    torch.cuda.synchronize()
    assert torch.equal(dyr3, dyr) and torch.equal(rm3, dyr_rm) and torch.equal(cm3, dyr_cm)


@pytest.mark.parametrize("R,S", [(33, 64), (7, 200), (29, 48)])
def test_encode_samples(dev, R, S):
    """Samples / encodings vs the oracle; S = 200 and 48 put ray boundaries inside the
    128-row blocks (the view-direction encoding is computed once per ray of a block)."""
    g = torch.Generator().manual_seed(7)
    o = _rand(R, 3, g=g) * 3
    d = torch.nn.functional.normalize(_rand(R, 3, g=g), dim=-1)
    view = -d
    noise = torch.rand(R, S, generator=g)
    Np = ((R * S + 127) // 128) * 128
    z = torch.empty(Np, device=dev)
    ep = torch.empty(Np, 64, device=dev)
    ed = torch.empty(Np, 64, device=dev)
    rp, rd = torch.full((Np,), -1.0, device=dev), torch.full((Np,), -1.0, device=dev)
    cp, cd = torch.full((Np // 128, 64), -1.0, device=dev), torch.full((Np // 128, 64), -1.0, device=dev)
    _hip.encode_samples(o.to(dev), d.to(dev), view.to(dev), noise.to(dev), R, S, Np, 0.01, 10.0, z, ep, ed,
                        enc_p_rmax=rp, enc_d_rmax=rd, enc_p_cmax=cp, enc_d_cmax=cd)
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
    if Np > R * S:
        assert ep.cpu()[R * S:].abs().max().item() == 0 and ed.cpu()[R * S:].abs().max().item() == 0
    assert torch.equal(rp, ep.abs().amax(1)) and torch.equal(rd, ed.abs().amax(1))
    # column bounds per 128-row group: exact on the coordinates, >= the sin / cos maxima, 0 on the pad
    for c, e in ((cp, ep), (cd, ed)):
        ex = e.abs().view(Np // 128, 128, 64).amax(1)
        assert torch.equal(c[:, :3], ex[:, :3]) and (c >= ex).all()
    assert (cp[:, 3:63] == 1).all() and (cp[:, 63] == 0).all()
    assert (cd[:, 3:27] == 1).all() and (cd[:, 27:] == 0).all()


@pytest.mark.parametrize("with_p2", [False, True])
def test_encode_bwd_matches_autograd(dev, with_p2):
    """nerf_encode_bwd (gradient of the encodings back to ray origin, direction and view) vs
    fp64 autograd of the oracle's encode_position at the same sample points."""
    R, S = 37, 128
    g = torch.Generator().manual_seed(17)
    o = _rand(R, 3, g=g) * 3
    d = torch.nn.functional.normalize(_rand(R, 3, g=g), dim=-1)
    view = -d
    z = 0.01 + 9.99 * torch.rand(R, S, generator=g)
    Np = ((R * S + 127) // 128) * 128
    gp = torch.zeros(Np, 64)
    gp[:R * S, :63] = _rand(R * S, 63, g=g)
    gp2 = torch.zeros(Np, 64)
    gp2[:R * S, :63] = _rand(R * S, 63, g=g)
    gd = torch.zeros(Np, 64)
    gd[:R * S, :27] = _rand(R * S, 27, g=g)
    outs = [torch.empty(R, 3, device=dev) for _ in range(3)]
    zd = torch.zeros(Np)
    zd[:R * S] = z.reshape(-1)
    _hip.encode_bwd(o.to(dev), d.to(dev), view.to(dev), zd.to(dev), gp.to(dev), gd.to(dev), R, S, *outs,
                    genc_p2=gp2.to(dev) if with_p2 else None)
    # the sample points as the kernel forms them (f32 o + d z), differentiated in fp64 there:
    # at 2^9 the encoding's phase amplifies a 1-ulp point difference ~500x
    pts32 = (o.unsqueeze(1) + d.unsqueeze(1) * z.unsqueeze(-1)).reshape(-1, 3)
    p64 = pts32.double().clone().requires_grad_(True)
    v64 = view.double().clone().requires_grad_(True)
    gsum = gp[:R * S, :63] + (gp2[:R * S, :63] if with_p2 else 0)
    loss = (orc.encode_position(p64, 10) * gsum.double()).sum()
    loss = loss + (orc.encode_position(v64.unsqueeze(1).expand(R, S, 3).reshape(-1, 3), 4)
                   * gd[:R * S, :27].double()).sum()
    loss.backward()
    gpt = p64.grad.view(R, S, 3)
    refs = (gpt.sum(1), (gpt * z.double().unsqueeze(-1)).sum(1), v64.grad)
    for h, r in zip(outs, refs):
        err = ((h.cpu().double() - r).abs().max() / r.abs().max()).item()
        assert err < 2e-5, err


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
    from model.optim import hyper_block
    hyper = hyper_block(1e-3, 0.9, 0.999, 1e-8, 0.0).to(dev)
    tp = torch.nn.Parameter(p0.clone().to(dev))
    opt = torch.optim.Adam([tp], lr=1e-3)
    for step in range(1, 6):
        gr = torch.randn(10007, generator=g).to(dev)
        tp.grad = gr.clone()
        opt.step()
        _hip.adam_step(p, gr, m, v, hyper)
    torch.cuda.synchronize()
    assert hyper[0].item() == 5.0
    # torch's GPU Adam (the foreach path) op for op: bit-equal parameters and moments
    st = opt.state[tp]
    assert torch.equal(p, tp.detach()), (p - tp.detach()).abs().max().item()
    assert torch.equal(m, st["exp_avg"]) and torch.equal(v, st["exp_avg_sq"])


def test_bad_arguments_raise(dev):
    y = torch.empty(100, 256, device=dev)
    x = torch.empty(100, 256, device=dev)
    W = torch.empty(256, 256, device=dev)
    with pytest.raises(RuntimeError, match="multiple of 128"):
        _hip.linear_fwd(x, 256, None, 0, W, None, y, 100, 256, 1)
    with pytest.raises(RuntimeError, match="GPU"):
        _hip.linear_fwd(x.cpu(), 256, None, 0, W, None, y, 128, 256, 1)

"""End-to-end parity of the HIP render path and training step against the oracle
(GPU only).  Bar (BASELINE.json north_star): rendered RGB / depth within 1e-4 relative
of the fp32 CPU restatement on identical inputs (same weights, rays, stratified noise)."""
import pytest
import torch

from model.official_nerf import OfficialStaticNerf
from model.rendering import Renderer
from oracle import nerf_oracle as orc
from tests.helpers import assert_elementwise, make_cfg, report_err, synthetic_rays

pytestmark = pytest.mark.gpu

RTOL = 1e-4


def _pair(cfg, seed=0):
    torch.manual_seed(seed)
    net = OfficialStaticNerf(cfg)
    r = cfg["rendering"]
    ref = orc.OracleNerf(hidden_dim=cfg["model"]["hidden_dim"], white_background=r["white_background"],
                         dist_alpha=r["dist_alpha"], occ_activation=cfg["model"]["occ_activation"])
    ref.load_state_dict(net.state_dict())
    return net, ref


def _rel(a, b):
    """max-normalised error (diagnostic; the bar is assert_elementwise)."""
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


@pytest.mark.parametrize("hidden,S,R,opts", [
    (256, 128, 1024, {}),                                   # config 2 shape
    (64, 64, 256, {}),                                      # config 1 shape
    (256, 128, 200, {"white_background": True}),
    (128, 96, 300, {"dist_alpha": True}),
    (128, 64, 256, {"sample_option": "ndc", "dist_alpha": True}),   # LLFF (configs/LLFF/fern.yaml:6-8)
    (64, 32, 128, {"use_ray_dir": False, "normalise_ray": False}),
    (64, 32, 128, {"occ_activation": "relu"}),
])
def test_render_forward_matches_oracle(dev, gemm_precision, hidden, S, R, opts):
    opts = dict(opts)
    occ = opts.pop("occ_activation", None)
    cfg = make_cfg(hidden=hidden, S=S, **opts)
    if occ is not None:
        cfg["model"]["occ_activation"] = occ
    net, ref = _pair(cfg)
    b = synthetic_rays(R=R, S=S, seed=hidden + S)
    rnd = Renderer(net.to(dev), cfg["rendering"], device=dev)
    with torch.no_grad():
        out = rnd.nope_nerf(b["pixels"].to(dev), b["depth"].to(dev), b["K"].to(dev), b["w2c"].to(dev),
                            b["scale"].to(dev), add_noise=True, noise=b["noise"].to(dev))
        o = orc.render_nope_nerf(ref, b["pixels"], b["depth"], b["K"], b["w2c"], b["scale"], cfg["rendering"],
                                 noise=b["noise"])
    assert_elementwise(out["rgb"], o["rgb"], what="rgb")
    assert_elementwise(out["depth_pred"], o["depth_pred"], what="depth")
    assert torch.equal(out["depth_gt"].cpu(), o["depth_gt"]) or _rel(out["depth_gt"].cpu(), o["depth_gt"]) < 1e-6
    assert (out["alpha"].cpu() - o["alpha"]).abs().max().item() < 1e-4
    assert _rel(out["z_vals"].cpu(), o["z_vals"]) < 1e-6


def test_render_eval_mode_full_frame_tile(dev, gemm_precision):
    """eval_=True (render/extraction path): no noise, depth normalised to z-depth."""
    cfg = make_cfg(hidden=256, S=128)
    net, ref = _pair(cfg, 3)
    b = synthetic_rays(R=2048, S=128, seed=9, zero_frac=0.0)
    rnd = Renderer(net.to(dev), cfg["rendering"], device=dev)
    with torch.no_grad():
        out = rnd.nope_nerf(b["pixels"].to(dev), torch.ones(1, 2048, 1, device=dev), b["K"].to(dev),
                            b["w2c"].to(dev), b["scale"].to(dev), add_noise=False, eval_=True)
        o = orc.render_nope_nerf(ref, b["pixels"], torch.ones(1, 2048, 1), b["K"], b["w2c"], b["scale"],
                                 cfg["rendering"], noise=None, eval_=True)
    assert_elementwise(out["rgb"], o["rgb"], what="rgb")
    assert_elementwise(out["depth_pred"], o["depth_pred"], what="depth")


def test_render_backward_matches_oracle(dev, gemm_precision):
    """parameter gradients of rgb-L2 + depth-L1 through the fused backward."""
    cfg = make_cfg(hidden=256, S=128)
    net, ref = _pair(cfg, 1)
    b = synthetic_rays(R=512, S=128, seed=5)
    net = net.to(dev)
    rnd = Renderer(net, cfg["rendering"], device=dev)
    gt = torch.rand(1, 512, 3)
    out = rnd.nope_nerf(b["pixels"].to(dev), b["depth"].to(dev), b["K"].to(dev), b["w2c"].to(dev),
                        b["scale"].to(dev), add_noise=True, noise=b["noise"].to(dev))
    loss = orc.rgb_full_loss(out["rgb"], gt.to(dev)) + 0.04 * orc.depth_l1_loss(out["depth_pred"], out["depth_gt"])
    loss.backward()
    o = orc.render_nope_nerf(ref, b["pixels"], b["depth"], b["K"], b["w2c"], b["scale"], cfg["rendering"],
                             noise=b["noise"])
    lo = orc.rgb_full_loss(o["rgb"], gt) + 0.04 * orc.depth_l1_loss(o["depth_pred"], o["depth_gt"])
    lo.backward()
    assert abs(loss.item() - lo.item()) < RTOL * abs(lo.item())
    for (n, p), (n2, q) in zip(net.named_parameters(), ref.named_parameters()):
        assert n == n2
        g, gr = p.grad.cpu(), q.grad
        err = report_err("render_backward", n, ((g - gr).norm() / gr.norm().clamp_min(1e-12)).item())
        assert err < 2e-3, f"{n}: rel grad err {err:.2e}"


_REF_GRADS = {}


def _reference_grads(cfg, ref, b, gt, dtype):
    """The oracle's parameter gradients of the render-backward loss in `dtype` (cached)."""
    key = dtype
    if key not in _REF_GRADS:
        r = orc.OracleNerf(hidden_dim=cfg["model"]["hidden_dim"]).to(dtype)
        r.load_state_dict({k: v.to(dtype) for k, v in ref.state_dict().items()})
        c = lambda t: t.to(dtype)                                          # noqa: E731
        o = orc.render_nope_nerf(r, c(b["pixels"]), c(b["depth"]), c(b["K"]), c(b["w2c"]), c(b["scale"]),
                                 cfg["rendering"], noise=c(b["noise"]))
        (orc.rgb_full_loss(o["rgb"], c(gt)) + 0.04 * orc.depth_l1_loss(o["depth_pred"], o["depth_gt"])).backward()
        _REF_GRADS[key] = {n: p.grad.double() for n, p in r.named_parameters()}
    return _REF_GRADS[key]


def test_render_backward_as_accurate_as_reference(dev, gemm_precision):
    """The HIP parameter gradients against the oracle evaluated in fp64: within 1.5x (+1e-5) of
    how far the fp32 reference itself lands from fp64.  The early layers' gradients of the
    fp32 reference are ~2e-3 off its own fp64 value (ReLU / sign decisions near zero), which is
    why the fp32-vs-fp32 bar of test_render_backward_matches_oracle is 2e-3."""
    cfg = make_cfg(hidden=256, S=128)
    net, ref = _pair(cfg, 1)
    b = synthetic_rays(R=512, S=128, seed=5)
    gt = torch.rand(1, 512, 3, generator=torch.Generator().manual_seed(6))
    net = net.to(dev)
    rnd = Renderer(net, cfg["rendering"], device=dev)
    out = rnd.nope_nerf(b["pixels"].to(dev), b["depth"].to(dev), b["K"].to(dev), b["w2c"].to(dev),
                        b["scale"].to(dev), add_noise=True, noise=b["noise"].to(dev))
    (orc.rgb_full_loss(out["rgb"], gt.to(dev)) + 0.04 * orc.depth_l1_loss(out["depth_pred"], out["depth_gt"])).backward()
    g32 = _reference_grads(cfg, ref, b, gt, torch.float32)
    g64 = _reference_grads(cfg, ref, b, gt, torch.float64)
    for n, p in net.named_parameters():
        e_hip = ((p.grad.double().cpu() - g64[n]).norm() / g64[n].norm()).item()
        e_ref = ((g32[n] - g64[n]).norm() / g64[n].norm()).item()
        report_err("vs_fp64_hip", n, e_hip)
        report_err("vs_fp64_ref32", n, e_ref)
        assert e_hip <= 1.5 * e_ref + 1e-5, f"{n}: HIP {e_hip:.2e} vs the fp32 reference's {e_ref:.2e} (both vs fp64)"


def test_render_ray_gradients(dev, gemm_precision):
    """pose learning: gradients w.r.t. the camera pose flow through the encodings."""
    cfg = make_cfg(hidden=64, S=64)
    net, ref = _pair(cfg, 2)
    b = synthetic_rays(R=128, S=64, seed=4, H=60, W=80)
    net = net.to(dev)
    rnd = Renderer(net, cfg["rendering"], device=dev)
    r = torch.zeros(3, requires_grad=True)
    t = torch.zeros(3, requires_grad=True)
    rd = r.detach().clone().to(dev).requires_grad_(True)
    td = t.detach().clone().to(dev).requires_grad_(True)
    c2w = b["c2w"]
    w2c_d = torch.inverse(orc.make_c2w(rd, td) @ c2w.to(dev)).unsqueeze(0)
    out = rnd.nope_nerf(b["pixels"].to(dev), b["depth"].to(dev), b["K"].to(dev), w2c_d, b["scale"].to(dev),
                        add_noise=True, noise=b["noise"].to(dev))
    out["rgb"].sum().backward()
    w2c = torch.inverse(orc.make_c2w(r, t) @ c2w).unsqueeze(0)
    o = orc.render_nope_nerf(ref, b["pixels"], b["depth"], b["K"], w2c, b["scale"], cfg["rendering"], noise=b["noise"])
    o["rgb"].sum().backward()
    for nm, a, bb in (("r", rd.grad.cpu(), r.grad), ("t", td.grad.cpu(), t.grad)):
        # observed <= 1.7e-5 in every GEMM mode (profiles/r03/grad_err_survey.json)
        assert report_err("render_ray_gradients", nm, ((a - bb).norm() / bb.norm()).item()) < 2e-4


def test_points_forward_api(dev, gemm_precision):
    """OfficialStaticNerf.forward(p, ray_d, return_addocc=True) on arbitrary points."""
    cfg = make_cfg(hidden=256)
    net, ref = _pair(cfg, 4)
    g = torch.Generator().manual_seed(0)
    p = torch.rand(1000, 3, generator=g) * 4 - 2
    d = torch.nn.functional.normalize(torch.randn(1000, 3, generator=g), dim=-1)
    net = net.to(dev)
    rgb, dens = net(p.to(dev), d.to(dev), return_addocc=True)
    rgb_r, dens_r = ref(p, d)
    assert_elementwise(rgb, rgb_r, what="rgb")
    assert_elementwise(dens, dens_r, what="density")


def test_render_image_full_frame(dev, gemm_precision):
    """model.render_dist.render_image (the config-4 render caller, single rank): every
    pixel of a small frame in eval mode (depth prior ones, z-depth output) vs the oracle."""
    from model.render_dist import render_image
    from tests.helpers import camera_K, rigid_c2w
    H, W = 24, 40
    cfg = make_cfg(hidden=64, S=32)
    net, ref = _pair(cfg, 4)
    rnd = Renderer(net.to(dev), cfg["rendering"], device=dev)
    K = camera_K(H, W, 30.0, 30.0)
    w2c = torch.inverse(rigid_c2w(2)).unsqueeze(0)
    scale = torch.eye(4).unsqueeze(0)
    pix = orc.arange_pixels(H, W)[1]
    rgb, depth = render_image(rnd, pix.to(dev), K.to(dev), w2c.to(dev), scale.to(dev))
    with torch.no_grad():
        o = orc.render_nope_nerf(ref, pix, torch.ones(1, H * W, 1), K, w2c, scale, cfg["rendering"], noise=None,
                                 eval_=True)
    assert rgb.shape == (H * W, 3) and depth.shape == (H * W,)
    assert_elementwise(rgb, o["rgb"].reshape(-1, 3), what="rgb")
    assert_elementwise(depth, o["depth_pred"].reshape(-1), what="depth")

"""Shared test fixtures: configs and seeded synthetic V_KITTI-shaped inputs."""
from __future__ import annotations

import torch

from model.synthetic import BASE_CFG, camera_K, make_cfg, rigid_c2w  # noqa: F401  (the package's builders)


def synthetic_rays(R=1024, S=128, H=188, W=621, seed=0, zero_frac=0.05, fx=362.5):
    """A V_KITTI-shaped batch: R random pixels of an HxW image, depth prior U[1,8] with
    some zeros (mask exercise), a fixed rigid pose, stratified noise U[0,1)."""
    g = torch.Generator().manual_seed(seed)
    idx = torch.randperm(H * W, generator=g)[:R]
    rows, cols = idx // W, idx % W
    px = 2.0 * cols.float() / (W - 1) - 1.0
    py = 2.0 * rows.float() / (H - 1) - 1.0
    pixels = torch.stack([px, py], -1).unsqueeze(0)
    depth = 1.0 + 7.0 * torch.rand(1, R, 1, generator=g)
    depth[torch.rand(1, R, 1, generator=g) < zero_frac] = 0.0
    c2w = rigid_c2w(seed)
    return {"pixels": pixels, "depth": depth, "K": camera_K(H, W, fx, fx), "c2w": c2w,
            "w2c": torch.inverse(c2w).unsqueeze(0), "scale": torch.eye(4).unsqueeze(0),
            "noise": torch.rand(1, R, S, generator=g), "ray_idx": idx}


# ---- parity bar (BASELINE.json north_star: 1e-4 rel on rendered RGB / depth) -----------
RENDER_RTOL = 1e-4     # elementwise, relative to the oracle value
RENDER_ATOL = 1e-6     # absolute floor for values near zero (dark pixels, masked depths)


def elementwise_excess(a, b, rtol=RENDER_RTOL, atol=RENDER_ATOL):
    """max over elements of |a - b| / (rtol |b| + atol): <= 1 passes the elementwise bar
    |a - b| <= rtol |b| + atol."""
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs() / (rtol * b.abs() + atol)).max().item()


def assert_elementwise(a, b, rtol=RENDER_RTOL, atol=RENDER_ATOL, what=""):
    """|a - b| <= rtol |b| + atol for every element; the message carries the worst element
    and, as a diagnostic, the max-normalised error max|a-b| / max|b|."""
    a_, b_ = a.detach().double().cpu(), b.detach().double().cpu()
    assert a_.shape == b_.shape, (what, a_.shape, b_.shape)
    err = (a_ - b_).abs()
    lim = rtol * b_.abs() + atol
    ratio = err / lim
    if ratio.numel() and ratio.max().item() > 1.0:
        i = int(ratio.argmax())
        raise AssertionError(f"{what}: element {i}: |{a_.flatten()[i].item():.9g} - {b_.flatten()[i].item():.9g}| = "
                             f"{err.flatten()[i].item():.3g} > {rtol:g}*|b| + {atol:g} "
                             f"(max-normalised error {(err.max() / b_.abs().max().clamp_min(1e-30)).item():.3g})")


def report_err(test: str, name: str, err: float) -> float:
    """Observed parity error of one checked quantity, appended to $NERF_ERR_REPORT (one JSON
    line each) when set -- the survey the gradient tolerances are set from; returns err."""
    import json
    import os
    path = os.environ.get("NERF_ERR_REPORT")
    if path:
        from model import _hip
        with open(path, "a") as f:
            f.write(json.dumps({"test": test, "name": name, "err": float(err),
                                "mode": _hip.gemm_get_precision()}) + "\n")
    return err

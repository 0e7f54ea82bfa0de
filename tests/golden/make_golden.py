"""Generates tests/golden/render_*.pt from the oracle (CPU restatement).

The reference publishes no vectors and may not be imported here, so
these fixtures freeze the oracle's outputs: inputs (weights, rays, noise) and expected
outputs (rgb, depth, alpha, loss, parameter gradients).  Regenerate only on purpose:
    python tests/golden/make_golden.py
"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import nerf_oracle as orc  # noqa: E402
from tests.helpers import synthetic_rays  # noqa: E402

CASES = {
    # name: (hidden, S, R, render-cfg overrides, seed)
    "cfg1_d64": (64, 64, 96, {}, 11),
    "cfg2_d256": (256, 128, 48, {}, 12),
    "llff_ndc_distalpha": (64, 32, 40, {"sample_option": "ndc", "dist_alpha": True, "depth_range": [0.0, 1.0]}, 13),
    "white_bkgd": (64, 48, 40, {"white_background": True}, 14),
}


def make(name):
    hidden, S, R, over, seed = CASES[name]
    torch.manual_seed(seed)
    cfg = {"num_points": S}
    cfg.update(over)
    net = orc.OracleNerf(hidden_dim=hidden, white_background=cfg.get("white_background", False),
                         dist_alpha=cfg.get("dist_alpha", False))
    b = synthetic_rays(R=R, S=S, seed=seed, H=60, W=90, fx=45.0)
    noise = None if cfg.get("sample_option") == "ndc" else b["noise"]
    out = orc.render_nope_nerf(net, b["pixels"], b["depth"], b["K"], b["w2c"], b["scale"], cfg, noise=noise)
    gt = torch.rand(1, R, 3, generator=torch.Generator().manual_seed(seed))
    loss = orc.rgb_full_loss(out["rgb"], gt) + 0.04 * orc.depth_l1_loss(out["depth_pred"], out["depth_gt"])
    loss.backward()
    return {"cfg": cfg, "hidden": hidden, "state_dict": net.state_dict(),
            "inputs": {k: b[k] for k in ("pixels", "depth", "K", "w2c", "scale")}, "noise": noise, "gt": gt,
            "rgb": out["rgb"].detach(), "depth_pred": out["depth_pred"].detach(),
            "depth_gt": out["depth_gt"].detach(), "alpha": out["alpha"].detach(), "loss": loss.detach(),
            "grads": {n: p.grad.clone() for n, p in net.named_parameters()
                      if hidden <= 64 or n.startswith(("fc_", "rgb_layers", "layers0.0"))}}


if __name__ == "__main__":
    for name in CASES:
        torch.save(make(name), os.path.join(HERE, f"render_{name}.pt"))
        print("wrote", name)

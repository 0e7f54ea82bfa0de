"""get_model (drop-in for model/config.py:4-18) without the DPT branch: every training
config sets depth.type None (DPT is offline preprocessing only)."""
from __future__ import annotations

from .network import nope_nerf


def get_model(renderer, cfg, device=None, **kwargs):
    if cfg["depth"]["type"] == "DPT":
        raise NotImplementedError("the DPT depth estimator is preprocessing, outside the MI355X hot path")
    return nope_nerf(cfg, renderer, None, device)

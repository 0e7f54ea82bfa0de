"""Per-camera depth-prior scale / shift (drop-in for model/distortions.py:4-27).

The reference clamps with a Python ``if scale < 0.01`` (a device->host sync every
step, distortions.py:21); the same value is produced here with ``torch.where``.
"""
from __future__ import annotations

import torch
import torch.nn as nn


class Learn_Distortion(nn.Module):
    def __init__(self, num_cams, learn_scale, learn_shift, cfg):
        super().__init__()
        self.global_scales = nn.Parameter(torch.ones(num_cams, 1, dtype=torch.float32), requires_grad=learn_scale)
        self.global_shifts = nn.Parameter(torch.zeros(num_cams, 1, dtype=torch.float32), requires_grad=learn_shift)
        self.fix_scaleN = cfg["distortion"]["fix_scaleN"]
        self.num_cams = num_cams

    def forward(self, cam_id):
        cam = int(cam_id)
        scale = self.global_scales[cam]
        # below 0.01 the reference substitutes a constant (no gradient): keep that
        scale = torch.where(scale < 0.01, torch.full_like(scale, 0.01).detach(), scale)
        if self.fix_scaleN and cam == self.num_cams - 1:
            scale = torch.ones_like(scale).detach()
        return scale, self.global_shifts[cam]

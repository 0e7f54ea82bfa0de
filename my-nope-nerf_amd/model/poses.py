"""Per-camera pose parameters (drop-in for model/poses.py:6-33).

c2w = [Exp(r) | t] @ init_c2w[cam]: a left-multiplied SO(3) x R^3 delta (not an SE(3)
exponential: the translation is not coupled to the rotation), common.py:290-310.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .rays import pose_c2w


class LearnPose(nn.Module):
    def __init__(self, num_cams, learn_R, learn_t, cfg=None, init_c2w=None):
        super().__init__()
        self.num_cams = num_cams
        self.init_c2w = None
        if init_c2w is not None:
            self.init_c2w = nn.Parameter(init_c2w, requires_grad=False)
        self.r = nn.Parameter(torch.zeros(num_cams, 3, dtype=torch.float32), requires_grad=learn_R)
        self.t = nn.Parameter(torch.zeros(num_cams, 3, dtype=torch.float32), requires_grad=learn_t)

    def forward(self, cam_id):
        cam = int(cam_id)   # a host-side index (img.idx comes from the data dict on the CPU)
        # one HIP launch on the device (Exp, [R|t], @ init_c2w), torch on the host
        return pose_c2w(self.r[cam], self.t[cam], None if self.init_c2w is None else self.init_c2w[cam])

    def get_t(self):
        return self.t

"""LearnFocal (drop-in for model/intrinsics.py:5-70): the learnable focal length the
drivers construct when ``pose.learn_focal`` is set (train.py:140, vis/render.py:78).

Never learned in the V_KITTI configs, so it stays a host-side torch
module; a learned K also makes the Trainer keep the torch pair terms (training.py).
Parameterisation: order 2 stores a with fx = a**2, order 1 stores fx itself."""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn


class LearnFocal(nn.Module):
    def __init__(self, req_grad, fx_only, order=2, init_focal=None):
        super().__init__()
        if order not in (1, 2):
            raise ValueError("Focal init order need to be 1 or 2")     # the reference prints and exits
        self.fx_only = fx_only
        self.order = order

        def coeff(f):
            return torch.tensor(np.sqrt(f) if order == 2 else f).float()

        if init_focal is None:
            init = (torch.tensor(1.0), torch.tensor(1.0))
        elif isinstance(init_focal, list) and not fx_only:
            init = (coeff(init_focal[0]), coeff(init_focal[1]))
        else:
            init = (coeff(init_focal), coeff(init_focal))
        self.fx = nn.Parameter(init[0], requires_grad=req_grad)
        if not fx_only:
            self.fy = nn.Parameter(init[1], requires_grad=req_grad)

    def forward(self, i=None):
        """intrinsics.py:59-70 -> [fx, fy] (fy = fx when fx_only)."""
        fy = self.fx if self.fx_only else self.fy
        f = torch.stack([self.fx, fy])
        return f ** 2 if self.order == 2 else f

"""OfficialStaticNerf on the MI355X path (drop-in for model/official_nerf.py).

Same constructor, same ``nn.Linear`` parameters and state_dict keys
(official_nerf.py:20-44) and the same ``forward`` signature (official_nerf.py:69-96), so
reference checkpoints load unchanged and ``torch.optim.Adam(model.parameters())`` works.
Evaluation goes through the nerf_hip kernels (field.py): FP32 MFMA layers, fused
encodings and heads.  The fused render path (rays -> composite) used by the Renderer
never materialises per-sample rgb/density at all.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .field import FieldRunner, eval_points, trunk_points


class _FirstOrderOnly(torch.autograd.Function):
    """Marks the normals of OfficialStaticNerf.gradient: the HIP backward is first order, so
    the normals carry no gradient of their own.  Anchored to a field parameter, a loss that
    reaches them (a second derivative through the field, e.g. rgb + w * normal) fails loudly
    in its backward instead of silently dropping the normal term."""

    @staticmethod
    def forward(ctx, g, anchor):
        return g.clone()

    @staticmethod
    def backward(ctx, gg):
        raise RuntimeError("nerf_hip: a loss reached OfficialStaticNerf.gradient()'s normals; second derivatives "
                           "through the HIP field are not supported (the reference's create_graph=True path, "
                           "official_nerf.py:46-58)")


class OfficialStaticNerf(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        D = cfg["model"]["hidden_dim"]
        pos_levels = cfg["model"]["pos_enc_levels"]
        dir_levels = cfg["model"]["dir_enc_levels"]
        # the encodings are hard-wired to L=10 / L=4 in the reference forward
        # (official_nerf.py:61,87) while the input widths follow the cfg (:14-15)
        if (pos_levels, dir_levels) != (10, 4):
            raise ValueError("reference forward hard-codes pos/dir encoding levels 10/4 "
                             f"(official_nerf.py:61,87); cfg asks {pos_levels}/{dir_levels}")
        pin = (2 * pos_levels + 1) * 3
        din = (2 * dir_levels + 1) * 3
        self.hidden_dim = D
        self.white_bkgd = cfg["rendering"]["white_background"]
        self.dist_alpha = cfg["rendering"]["dist_alpha"]
        self.occ_activation = cfg["model"]["occ_activation"]

        def trunk(first_in):
            return nn.Sequential(nn.Linear(first_in, D), nn.ReLU(), nn.Linear(D, D), nn.ReLU(),
                                 nn.Linear(D, D), nn.ReLU(), nn.Linear(D, D), nn.ReLU())

        self.layers0 = trunk(pin)
        self.layers1 = trunk(D + pin)            # skip: cat[x, pos_enc]
        self.fc_density = nn.Linear(D, 1)
        self.fc_feature = nn.Linear(D, D)
        self.rgb_layers = nn.Sequential(nn.Linear(D + din, D // 2), nn.ReLU())
        self.fc_rgb = nn.Linear(D // 2, 3)
        self.fc_density.bias.data = torch.tensor([0.1]).float()
        self.sigmoid = nn.Sigmoid()
        rgb_b = 0.8 if self.white_bkgd else 0.02
        self.fc_rgb.bias.data = torch.tensor([rgb_b, rgb_b, rgb_b]).float()
        self._runner = None

    def hip_runner(self) -> FieldRunner:
        if self._runner is None:
            self._runner = FieldRunner(self)
        return self._runner

    def _density(self, raw):
        sigma = F.softplus(raw) if self.occ_activation == "softplus" else raw.relu()
        if not self.dist_alpha:
            sigma = 1 - torch.exp(-1.0 * sigma)
        return sigma

    def infer_occ(self, p):
        """official_nerf.py:60-67: (x, density) = (trunk output [..,D], fc_density(x) [..,1],
        before the activation), from one HIP forward.  Both are differentiable w.r.t. p and
        the parameters (first order; see field.FieldTrunkFn)."""
        shape = p.shape[:-1]
        x, density = trunk_points(self, p.reshape(-1, 3).float())
        return x.reshape(*shape, self.hidden_dim), density.reshape(*shape, 1)

    def forward(self, p, ray_d=None, only_occupancy=False, return_logits=False, return_addocc=False,
                noise=False, it=100000, **kwargs):
        """official_nerf.py:69-96 on the HIP path: p [..,3], ray_d [..,3]."""
        shape = p.shape[:-1]
        pf = p.reshape(-1, 3).float()
        df = (ray_d if ray_d is not None else torch.zeros_like(p)).reshape(-1, 3).float()
        raw = eval_points(self, pf, df)
        density = self._density(raw[:, 0:1]).reshape(*shape, 1)
        if only_occupancy:
            return density
        if ray_d is None:
            return None
        rgb = torch.sigmoid(raw[:, 1:4]).reshape(*shape, 3)
        if return_addocc:
            return rgb, density
        return rgb

    def gradient(self, p, it):
        """official_nerf.py:46-58: -d(density_raw)/dp, through the HIP backward.  The reference
        builds the result with create_graph=True; the HIP backward is first order, so the
        values are the same but they carry no second-order graph: when the field's parameters
        require grad the result is anchored to them by _FirstOrderOnly, and any loss that
        reaches it raises in its backward (no reference loss does, losses.py:164-228)."""
        with torch.enable_grad():
            p = p.detach().requires_grad_(True)
            raw = eval_points(self, p.reshape(-1, 3), torch.zeros_like(p).reshape(-1, 3))
            y = raw[:, 0:1]
            g = torch.autograd.grad(y, p, torch.ones_like(y), retain_graph=False)[0]
            # that backward's parameter gradients are discarded (autograd.grad returns dp only):
            # hand the data-parallel gradient buffer back, so the step's real backward writes
            # into it in place instead of into a fresh flat that the all-reduce must copy
            if self._runner is not None:
                self._runner.release_grad_buffer()
            anchor = self.fc_density.bias
            if anchor.requires_grad:
                g = _FirstOrderOnly.apply(g, anchor)
            return -g.unsqueeze(1)

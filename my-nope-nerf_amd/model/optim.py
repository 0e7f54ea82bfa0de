"""Adam on one flat fp32 buffer with a single nerf_adam_step launch per step.

Same update as torch.optim.Adam (amsgrad=False, train.py:59 / :100 / :118 use the
defaults betas=(0.9, 0.999), eps=1e-8), and the same state_dict format (per-parameter
``step`` / ``exp_avg`` / ``exp_avg_sq``), so optimizer states in reference checkpoints
(checkpoints.py:29-41, key ``optimizer``) load here and vice versa.  At construction the parameters' storage is
moved into one contiguous buffer (each ``p.data`` becomes a view of it) so the update
is one launch; the FieldRunner backward already produces the NeRF gradients as views of
one flat buffer in parameter order, in which case no gather copy is made either.
"""
from __future__ import annotations

import torch

from . import _hip


def hyper_block(lr, beta1, beta2, eps, weight_decay, step=0.0):
    """k_adam's hyper-parameter block as a CPU float32 [16] tensor: the scalars torch's Adam
    forms from its Python doubles -- 1 - beta1 and 1 - beta2 rounded once to f32 (slots 14, 6),
    lr / beta1 / beta2 kept as doubles (slots 8-13) for the bias corrections lr / (1 - beta1^t)
    and sqrt(1 - beta2^t), which the kernel takes in double at the device step count."""
    import numpy as np
    b = np.zeros(16, dtype=np.float32)
    b[:7] = (step, lr, beta1, beta2, eps, weight_decay, 1.0 - beta2)
    b[8:14].view(np.float64)[:] = (lr, beta1, beta2)
    b[14] = 1.0 - beta1
    b[15] = 1.0
    return torch.from_numpy(b)


class HipAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        if len(self.param_groups) != 1:
            raise ValueError("HipAdam supports one parameter group")
        ps = [p for p in self.param_groups[0]["params"] if p.requires_grad]
        if not ps:
            raise ValueError("no trainable parameters")
        dev = ps[0].device
        n = sum(p.numel() for p in ps)
        self._flat = torch.empty(n, device=dev, dtype=torch.float32)
        off = 0
        self._slices = {}
        for p in ps:
            k = p.numel()
            self._flat[off:off + k].copy_(p.data.reshape(-1))
            p.data = self._flat[off:off + k].view_as(p)
            self._slices[id(p)] = (off, k)
            off += k
        self._params = ps
        self._m = torch.zeros_like(self._flat)
        self._v = torch.zeros_like(self._flat)
        # the device block k_adam reads (graph-replay safe), 16 floats: {step, lr, beta1, beta2,
        # eps, weight_decay, 1 - beta2, ticket, lr / beta1 / beta2 as doubles (slots 8-13),
        # 1 - beta1, 1.0 = the doubles are valid}
        self._hyper = torch.zeros(16, device=dev, dtype=torch.float32)
        self._hyper_host = None
        self._sync_hyper()

    def sync_hyper(self):
        """Push the param-group hyper-parameters (lr, betas, eps, weight decay) into the
        device block k_adam reads.  step() does this itself when run eagerly; a captured
        hipGraph replays the launch without the host, so a caller whose LR scheduler edits
        param_groups between replays calls sync_hyper() after the scheduler step."""
        self._sync_hyper()

    def _sync_hyper(self):
        g = self.param_groups[0]
        h = (float(g["lr"]), float(g["betas"][0]), float(g["betas"][1]), float(g["eps"]), float(g["weight_decay"]))
        if h != self._hyper_host:      # lr schedulers edit param_groups; push the change
            self._hyper[1:].copy_(hyper_block(*h)[1:], non_blocking=False)
            self._hyper_host = h

    def _flat_grad(self):
        gs = [p.grad for p in self._params]
        if any(g is None for g in gs):
            # torch.optim.Adam skips such a parameter (no moment decay, no step count); one
            # fused update over the flat buffer cannot, so refuse instead of diverging silently
            raise RuntimeError("HipAdam: a parameter has no gradient this step; torch.optim.Adam would skip it. "
                               "Use HipAdam for modules whose parameters all receive gradients (the NeRF field).")
        g0 = gs[0]
        base = g0.untyped_storage().data_ptr() if g0.is_contiguous() else None
        if base is not None:
            ptr = g0.data_ptr()
            ok = True
            for g, p in zip(gs, self._params):
                if not g.is_contiguous() or g.data_ptr() != ptr:
                    ok = False
                    break
                ptr += p.numel() * 4
            if ok:
                return torch.as_strided(g0, (self._flat.numel(),), (1,))
        return torch.cat([g.reshape(-1) for g in gs])

    # ---- torch.optim.Adam-compatible state_dict --------------------------------------
    _ADAM_DEFAULTS = {"amsgrad": False, "maximize": False, "foreach": None, "capturable": False,
                      "differentiable": False, "fused": None}

    def state_dict(self):
        sd = super().state_dict()
        g = sd["param_groups"][0]
        for k, v in self._ADAM_DEFAULTS.items():
            g.setdefault(k, v)
        step = float(self._hyper[0].item())
        if step > 0:
            for idx, p in enumerate(self.param_groups[0]["params"]):
                if id(p) not in self._slices:
                    continue
                off, k = self._slices[id(p)]
                sd["state"][idx] = {"step": torch.tensor(step, dtype=torch.float32),
                                    "exp_avg": self._m[off:off + k].view_as(p).clone(),
                                    "exp_avg_sq": self._v[off:off + k].view_as(p).clone()}
        return sd

    @torch.no_grad()
    def load_state_dict(self, state_dict):
        groups = state_dict["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(self.param_groups[0]["params"]):
            raise ValueError("HipAdam.load_state_dict: parameter groups do not match")
        g = self.param_groups[0]
        for k in ("lr", "betas", "eps", "weight_decay"):
            if k in groups[0]:
                g[k] = groups[0][k]
        if groups[0].get("amsgrad", False):
            raise ValueError("HipAdam: amsgrad states are not supported")
        self._m.zero_()
        self._v.zero_()
        step = 0.0
        pos = {pid: i for i, pid in enumerate(groups[0]["params"])}
        for pid, st in state_dict["state"].items():
            p = g["params"][pos[pid]]
            if id(p) not in self._slices:
                continue
            off, k = self._slices[id(p)]
            self._m[off:off + k].copy_(st["exp_avg"].reshape(-1))
            self._v[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
            step = float(st["step"])
        self._hyper_host = None
        self._sync_hyper()
        self._hyper[0].fill_(step)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        if not torch.cuda.is_current_stream_capturing():
            self._sync_hyper()
        _hip.adam_step(self._flat, self._flat_grad().contiguous(), self._m, self._v, self._hyper)
        return loss

"""Host orchestration of the MI355X per-sample hot path.

One call renders R rays x S samples through
  samples + encodings  (rendering.py:183-198, official_nerf.py:99-119)
  -> 8-layer trunk with skip, feature, colour layer on FP32 MFMA (official_nerf.py:60-91)
  -> density / colour heads (official_nerf.py:66, 91)
  -> sigma->alpha + exclusive-product compositing (rendering.py:113-141)
and its backward (training.py:92), entirely in the nerf_hip kernels.  Parameters stay the
reference ``nn.Linear`` tensors (so state_dicts and ``torch.optim`` keep working); a pack
kernel copies them into zero-padded MFMA-friendly layouts once per call.

Data layout in HBM (N_pad = R*S rounded up to 128 rows, samples ray-major):
  enc_p, enc_d : [N_pad][64] fp32        z, raw4 : [N_pad], [N_pad][4]
  h1..h8, f    : [N_pad][D] fp32 (post-ReLU, saved for the backward)
  hr           : [N_pad][HR] fp32 (HR = max(64, D/2))
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
from torch.autograd.function import once_differentiable

from . import _hip

F_DIST_ALPHA, F_WHITE_BKGD, F_RELU = 1, 2, 4


def _pad_rows(n: int) -> int:
    return (n + _hip.ROW_TILE - 1) // _hip.ROW_TILE * _hip.ROW_TILE


def _dw_splits(m: int, tiles: int, target_blocks: int = 512) -> int:
    """Split-K factor for the weight-gradient GEMM: a power of two giving ~target blocks
    with each split a whole number of 32-row K tiles."""
    splits = 1
    while (splits * 2 * tiles <= target_blocks and m % (splits * 2 * 32) == 0
           and m // (splits * 2) >= 256):
        splits *= 2
    return splits


@dataclass
class LayerSpec:
    name: str
    linear: torch.nn.Linear
    k1: int          # columns taken from the first input
    seg2: Optional[str]  # 'enc_p' / 'enc_d' / None (second K segment, 64 wide)
    out_p: int       # padded output rows
    relu: bool

    @property
    def kp(self) -> int:
        return self.k1 + (_hip.ENC_P if self.seg2 else 0)


class FieldRunner:
    """Owns the packed weights of one OfficialStaticNerf and launches the kernels."""

    def __init__(self, module):
        self.m = module
        D = module.hidden_dim
        if D % 64 != 0:
            raise ValueError(f"nerf_hip: hidden_dim {D} must be a multiple of 64")
        self.D = D
        self.HR = max(64, D // 2)
        m = module
        L = [
            LayerSpec("l0", m.layers0[0], _hip.ENC_P, None, D, True),
            LayerSpec("l1", m.layers0[2], D, None, D, True),
            LayerSpec("l2", m.layers0[4], D, None, D, True),
            LayerSpec("l3", m.layers0[6], D, None, D, True),
            LayerSpec("l4", m.layers1[0], D, "enc_p", D, True),
            LayerSpec("l5", m.layers1[2], D, None, D, True),
            LayerSpec("l6", m.layers1[4], D, None, D, True),
            LayerSpec("l7", m.layers1[6], D, None, D, True),
            LayerSpec("lf", m.fc_feature, D, None, D, False),
            LayerSpec("lr", m.rgb_layers[0], D, "enc_d", self.HR, True),
        ]
        self.layers = L
        self.device = None
        self._side = None
        self._plist = None
        # optional persistent gradient buffer (Trainer.allreduce_grads): when set, the backward
        # writes the parameter gradients as views of grad_buffer[:n] in param_list() order, so
        # the data-parallel all-reduce runs in place on it.  It is handed out once per step: the
        # first backward that finds every field gradient None takes it (grad_buffer_taken), a
        # second field backward in the same autograd pass (e.g. a render and an infer_occ summed
        # into one loss: autograd accumulates into param.grad only after both ran) writes a
        # fresh flat instead of overwriting the first one's views; the Trainer releases it after
        # the all-reduce and at the start of every step (release_grad_buffer)
        self.grad_buffer = None
        self.grad_buffer_taken = False

    # ------------------------------------------------------------------ packing
    def _alloc(self, device):
        D, HR = self.D, self.HR
        z = lambda *s: torch.zeros(*s, device=device, dtype=torch.float32)
        self.w = {l.name: z(l.out_p, l.kp) for l in self.layers}
        self.wt = {l.name: z(l.kp, l.out_p) for l in self.layers}
        # bf16x3 split images of w / wt: the B operands of GEMM precision mode 1
        self.ws = {l.name: _hip.split_image(l.out_p, l.kp, device) for l in self.layers}
        self.wts = {l.name: _hip.split_image(l.kp, l.out_p, device) for l in self.layers}
        # precision mode 2's chain images (nerf_pack_desc dst_cs / dst_cts): the same fp16 pair
        # form with K in the order the two-wave chains hold a layer's outputs (chain.hip)
        self.wsc = {l.name: _hip.split_image(l.out_p, l.kp, device) for l in self.layers}
        self.wtsc = {l.name: _hip.split_image(l.kp, l.out_p, device) for l in self.layers}
        # padded, 16-byte-aligned copies of every layer bias (the chain kernel loads them by
        # 16-byte LDS-DMA; HipAdam's flat parameter buffer leaves biases 4-byte aligned)
        self.bias_p = {l.name: z(l.out_p) for l in self.layers}
        self.b_r = self.bias_p["lr"]
        self.wc = z(3, HR)         # padded fc_rgb weight
        self.wd = z(1, D)          # 16-byte-aligned fc_density weight (the fused density head reads it by float4)
        self.device = device

    def pack(self):
        dev = self.m.layers0[0].weight.device
        if dev.type != "cuda":
            raise RuntimeError("nerf_hip: the field must live on the GPU (no CPU fallback)")
        if self.device != dev:
            self._alloc(dev)
        # split images only when the GEMMs run in a split mode (1: bf16x3, 2: fp16 pair;
        # the pack kernel writes the form of the current mode)
        prec = _hip.gemm_get_precision()
        self.split = prec >= 1
        self.h16 = prec == 2
        descs = []
        for l in self.layers:
            W = l.linear.weight
            assert W.is_contiguous() and W.dtype == torch.float32
            ws = self.ws[l.name].data_ptr() if self.split else None
            wts = self.wts[l.name].data_ptr() if self.split else None
            chain = self.h16 and self.D == 256 and self.HR == 128
            wsc = self.wsc[l.name].data_ptr() if chain else None
            wtsc = self.wtsc[l.name].data_ptr() if chain else None
            descs.append(_hip.PackDesc(W.data_ptr(), self.w[l.name].data_ptr(), self.wt[l.name].data_ptr(),
                                       W.shape[0], W.shape[1], l.kp, l.kp, l.out_p, ws, wts, l.out_p, wsc, wtsc,
                                       l.k1 if l.name != "l0" else 0))
        for l in self.layers:
            b = l.linear.bias
            descs.append(_hip.PackDesc(b.data_ptr(), self.bias_p[l.name].data_ptr(), None, 1, b.shape[0], l.out_p, 0, 0))
        wc = self.m.fc_rgb.weight
        descs.append(_hip.PackDesc(wc.data_ptr(), self.wc.data_ptr(), None, 3, wc.shape[1], self.HR, 0, 0))
        wd = self.m.fc_density.weight
        descs.append(_hip.PackDesc(wd.data_ptr(), self.wd.data_ptr(), None, 1, wd.shape[1], self.D, 0, 0))
        _hip.pack_weights(descs)

    def bias(self, l: LayerSpec):
        return self.bias_p[l.name]

    # ------------------------------------------------------------------ forward
    def forward(self, pts_o, pts_d, view, noise, near, far, S: int, flags: int, keep: bool,
                composite: bool = True):
        """Renders R = pts_o.shape[0] rays.  Returns rgb [R,3], dist [R], alpha [R,S], z [R,S]
        and (if keep) the saved state for backward().  With composite=False the first
        output is the raw head tensor raw4 [N_pad,4] (sigma_raw, rgb logits)."""
        R = pts_o.shape[0]
        N = R * S
        Np = _pad_rows(N)
        dev = pts_o.device
        D, HR = self.D, self.HR
        e = lambda *s: torch.empty(*s, device=dev, dtype=torch.float32)
        self.pack()
        z = e(Np)
        enc_p = e(Np, _hip.ENC_P)
        enc_d = e(Np, _hip.ENC_D)
        # precision mode 2: every GEMM A operand travels with its row max (written by its producer)
        rm, cm = self._rmax_alloc(Np, dev), self._cmax_alloc(Np, dev, keep)
        enc_p_rm, enc_d_rm = rm(64), rm(64)
        enc_p_cm, enc_d_cm = cm(64), cm(64)
        _hip.encode_samples(pts_o, pts_d, view, noise, R, S, Np, near, far, z, enc_p, enc_d,
                            enc_p_rmax=enc_p_rm, enc_d_rmax=enc_d_rm, enc_p_cmax=enc_p_cm, enc_d_cmax=enc_d_cm)
        acts = []
        if keep:
            outs = [e(Np, D) for _ in range(9)] + [e(Np, HR)]
        else:
            ping = [e(Np, D), e(Np, D)]
            outs = [ping[i % 2] for i in range(9)] + [e(Np, HR)]
        x = enc_p
        x_rm = enc_p_rm
        segs = {"enc_p": enc_p, "enc_d": enc_d}
        seg_rm = {"enc_p": enc_p_rm, "enc_d": enc_d_rm}
        masks = {}
        cmaxes = {"enc_p": enc_p_cm, "enc_d": enc_d_cm}
        raw4 = e(Np, 4)
        m = self.m
        chain_heads = False
        if self.use_chain(keep):
            # all ten linears in one launch, activations resident in registers (chain.hip);
            # training (keep): nerf_mlp_chain_train saves every output, ReLU word and column
            # maximum the per-layer path saves, and computes raw4 in its epilogues
            descs = []
            for i, l in enumerate(self.layers):
                y = outs[i] if (keep or l.name in ("l7", "lr")) else None
                mo = None
                if keep and l.relu:
                    mo = torch.empty(Np, l.out_p // 32, device=dev, dtype=torch.int32)
                    # as the per-layer path: the colour layer's bits only with the split heads backward
                    if l.name != "lr" or self.heads_side(Np):
                        masks[l.name] = mo
                y_cm = cm(l.out_p) if l.name != "lr" else None
                cmaxes[l.name] = y_cm
                # the training chain reads the chain images, the one-wave eval chain the plain ones
                ws = self.wsc[l.name] if keep else self.ws[l.name]
                descs.append(_hip.ChainLayer(ws.data_ptr(), ws.shape[2], self.bias(l).data_ptr(),
                                             y.data_ptr() if y is not None else None, l.out_p,
                                             mo.data_ptr() if mo is not None else None, l.out_p // 32,
                                             y_cm.data_ptr() if y_cm is not None else None))
                acts.append(y if y is not None else outs[i])
            if keep:
                _hip.mlp_chain_train(enc_p, enc_d, enc_p_rm, enc_d_rm, Np, descs, m.fc_density.weight,
                                     m.fc_density.bias, self.wc, m.fc_rgb.bias, raw4)
                chain_heads = True
            else:
                _hip.mlp_chain_fwd(enc_p, enc_d, enc_p_rm, enc_d_rm, Np, descs)
            h8 = acts[7]
        # precision mode 2 at hidden 256: the density / colour heads run in the l7 / colour-layer
        # epilogues (nerf_linear_fwd_heads) instead of a separate pass over h8 and hr
        fuse_heads = self.h16 and D == 256 and HR == 128 and not self.use_chain(keep)
        head_args = {"l7": (self.wd, m.fc_density.bias, raw4, 0), "lr": (self.wc, m.fc_rgb.bias, raw4, 1)}
        for i, l in enumerate(self.layers if not self.use_chain(keep) else []):
            y = outs[i]
            x2 = segs[l.seg2] if l.seg2 else None
            k1 = l.k1
            mo = None
            # ReLU bits for the backward's input masks (and, with the split heads backward,
            # the colour layer's own: they gate dyr instead of a re-read of hr)
            if keep and l.relu and (l.name != "lr" or self.heads_side(Np)):
                mo = torch.empty(Np, l.out_p // 32, device=dev, dtype=torch.int32)
                masks[l.name] = mo
            y_rm = rm(l.out_p)
            y_cm = cm(l.out_p) if l.name != "lr" else None     # hr feeds no weight gradient GEMM
            cmaxes[l.name] = y_cm
            _hip.linear_fwd(x, k1, x2, _hip.ENC_P if x2 is not None else 0, self.w[l.name], self.bias(l), y,
                            Np, l.out_p, l.relu, mask_out=mo, w_split=self.ws[l.name] if self.split else None,
                            x1_rmax=x_rm, x2_rmax=seg_rm[l.seg2] if l.seg2 else None, y_rmax=y_rm, y_cmax=y_cm,
                            heads=head_args.get(l.name) if fuse_heads else None)
            acts.append(y)
            x = y
            x_rm = y_rm
            if l.name == "l7":
                h8 = y
        hr = acts[9]
        if not (fuse_heads or chain_heads):
            _hip.heads_fwd(h8, hr, D, m.fc_density.weight, m.fc_density.bias, self.wc, m.fc_rgb.bias, raw4, Np)
        if composite:
            rgb = e(R, 3)
            dist = e(R)
            alpha = e(R, S)
            _hip.composite_fwd(raw4, z, R, S, flags, rgb, dist, alpha)
        else:
            rgb, dist, alpha = raw4, None, None
        state = None
        if keep:
            state = dict(R=R, S=S, Np=Np, flags=flags, z=z, enc_p=enc_p, enc_d=enc_d, acts=acts, raw4=raw4,
                         masks=masks, pts_o=pts_o, pts_d=pts_d, view=view, cmaxes=cmaxes)
        return rgb, dist, alpha, z[:N].view(R, S), state

    def use_chain(self, keep: bool = False) -> bool:
        """The fused layer chain (chain.hip) covers precision mode 2 at hidden 256 / colour
        128, and is the default there.  Eval renders (keep=False) run nerf_mlp_chain_fwd (or
        the fused per-ray kernel, use_fused_eval); training (keep=True) runs
        nerf_mlp_chain_train at two waves per SIMD, which saves every output, ReLU word and
        column maximum beside its MFMAs: 736-768 vs 877-904 us per 131072-sample forward and
        2.474 vs 2.550 ms per cfg2 step (profiles/r03/train_chain_ab.txt).  NERF_CHAIN=0
        runs one launch per layer; NERF_CHAIN=1 forces the chain."""
        if not (_hip.gemm_get_precision() == 2 and self.D == 256 and self.HR == 128):
            return False
        return os.environ.get("NERF_CHAIN", "1") != "0"

    def use_fused_eval(self, S: int) -> bool:
        """The fused per-ray eval kernel (nerf_render_eval_fused: samples, encodings, the
        layer chain, heads and composite in one launch) covers the chain's configurations
        when a ray's samples tile the 128-row block (S >= 2 divides 128).  NERF_FUSED=0
        falls back to the chain + separate encode / heads / composite launches."""
        if os.environ.get("NERF_FUSED") == "0":
            return False
        return self.use_chain(False) and S >= 2 and 128 % S == 0

    def render_eval_fused(self, pts_o, pts_d, view, near, far, S: int, flags: int):
        """-> rgb [R,3], dist [R], alpha [R,S], z [R,S] in one launch (no saved state)."""
        R = pts_o.shape[0]
        dev = pts_o.device
        self.pack()
        descs = [_hip.ChainLayer(self.wsc[l.name].data_ptr(), self.wsc[l.name].shape[2], self.bias(l).data_ptr(),
                                 None, l.out_p, None, l.out_p // 32, None) for l in self.layers]
        e = lambda *sh: torch.empty(*sh, device=dev, dtype=torch.float32)
        rgb, dist, alpha, z = e(R, 3), e(R), e(R, S), e(R, S)
        m = self.m
        _hip.render_eval_fused(pts_o, pts_d, view, R, S, near, far, flags, descs, m.fc_density.weight,
                               m.fc_density.bias, self.wc, m.fc_rgb.bias, rgb, dist, alpha, z)
        return rgb, dist, alpha, z

    def _rmax_alloc(self, Np: int, dev):
        """Row-max buffer factory for precision mode 2 (None otherwise): a buffer for an
        operand of `width` columns; wider than one 256-column GEMM block it is max-accumulated
        by the kernel and starts at zero."""
        if not self.h16:
            return lambda width: None
        return lambda width: (torch.zeros if width > 256 else torch.empty)(Np, device=dev, dtype=torch.float32)

    def _cmax_alloc(self, Np: int, dev, keep: bool = True):
        """Column-max buffer factory (mode 2, training only): [Np/128][width] per 128-row
        group, the column scales of the weight-gradient GEMMs."""
        if not (self.h16 and keep):
            return lambda width: None
        return lambda width: torch.empty(Np // 128, width, device=dev, dtype=torch.float32)

    # ------------------------------------------------------------------ backward
    def heads_side(self, Np: int) -> bool:
        """Split heads backward (nerf_heads_bwd_mode): at the training size dyr alone stays on
        the input-gradient chain, gated by the colour layer's ReLU bits, and the head-weight
        partials run on the side stream (profiles/r02/heads_side_step_ab.txt)."""
        default = "1" if (self.D == 256 and Np >= 65536) else "0"
        return int(os.environ.get("NERF_HEADS_SIDE", default)) != 0

    def native_backward(self, Np: int) -> bool:
        """The training backward as one native call (nerf_field_backward, csrc/field_bwd.cpp):
        the Python schedule below, launch for launch, for the configuration it covers -- GEMM
        precision mode 2, hidden 256 / colour 128, the split heads backward (Np >= 65536).
        Bit-identical gradients (tests/test_gpu_native_bwd.py); 0.8 ms of Python host time per
        cfg2 step become a few microseconds per launch.  NERF_NATIVE_BWD=0 keeps the Python
        schedule."""
        return (self.h16 and self.D == 256 and self.HR == 128 and self.heads_side(Np)
                and os.environ.get("NERF_NATIVE_BWD", "1") != "0")

    def bwd_chain(self) -> bool:
        """The native backward's input gradients as one launch (nerf_mlp_chain_bwd: dyr and the
        nine input-gradient GEMMs with dy resident in registers) -- the default; NERF_BWD_CHAIN=0
        runs them as nine nerf_linear_bwd_data launches beside the weight gradients."""
        return os.environ.get("NERF_BWD_CHAIN", "1") != "0"

    def _backward_native(self, st, g_rgb, g_dist, want_ray_grad, graw4, G):
        Np, R, S = st["Np"], st["R"], st["S"]
        dev = st["z"].device
        m = self.m
        if self._side is None or self._side[0].device != dev:
            self._side = [torch.cuda.Stream(dev)]
        acts, masks, cms = st["acts"], st["masks"], st["cmaxes"]
        names = [l.name for l in self.layers]
        P = lambda t: None if t is None else t.data_ptr()            # noqa: E731
        ray = None
        ray_ptrs = (None, None, None)
        if want_ray_grad:
            ray = tuple(torch.empty(R, 3, device=dev) for _ in range(3))
            ray_ptrs = tuple(t.data_ptr() for t in ray)
        ws = torch.empty(_hip.field_bwd_workspace_bytes(Np, want_ray_grad), device=dev, dtype=torch.uint8)
        tail_default = 2 if Np >= 65536 else 0
        args = _hip.FieldBwd(
            Np, R, S, st["flags"], int(want_ray_grad), int(os.environ.get("NERF_TAIL_MAIN", str(tail_default))),
            int(self.bwd_chain()), P(st["z"]), P(st["raw4"]), P(st["enc_p"]), P(st["enc_d"]), P(st["cmaxes"]["enc_p"]),
            P(st["cmaxes"]["enc_d"]), _hip._P10(*[a.data_ptr() for a in acts]),
            _hip._P10(*[P(masks.get(n)) for n in names]), _hip._P10(*[P(cms.get(n)) for n in names]),
            P(st["pts_o"]), P(st["pts_d"]), P(st["view"]),
            _hip._P10(*[self.wt[n].data_ptr() for n in names]), _hip._P10(*[self.wts[n].data_ptr() for n in names]),
            _hip._P10(*[self.wtsc[n].data_ptr() for n in names]), self.wd.data_ptr(), self.wc.data_ptr(), P(g_rgb), P(g_dist), P(graw4),
            _hip._P10(*[G(l.linear.weight).data_ptr() for l in self.layers]),
            _hip._P10(*[G(l.linear.bias).data_ptr() for l in self.layers]),
            G(m.fc_density.weight).data_ptr(), G(m.fc_density.bias).data_ptr(), G(m.fc_rgb.weight).data_ptr(),
            G(m.fc_rgb.bias).data_ptr(), *ray_ptrs, ws.data_ptr())
        _hip.field_backward(args, self._side[0].cuda_stream)
        return ray

    def release_grad_buffer(self):
        """The persistent gradient buffer may be handed out again (Trainer: after the
        all-reduce and when a step starts)."""
        self.grad_buffer_taken = False

    def param_list(self) -> List[torch.nn.Parameter]:
        """The field's parameters in module order.  Cached: walking the module tree costs ~75 us
        of host time and runs twice per training step; the runner already binds the layers'
        nn.Linear objects at construction, so the tree is fixed for its lifetime (a parameter
        re-assigned as a new object is caught by the identity check on the bound layers)."""
        pl = self._plist
        if pl is None or pl[0] is not self.layers[0].linear.weight:
            pl = self._plist = list(self.m.parameters())
        return pl

    def backward(self, st, g_rgb, g_dist, want_ray_grad: bool, graw4=None, g_h8=None):
        """Returns (list of parameter gradients in self.param_list() order, ray grads or None).
        Starts from the ray gradients (composite backward) or, when ``graw4`` is given,
        directly from the gradient of the raw head outputs.  ``g_h8`` [Np, D] (optional): an
        extra gradient w.r.t. the trunk output h8 (infer_occ's x), added where l7's ReLU
        passes it."""
        R, S, Np, flags = st["R"], st["S"], st["Np"], st["flags"]
        D, HR = self.D, self.HR
        dev = st["z"].device
        e = lambda *s: torch.empty(*s, device=dev, dtype=torch.float32)
        acts = st["acts"]
        h = {l.name: acts[i] for i, l in enumerate(self.layers)}
        m = self.m
        params = self.param_list()
        n_par = sum(p.numel() for p in params)
        buf = self.grad_buffer
        if (buf is not None and not self.grad_buffer_taken and buf.device == dev and buf.numel() >= n_par
                and all(p.grad is None for p in params)):
            # autograd hands these views on as param.grad (no other gradient to accumulate into)
            flat = buf[:n_par]
            self.grad_buffer_taken = True
        else:
            flat = torch.empty(n_par, device=dev, dtype=torch.float32)
        grads, off = {}, 0
        for p in params:
            grads[id(p)] = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        G = lambda p: grads[id(p)]

        if g_h8 is None and self.native_backward(Np):
            return [G(p) for p in params], self._backward_native(st, g_rgb, g_dist, want_ray_grad, graw4, G)
        if graw4 is None:
            graw4 = e(Np, 4)
            _hip.composite_bwd(st["raw4"], st["z"], R, S, flags, g_rgb, g_dist, graw4, Np)
        # walk the layers backwards; dy = gradient w.r.t. the layer's pre-activation output.
        # The weight gradients (split-K GEMM + slab reduce) of layer l depend only on dy_l and
        # the saved input, so they run on a side stream beside the dX chain: compute-bound
        # GEMM phases overlap the memory-bound reductions and each other's prologue/epilogue.
        main = torch.cuda.current_stream(dev)
        if self._side is None or self._side[0].device != dev:
            self._side = [torch.cuda.Stream(dev)]
        sides = self._side

        # heads: d(fc_density), d(fc_rgb), dY of the colour layer.  Only dyr (+ its maxima) is
        # on the input-gradient chain; at the training size the head-weight partials (which
        # re-read h8 and hr) and their reduce run on the side stream, beside dyr and the colour
        # layer's input gradient, before that stream's first weight gradient needs dyr
        dyr = e(Np, HR)
        rm, cm = self._rmax_alloc(Np, dev), self._cmax_alloc(Np, dev)
        dy_rm, dy_cm = rm(HR), cm(HR)
        split_heads = self.heads_side(Np)
        gw = (G(m.fc_density.weight), G(m.fc_density.bias), G(m.fc_rgb.bias))

        def head_weights(mode):
            part = e(_hip.heads_part_size(D, Np))
            gwc = G(m.fc_rgb.weight) if HR == D // 2 else e(3, HR)
            _hip.heads_bwd(graw4, h["l7"], h["lr"], D, self.wc, dyr if mode == 3 else None, part, Np,
                           dyr_rmax=dy_rm if mode == 3 else None, dyr_cmax=dy_cm if mode == 3 else None, mode=mode)
            _hip.heads_reduce(part, D, Np, gw[0], gw[1], gwc, gw[2])
            if HR != D // 2:
                G(m.fc_rgb.weight).copy_(gwc[:, :D // 2])

        if split_heads:
            ev = torch.cuda.Event()
            ev.record(main)
            sides[0].wait_event(ev)
            for t in (graw4, h["l7"], h["lr"]):
                t.record_stream(sides[0])
            with torch.cuda.stream(sides[0]):
                head_weights(2)
            lr_mask = st["masks"].get("lr")
            _hip.heads_bwd(graw4, None, h["lr"] if lr_mask is None else None, D, self.wc, dyr, None, Np,
                           dyr_rmax=dy_rm, dyr_cmax=dy_cm, mode=1, hr_mask=lr_mask)
        else:
            head_weights(3)
        fcm = st.get("cmaxes", {})
        prev_cm = {"l0": "enc_p", "l1": "l0", "l2": "l1", "l3": "l2", "l4": "l3", "l5": "l4", "l6": "l5",
                   "l7": "l6", "lf": "l7", "lr": "lf"}

        # encoding gradients (pose learning): enc_p reaches layers l0 and l4 (skip), enc_d the
        # colour layer; each GEMM writes its own buffer and encode_bwd sums the two enc_p ones
        genc = {}

        # at the training size the side stream trails the input-gradient chain by ~3 layers, and
        # the last layers' weight gradients finish sooner on the main stream behind the chain than
        # behind more cross-stream waits: 2 of them before the heads split (2.60 vs 2.67 ms/step,
        # profiles/r02/backward_schedule_ab2.json), 3 since it put the head-weight partials on the
        # side stream (2.552 vs 2.567, tail_schedule_ab_heads_side.json), 2 again since the faster
        # XCD-paired weight-gradient tiles (TN policy 7) let the side stream keep up (2.575 vs
        # 2.602 and 2.535 vs 2.539, tail_schedule_ab_policy7.txt); small batches keep everything
        # beside the chain
        tail_default = 2 if (D == 256 and Np >= 65536) else 0
        tail_main = int(os.environ.get("NERF_TAIL_MAIN", str(tail_default)))
        dy = dyr
        prev_in = {"l0": st["enc_p"], "l1": h["l0"], "l2": h["l1"], "l3": h["l2"], "l4": h["l3"],
                   "l5": h["l4"], "l6": h["l5"], "l7": h["l6"], "lf": h["l7"], "lr": h["lf"]}
        order = ["lr", "lf", "l7", "l6", "l5", "l4", "l3", "l2", "l1", "l0"]
        prev_name = {"l1": "l0", "l2": "l1", "l3": "l2", "l4": "l3", "l5": "l4", "l6": "l5", "l7": "l6",
                     "lf": "l7", "lr": "lf"}
        spec = {l.name: l for l in self.layers}
        seg_buf = {"enc_p": st["enc_p"], "enc_d": st["enc_d"]}
        def weight_grad(l, dy, dy_cm, x_in):
            W = l.linear.weight
            nout_ref, kin_ref = W.shape
            k1 = l.k1
            # a layer with a 64-wide second segment (l4's skip input) shares one split count over
            # both launches, sized for the wide one (profiles/r02/seg2_splits_ab.txt)
            splits = _hip.bwd_weight_splits(l.out_p, k1, Np)
            slab = e(splits * l.out_p * l.kp)
            bslab = e(splits * l.out_p)
            if l.seg2 and os.environ.get("NERF_DW_SEG", "1") != "0":
                # both input segments in one launch (dy read once; nerf_linear_bwd_weight_seg).
                # NERF_DW_SEG=0 (A/B only): the two launches of round 3's first half
                _hip.linear_bwd_weight_seg(dy, l.out_p, x_in, k1, seg_buf[l.seg2], 64, Np, splits, slab, l.kp, bslab,
                                           dy_cmax=dy_cm, x1_cmax=fcm.get(prev_cm[l.name]), x2_cmax=fcm.get(l.seg2))
            else:
                _hip.linear_bwd_weight(dy, l.out_p, x_in, k1, Np, splits, slab, l.kp, 0, bslab, dy_cmax=dy_cm,
                                       x_cmax=fcm.get(prev_cm[l.name]))
                if l.seg2:
                    _hip.linear_bwd_weight(dy, l.out_p, seg_buf[l.seg2], 64, Np, splits, slab, l.kp, k1, None,
                                           dy_cmax=dy_cm, x_cmax=fcm.get(l.seg2))
            gb = G(l.linear.bias) if l.out_p == nout_ref else e(l.out_p)
            _hip.slab_reduce(slab, splits, l.out_p, l.kp, nout_ref, kin_ref, bslab, G(W), gb)
            if l.out_p != nout_ref:
                G(l.linear.bias).copy_(gb[:nout_ref])

        deferred = []
        for step, name in enumerate(order):
            l = spec[name]
            W = l.linear.weight
            x_in = prev_in[name]
            k1 = l.k1
            # --- weight / bias gradient on a side stream: split-K slabs + reduce.  The last
            # NERF_TAIL_MAIN layers' run on the main stream once the input-gradient chain is done
            # (every cross-stream wait costs ~15 us before the next launch)
            if step >= len(order) - tail_main:
                deferred.append((l, dy, dy_cm, x_in))
            else:
                side = sides[0]
                ev = torch.cuda.Event()
                ev.record(main)
                side.wait_event(ev)
                dy.record_stream(side)          # dy_l is freed by the main loop while side reads it
                if dy_cm is not None:
                    dy_cm.record_stream(side)
                with torch.cuda.stream(side):
                    weight_grad(l, dy, dy_cm, x_in)
            # --- input gradient
            wt = self.wt[name]
            wts = self.wts[name] if self.split else None
            rows = (lambda a, b: wts[:, :, a:b]) if self.split else (lambda a, b: None)
            if name == "l0":
                if want_ray_grad:
                    genc["p0"] = e(Np, _hip.ENC_P)
                    _hip.linear_bwd_data(dy, l.out_p, wt, genc["p0"], Np, _hip.ENC_P, wt_split=wts, dy_rmax=dy_rm)
                break
            if l.seg2 and want_ray_grad:
                key = "p4" if l.seg2 == "enc_p" else "d"
                genc[key] = e(Np, 64)
                _hip.linear_bwd_data(dy, l.out_p, wt[k1:k1 + 64], genc[key], Np, 64, wt_split=rows(k1, k1 + 64),
                                     dy_rmax=dy_rm)
            dx = e(Np, k1)
            dx_rm, dx_cm = rm(k1), cm(k1)
            # ReLU bits of this layer's input (f, the input of lr, has no activation)
            mask = None if name == "lr" else st["masks"][prev_name[name]]
            if name == "lf":   # + density path: d sigma_raw (graw4[:,0]) x w_density
                _hip.linear_bwd_data(dy, l.out_p, wt[:k1], dx, Np, k1, mask=mask, u=graw4, ldu=4,
                                     v=self.wd.view(-1), wt_split=rows(0, k1), dy_rmax=dy_rm, dx_rmax=dx_rm,
                                     dx_cmax=dx_cm)     # v: the 16-byte-aligned copy (float4 epilogue reads)
                if g_h8 is not None:
                    # infer_occ's x = h8 (post-ReLU): its gradient joins l7's pre-activation gradient
                    # through the same ReLU; the row / column maxima the next GEMMs scale by are
                    # re-taken (the epilogue wrote those of dx without it)
                    dx.add_(g_h8 * (h["l7"] > 0))
                    if dx_rm is not None:
                        torch.amax(dx.abs(), 1, out=dx_rm)
                    if dx_cm is not None:
                        torch.amax(dx.abs().view(Np // 128, 128, k1), 1, out=dx_cm)
            else:
                _hip.linear_bwd_data(dy, l.out_p, wt[:k1], dx, Np, k1, mask=mask, wt_split=rows(0, k1),
                                     dy_rmax=dy_rm, dx_rmax=dx_rm, dx_cmax=dx_cm)
            dy = dx
            dy_rm, dy_cm = dx_rm, dx_cm

        for args in deferred:
            weight_grad(*args)
        for side in sides:
            done = torch.cuda.Event()
            done.record(side)
            main.wait_event(done)           # gradients complete before autograd hands them on
        ray = None
        if want_ray_grad:
            g_po, g_pd, g_view = e(R, 3), e(R, 3), e(R, 3)
            _hip.encode_bwd(st["pts_o"], st["pts_d"], st["view"], st["z"], genc["p0"], genc["d"], R, S,
                            g_po, g_pd, g_view, genc_p2=genc["p4"])
            ray = (g_po, g_pd, g_view)
        return [G(p) for p in params], ray


class FieldRenderFn(torch.autograd.Function):
    """autograd boundary of the fused HIP render path.  Inputs: ray origins/directions
    used for the sample points, the view direction fed to the colour branch, the
    injected stratified noise, and the field parameters (so autograd routes their
    gradients to ``param.grad`` exactly as nn.Linear would)."""

    @staticmethod
    def forward(ctx, runner: FieldRunner, pts_o, pts_d, view, noise, near, far, S, flags, *params):
        ctx.set_materialize_grads(False)      # alpha / z (and an unused dist) get no zero fill
        rgb, dist, alpha, z, st = runner.forward(pts_o, pts_d, view, noise, near, far, S, flags, keep=True)
        ctx.runner = runner
        ctx.state = st
        ctx.ray_grad = any(ctx.needs_input_grad[1:4])
        ctx.mark_non_differentiable(alpha, z)
        return rgb, dist, alpha, z

    @staticmethod
    @once_differentiable
    def backward(ctx, g_rgb, g_dist, g_alpha, g_z):
        st = ctx.state
        R = st["R"]
        if g_rgb is None:
            g_rgb = torch.zeros(R, 3, device=st["z"].device)
        if g_dist is None:
            g_dist = torch.zeros(R, device=st["z"].device)
        grads, ray = ctx.runner.backward(st, g_rgb.contiguous(), g_dist.contiguous(), ctx.ray_grad)
        ctx.state = None
        g_po = g_pd = g_view = None
        if ray is not None:
            g_po, g_pd, g_view = ray
        return (None, g_po, g_pd, g_view, None, None, None, None, None, *grads)


def render_field(module, pts_o, pts_d, view, noise, near, far, S, flags):
    """Differentiable render of R rays through the HIP path (training)."""
    runner = module.hip_runner()
    params = runner.param_list()
    return FieldRenderFn.apply(runner, pts_o.contiguous(), pts_d.contiguous(), view.contiguous(),
                               None if noise is None else noise.contiguous(), float(near), float(far),
                               int(S), int(flags), *params)


@torch.no_grad()
def render_field_eval(module, pts_o, pts_d, view, near, far, S, flags, ray_chunk: int = 32768):
    """Forward-only render in ray chunks (ping-pong activations, no saved state).  A chunk of
    32768 rays x 128 samples is 4.2 M rows per GEMM launch (~9 GB of transient activations):
    few, large launches on a 288 GB device."""
    runner = module.hip_runner()
    R = pts_o.shape[0]
    if runner.use_fused_eval(S):
        # one launch for the whole frame: nothing per-sample is materialised but alpha / z
        return runner.render_eval_fused(pts_o.contiguous(), pts_d.contiguous(), view.contiguous(), near, far, S,
                                        flags)
    outs = []
    for r0 in range(0, R, ray_chunk):
        r1 = min(R, r0 + ray_chunk)
        rgb, dist, alpha, z, _ = runner.forward(pts_o[r0:r1].contiguous(), pts_d[r0:r1].contiguous(),
                                                view[r0:r1].contiguous(), None, near, far, S, flags, keep=False)
        outs.append((rgb, dist, alpha, z))
    return tuple(torch.cat([o[i] for o in outs], 0) for i in range(4))


class FieldRawFn(torch.autograd.Function):
    """Per-point evaluation (OfficialStaticNerf.forward, official_nerf.py:69-96): points
    p [n,3] and view directions [n,3] -> raw head outputs [n,4] (sigma_raw, rgb logits),
    differentiable w.r.t. the points, the directions and the parameters."""

    @staticmethod
    def forward(ctx, runner: FieldRunner, p, d, *params):
        n = p.shape[0]
        zeros = torch.zeros_like(p)
        raw4, _, _, _, st = runner.forward(p, zeros, d, None, 0.0, 0.0, 1, 0, keep=True, composite=False)
        ctx.runner, ctx.state, ctx.n = runner, st, n
        ctx.ray_grad = any(ctx.needs_input_grad[1:3])
        return raw4[:n]

    @staticmethod
    @once_differentiable      # no second derivatives through the HIP kernels: a double backward raises
    def backward(ctx, g_raw):
        st = ctx.state
        Np = st["Np"]
        graw4 = torch.zeros(Np, 4, device=g_raw.device)
        graw4[:ctx.n] = g_raw
        grads, ray = ctx.runner.backward(st, None, None, ctx.ray_grad, graw4=graw4)
        ctx.state = None
        g_p = g_d = None
        if ray is not None:
            g_p, _, g_d = ray
        return (None, g_p, g_d, *grads)


class FieldTrunkFn(torch.autograd.Function):
    """OfficialStaticNerf.infer_occ (official_nerf.py:60-67) in one HIP forward: points
    p [n,3] -> (x [n,D] the trunk output h8, sigma_raw [n,1] = fc_density(x)), both
    differentiable w.r.t. the points and the parameters (one runner backward that starts from
    d sigma_raw and adds dL/dx at the trunk output).  First order only: a double backward
    (create_graph=True, e.g. a loss on gradient()'s normals) raises."""

    @staticmethod
    def forward(ctx, runner: FieldRunner, p, *params):
        # an unused output gets None, not a zero tensor: g_h8 None keeps the native backward
        ctx.set_materialize_grads(False)
        n = p.shape[0]
        zeros = torch.zeros_like(p)
        raw4, _, _, _, st = runner.forward(p, zeros, zeros, None, 0.0, 0.0, 1, 0, keep=True, composite=False)
        h8 = st["acts"][7][:n, :runner.D].clone()
        ctx.runner, ctx.state, ctx.n = runner, st, n
        ctx.ray_grad = ctx.needs_input_grad[1]
        return h8, raw4[:n, 0:1].clone()

    @staticmethod
    @once_differentiable
    def backward(ctx, g_h8, g_sigma):
        st = ctx.state
        Np, n = st["Np"], ctx.n
        dev = st["z"].device
        graw4 = torch.zeros(Np, 4, device=dev)
        if g_sigma is not None:
            graw4[:n, 0:1] = g_sigma
        gx = None
        if g_h8 is not None:
            gx = torch.zeros(Np, ctx.runner.D, device=dev)
            gx[:n] = g_h8
        grads, ray = ctx.runner.backward(st, None, None, ctx.ray_grad, graw4=graw4, g_h8=gx)
        ctx.state = None
        g_p = ray[0] if ray is not None else None
        return (None, g_p, *grads)


def trunk_points(module, p):
    """(x [n,D], sigma_raw [n,1]) of points p [n,3] (infer_occ)."""
    runner = module.hip_runner()
    return FieldTrunkFn.apply(runner, p.contiguous(), *runner.param_list())


def eval_points(module, p, d):
    """raw head outputs for arbitrary points (autograd-aware)."""
    runner = module.hip_runner()
    return FieldRawFn.apply(runner, p.contiguous(), d.contiguous(), *runner.param_list())

"""Ray prologue and loss epilogue of the training step on the HIP kernels of rays.hip
(on-device ray generation).

The reference builds every step's rays from ~150 ATen launches: ``randperm`` + gathers
(training.py:277-283), ``Exp``/``make_c2w`` (common.py:277-310), three 4x4 inversions per
unprojection (common.py:139-141, 205-208), ``transform_to_world``/``origin_to_world``
(rendering.py:52-80) and the loss terms with their autograd backward (losses.py:28-66,
164-228).  Here each is one launch, wrapped in an autograd Function whose backward is
exact (the camera-ray and loss backwards are HIP kernels; the 4x4 chains, which only
need gradients when poses / focals are learned, use the closed-form matrix identities).

Device tensors always take these kernels (no silent fallback).  Host tensors (dataset
preparation, CPU tools) use the torch expressions of the reference functions.
"""
from __future__ import annotations

import torch

from . import _hip


def _f32c(t):
    return t.detach().float().contiguous()


# ------------------------------------------------------------------ 4x4 inverse
class _Inv4(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a):
        ctx.set_materialize_grads(False)
        a_c = _f32c(a)
        out = torch.empty_like(a_c)
        _hip.mat4_inv(a_c, out)
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return None
        (y,) = ctx.saved_tensors          # d inv(A) = -Y dA Y  ->  gA = -Y^T g Y^T (one launch)
        ga = torch.empty_like(y)
        _hip.mat4_inv_bwd(y, _f32c(g), ga)
        return ga


def inv(m):
    """torch.inverse of [..., 4, 4] (training.py:255-257, losses.py:162)."""
    if not m.is_cuda:
        return torch.linalg.inv_ex(m)[0]
    if m.shape[-2:] != (4, 4):
        raise ValueError(f"inv: expected [..., 4, 4], got {tuple(m.shape)}")
    return _Inv4.apply(m)


# ------------------------------------------------------------------ 4x4 product
class _Mat4Mul(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        ctx.set_materialize_grads(False)
        ac, bc = _f32c(a), _f32c(b)
        out = torch.empty(ac.shape, device=a.device, dtype=torch.float32)
        _hip.mat4_mul(ac, bc, out)
        ctx.save_for_backward(ac, bc)
        return out

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return None, None
        ac, bc = ctx.saved_tensors
        want_a, want_b = ctx.needs_input_grad
        ga = torch.empty_like(ac) if want_a else None
        gb = torch.empty_like(bc) if want_b else None
        if want_a or want_b:
            _hip.mat4_mul_bwd(ac, bc, _f32c(g), ga, gb)
        return ga, gb


def mat4_mul(a, b):
    """a @ b for equally shaped [..., 4, 4] (training.py:337-343's relative poses): one launch
    forward and one backward on the device, torch matmul on the host."""
    if not a.is_cuda or a.shape != b.shape or a.shape[-2:] != (4, 4):
        return a @ b
    return _Mat4Mul.apply(a, b)


# ------------------------------------------------------------------ depth-prior distortion
class _DepthAffine(torch.autograd.Function):
    @staticmethod
    def forward(ctx, d, scale, shift, shift_first, lo):
        ctx.set_materialize_grads(False)
        dc, sc, tc = _f32c(d), _f32c(scale), _f32c(shift)
        y = torch.empty_like(dc)
        _hip.depth_affine(dc, sc, tc, shift_first, lo, y)
        ctx.save_for_backward(dc, sc, tc)
        ctx.meta = (shift_first, lo, scale.shape, shift.shape)
        return y.view(d.shape)

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return None, None, None, None, None
        dc, sc, tc = ctx.saved_tensors
        shift_first, lo, ssh, tsh = ctx.meta
        want_s, want_t = ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        gs = torch.empty(1, device=dc.device, dtype=torch.float32) if want_s else None
        gt = torch.empty(1, device=dc.device, dtype=torch.float32) if want_t else None
        if want_s or want_t:
            _hip.depth_affine_bwd(dc, sc, tc, shift_first, lo, _f32c(g), gs, gt)
        return (None, gs.view(ssh) if want_s else None, gt.view(tsh) if want_t else None, None, None)


def depth_affine(d, scale, shift, shift_first=False, lo=float("-inf")):
    """The depth prior's scale / shift (training.py:259-264, 325-329) on prior values d, then
    the nearest_limit clamp y < lo -> lo (training.py:346-347): one launch forward, one
    backward (gradients to scale / shift only: the prior is data).  Torch on the host or when
    the prior itself needs a gradient."""
    if not d.is_cuda or d.requires_grad or scale.numel() != 1 or shift.numel() != 1:
        y = (d + shift) * scale if shift_first else d * scale + shift
        return y.clamp_min(lo) if lo != float("-inf") else y
    return _DepthAffine.apply(d, scale, shift, int(bool(shift_first)), float(lo))


# ------------------------------------------------------------------ pose
def _pose_torch(r, t, init):
    """common.py:277-310 / poses.py:27-30 in torch (host tensors, and the backward)."""
    z = torch.zeros_like(r[0:1])
    K = torch.stack([torch.cat([z, -r[2:3], r[1:2]]), torch.cat([r[2:3], z, -r[0:1]]),
                     torch.cat([-r[1:2], r[0:1], z])], dim=0)
    th = r.norm() + 1e-15
    I = torch.eye(3, dtype=r.dtype, device=r.device)
    R = I + (torch.sin(th) / th) * K + ((1 - torch.cos(th)) / th ** 2) * (K @ K)
    top = torch.cat([R, t.unsqueeze(1)], dim=1)
    c2w = torch.cat([top, torch.eye(4, dtype=r.dtype, device=r.device)[3:]], dim=0)
    return c2w if init is None else c2w @ init


class _PoseC2W(torch.autograd.Function):
    @staticmethod
    def forward(ctx, r, t, init):
        ctx.set_materialize_grads(False)
        out = torch.empty(4, 4, device=r.device, dtype=torch.float32)
        _hip.pose_c2w(_f32c(r), _f32c(t), None if init is None else _f32c(init), out)
        ctx.save_for_backward(r, t, init)
        return out

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return None, None, None
        r, t, init = ctx.saved_tensors
        want_r, want_t, want_i = ctx.needs_input_grad
        g_init = None
        if want_i:
            # a learned init_c2w (never in the reference configs): torch autograd of the expression
            with torch.enable_grad():
                ii = init.detach().requires_grad_(True)
                (g_init,) = torch.autograd.grad(_pose_torch(r.detach(), t.detach(), ii), [ii], g)
        if not (want_r or want_t):
            return None, None, g_init
        # the closed-form derivative of Exp / [R | t] @ init: one launch (nerf_pose_c2w_bwd)
        g_r = torch.empty(3, device=r.device, dtype=torch.float32) if want_r else None
        g_t = torch.empty(3, device=r.device, dtype=torch.float32) if want_t else None
        _hip.pose_c2w_bwd(_f32c(r), None if init is None else _f32c(init), _f32c(g), g_r, g_t)
        return (g_r.view_as(r) if want_r else None, g_t.view_as(t) if want_t else None, g_init)


def pose_c2w(r, t, init=None):
    """[Exp(r) | t; 0 0 0 1] @ init for one camera (r, t: [3]; init: [4,4] or None)."""
    if not r.is_cuda:
        return _pose_torch(r, t, init)
    return _PoseC2W.apply(r, t, init)


# ------------------------------------------------------------------ unprojection matrix
class _Unproject(torch.autograd.Function):
    @staticmethod
    def forward(ctx, K, world, scale):
        ctx.set_materialize_grads(False)
        M = torch.empty(4, 4, device=K.device, dtype=torch.float32)
        invs = torch.empty(3, 4, 4, device=K.device, dtype=torch.float32)
        _hip.unproject_matrix(_f32c(K), _f32c(world), _f32c(scale), M, invs)
        ctx.save_for_backward(invs)
        ctx.shapes = (K.shape, world.shape, scale.shape)
        return M.view(1, 4, 4)

    @staticmethod
    def backward(ctx, gM):
        if gM is None:
            return None, None, None
        (invs,) = ctx.saved_tensors
        # M = Si Wi Ki and d inv(A) = -inv(A) dA inv(A): all three in one launch
        want = ctx.needs_input_grad
        e = lambda: torch.empty(4, 4, device=invs.device, dtype=torch.float32)
        gK, gW, gS = (e() if want[0] else None), (e() if want[1] else None), (e() if want[2] else None)
        _hip.unproject_matrix_bwd(invs, _f32c(gM), gK, gW, gS)
        sh = ctx.shapes
        return (gK.reshape(sh[0]) if gK is not None else None, gW.reshape(sh[1]) if gW is not None else None,
                gS.reshape(sh[2]) if gS is not None else None)


def unproject_matrix(camera_mat, world_mat, scale_mat):
    """scale^-1 @ world^-1 @ K^-1 in the reference's association order -> [1,4,4]."""
    if not camera_mat.is_cuda:
        iv = lambda m: torch.linalg.inv_ex(m)[0]
        return (iv(scale_mat) @ iv(world_mat)) @ iv(camera_mat)
    for m in (camera_mat, world_mat, scale_mat):
        if m.numel() != 16:
            raise ValueError("unproject_matrix: one camera per call (batch 1)")
    return _Unproject.apply(camera_mat, world_mat, scale_mat)


# ------------------------------------------------------------------ camera rays
class _CameraRays(torch.autograd.Function):
    @staticmethod
    def forward(ctx, M, pixels, depth, flags):
        ctx.set_materialize_grads(False)      # unused outputs (mask, ray_norm ...) get no zero fill
        R = pixels.shape[1]
        dev = pixels.device
        e = lambda *s: torch.empty(*s, device=dev, dtype=torch.float32)
        cam, ray, view, ray_norm, d_src = e(R, 3), e(R, 3), e(R, 3), e(R), e(R)
        mask = torch.empty(R, device=dev, dtype=torch.bool)
        Mc, pc = _f32c(M), _f32c(pixels)
        dc = None if depth is None else _f32c(depth)
        _hip.camera_rays(Mc, pc, dc, R, flags, cam, ray, view, ray_norm, d_src, mask)
        ctx.save_for_backward(Mc, pc, dc)
        ctx.flags = flags
        ctx.shapes = (M.shape, None if depth is None else depth.shape)
        ctx.mark_non_differentiable(mask)
        return cam, ray, view, ray_norm, d_src, mask

    @staticmethod
    def backward(ctx, g_cam, g_ray, g_view, g_norm, g_dsrc, g_mask):
        Mc, pc, dc = ctx.saved_tensors
        R = pc.shape[1]
        c = lambda g: None if g is None else g.float().contiguous()
        gM = torch.empty(4, 4, device=pc.device, dtype=torch.float32)
        want_d = dc is not None and ctx.needs_input_grad[2]
        g_depth = torch.empty(R, device=pc.device, dtype=torch.float32) if want_d else None
        _hip.camera_rays_bwd(Mc, pc, dc, R, ctx.flags, c(g_cam), c(g_ray), c(g_view), c(g_norm), c(g_dsrc), gM,
                             g_depth)
        return (gM.reshape(ctx.shapes[0]) if ctx.needs_input_grad[0] else None, None,
                g_depth.reshape(ctx.shapes[1]) if want_d else None, None)


def camera_rays_hip(M, pixels, depth, normalise_ray=True, view_ones=False):
    """(cam, ray, view, ray_norm, d_src, mask) of pixels [1,R,2], depth [1,R,1] or None."""
    flags = (_hip.RAYS_NORMALISE if normalise_ray else 0) | (_hip.RAYS_VIEW_ONES if view_ones else 0)
    return _CameraRays.apply(M, pixels, depth, flags)


# ------------------------------------------------------------------ loss terms
class _RayLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rgb, rgb_gt, dpred, dgt, mask, l1, w_rgb, w_depth):
        ctx.set_materialize_grads(False)      # the three logged scalars usually get no gradient
        dev = rgb.device
        R = rgb.numel() // 3
        out = [torch.empty((), device=dev, dtype=torch.float32) for _ in range(4)]
        cnt = torch.empty((), device=dev, dtype=torch.float32)
        rc, gc = _f32c(rgb), _f32c(rgb_gt)
        dpc = None if dpred is None else _f32c(dpred)
        dgc = None if dgt is None else _f32c(dgt)
        mc = None if mask is None else mask.contiguous()
        n_d = 0 if dpc is None else dpc.numel()
        _hip.ray_loss(rc, gc, R, dpc, dgc, mc, n_d, l1, w_rgb, w_depth, out, cnt)
        ctx.save_for_backward(rc, gc, dpc, dgc, mc, cnt)
        ctx.meta = (R, n_d, l1, w_rgb, w_depth, rgb.shape, None if dpred is None else dpred.shape)
        return out[0], out[1], out[2], out[3]

    @staticmethod
    def backward(ctx, g_total, g_rgb_l, g_depth_l, g_l2):
        rc, gc, dpc, dgc, mc, cnt = ctx.saved_tensors
        R, n_d, l1, w_rgb, w_depth, rshape, dshape = ctx.meta
        c = lambda g: None if g is None else g.float().contiguous()
        want_rgb = ctx.needs_input_grad[0]
        want_dp = dpc is not None and ctx.needs_input_grad[2]
        want_dg = dgc is not None and ctx.needs_input_grad[3]
        if not (want_rgb or want_dp or want_dg):
            return (None,) * 8
        g_rgb = torch.empty(R, 3, device=rc.device, dtype=torch.float32) if want_rgb else None
        g_dp = torch.empty(n_d, device=rc.device, dtype=torch.float32) if want_dp else None
        g_dg = torch.empty(n_d, device=rc.device, dtype=torch.float32) if want_dg else None
        _hip.ray_loss_bwd(rc, gc, R, dpc, dgc, mc, n_d, l1, w_rgb, w_depth,
                          [c(g_total), c(g_rgb_l), c(g_depth_l), c(g_l2)], cnt, g_rgb, g_dp, g_dg)
        return (g_rgb.reshape(rshape) if want_rgb else None, None,
                g_dp.reshape(dshape) if want_dp else None, g_dg.reshape(dshape) if want_dg else None,
                None, None, None, None)


def ray_loss(rgb, rgb_gt, depth_pred, depth_gt, depth_mask, rgb_l1: bool, w_rgb: float, w_depth: float):
    """(total = w_rgb l_rgb + w_depth l_depth, l_rgb, l_depth, l2_mean) in one launch; the
    depth term is skipped (0) when depth_pred is None."""
    return _RayLoss.apply(rgb, rgb_gt, depth_pred, depth_gt, depth_mask, int(bool(rgb_l1)), float(w_rgb),
                          float(w_depth))


# ------------------------------------------------------------------ ray sampling
def sample_rays(n_pix, n_rays, width, height, img=None, seed=None, device=None, seed_counter=None):
    """Device replacement of ``randperm(n_pix)[:n_rays]`` + the pixel / colour gathers:
    returns (ray_idx int64 [R], pixels [1,R,2], rgb_gt [1,R,3] or None).  ``seed``
    defaults to a draw from torch's host generator (deterministic under manual_seed);
    ``seed_counter`` (device int64 [1]) makes the draw advance on the device instead."""
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    dev = device if device is not None else img.device
    idx = torch.empty(n_rays, device=dev, dtype=torch.int64)
    pix = torch.empty(1, n_rays, 2, device=dev, dtype=torch.float32)
    rgb = None
    imc = None
    if img is not None:
        imc = _f32c(img)
        rgb = torch.empty(1, n_rays, 3, device=dev, dtype=torch.float32)
    _hip.sample_rays(n_pix, n_rays, seed, width, height, imc, idx, pix, rgb, seed_counter=seed_counter)
    return idx, pix, rgb


def can_sample_on_device(n_pix, n_rays) -> bool:
    return 0 < n_rays <= _hip.SAMPLE_MAX_RAYS and n_pix >= 2 * n_rays

"""ctypes binding of the nerf_hip C-ABI (include/nerf_hip.h).

This is the reference-side binding a maintainer adds to call the MI355X kernels:
every function takes torch tensors, checks dtype/device/contiguity, passes raw
device pointers plus the current HIP stream, and raises ``RuntimeError`` with the
library's message on a non-zero return code (the reference's own ops raise
``RuntimeError`` from ATen on bad shapes; same error behaviour here).

There is deliberately no CPU fallback: importing this module on a machine without
the built library, or calling into it without a GPU, fails loudly.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NERF_HIP_LIB", os.path.join(_HERE, "..", "lib", "libnerf_hip.so"))

ROW_TILE = 128
SAMPLE_MAX_RAYS = 4096      # NERF_SAMPLE_MAX_RAYS
RAYS_NORMALISE = 1          # NERF_RAYS_NORMALISE
RAYS_VIEW_ONES = 2          # NERF_RAYS_VIEW_ONES
ENC_P = 64
ENC_D = 64

_c_f = ctypes.c_float
_c_i = ctypes.c_int
_c_p = ctypes.c_void_p
_c_i64 = ctypes.c_int64


class PackDesc(ctypes.Structure):
    _fields_ = [("src", _c_p), ("dst", _c_p), ("dst_t", _c_p), ("rows", _c_i), ("cols", _c_i),
                ("ld_dst", _c_i), ("rows_t", _c_i), ("ld_t", _c_i), ("dst_s", _c_p), ("dst_ts", _c_p),
                ("rows_s", _c_i), ("dst_cs", _c_p), ("dst_cts", _c_p), ("perm_k", _c_i)]


class ProfKind(ctypes.Structure):
    """nerf_prof_kind (include/nerf_hip.h)."""
    _fields_ = [("ms", ctypes.c_double), ("launches", _c_i64), ("flops", ctypes.c_double),
                ("bytes", ctypes.c_double), ("mfma_flops", ctypes.c_double), ("exact_f32", _c_i)]


PROF_KINDS = ("fwd", "dx", "dw", "dw_narrow", "chain_fwd", "chain_bwd")   # NERF_PROF_FWD .. _CHAIN_BWD
ABI_VERSION = 15                   # NERF_HIP_ABI_VERSION


_P10 = _c_p * 10


class FieldBwd(ctypes.Structure):
    """nerf_field_bwd (include/nerf_hip.h): the native backward's arguments."""
    _fields_ = [("n_pad", _c_i), ("n_rays", _c_i), ("n_samples", _c_i), ("flags", _c_i), ("ray_grad", _c_i),
                ("tail_main", _c_i), ("bwd_chain", _c_i), ("z", _c_p), ("raw4", _c_p), ("enc_p", _c_p), ("enc_d", _c_p),
                ("enc_p_cmax", _c_p), ("enc_d_cmax", _c_p), ("act", _P10), ("mask", _P10), ("cmax", _P10),
                ("pts_o", _c_p), ("pts_d", _c_p), ("view", _c_p), ("wt", _P10), ("wt_img", _P10), ("wt_cimg", _P10),
                ("wd", _c_p),
                ("wc", _c_p), ("g_rgb", _c_p), ("g_dist", _c_p), ("graw4", _c_p), ("gw", _P10), ("gb", _P10),
                ("g_wd", _c_p), ("g_bd", _c_p), ("g_wc", _c_p), ("g_bc", _c_p), ("g_pts_o", _c_p), ("g_pts_d", _c_p),
                ("g_view", _c_p), ("workspace", _c_p)]


class WgradJob(ctypes.Structure):
    """nerf_wgrad_job (include/nerf_hip.h): one 256 x 256 layer of nerf_linear_bwd_weight_multi."""
    _fields_ = [("dy", _c_p), ("lddy", _c_i), ("x", _c_p), ("ldx", _c_i), ("slab", _c_p), ("ldslab", _c_i),
                ("bslab", _c_p), ("dy_cmax", _c_p), ("x_cmax", _c_p)]


class WgradTileJob(ctypes.Structure):
    """nerf_wgrad_tile_job (include/nerf_hip.h): one weight gradient of nerf_linear_bwd_weight_jobs."""
    _fields_ = [("dy", _c_p), ("lddy", _c_i), ("nout", _c_i), ("x", _c_p), ("ldx", _c_i), ("kin", _c_i),
                ("splits", _c_i), ("slab", _c_p), ("ldslab", _c_i), ("col0", _c_i), ("bslab", _c_p),
                ("dy_cmax", _c_p), ("x_cmax", _c_p)]


class ChainBwd(ctypes.Structure):
    """nerf_chain_bwd (include/nerf_hip.h): the input-gradient chain's arguments."""
    _fields_ = [("graw4", _c_p), ("hr_mask", _c_p), ("ld_hr_mask", _c_i), ("wd", _c_p), ("wc", _c_p),
                ("wt_img", _c_p * 9), ("wt_img_rows", _c_i * 9), ("in_mask", _c_p * 9), ("ld_in_mask", _c_i * 9),
                ("dy", _c_p * 10), ("lddy", _c_i * 10), ("dy_cmax", _c_p * 10), ("dy_rmax", _c_p * 10),
                ("scratch", _c_p), ("n_pad", _c_i)]


class ChainLayer(ctypes.Structure):
    """nerf_chain_layer (include/nerf_hip.h)."""
    _fields_ = [("img", _c_p), ("img_rows", _c_i), ("bias", _c_p), ("out", _c_p), ("ldo", _c_i), ("mask", _c_p),
                ("ldmask", _c_i), ("cmax", _c_p)]


_SIGS = {
    "nerf_hip_abi_version": ([], _c_i),
    "nerf_hip_last_error": ([], ctypes.c_char_p),
    "nerf_encode_samples": ([_c_p, _c_p, _c_p, _c_p, _c_i, _c_i, _c_i, _c_f, _c_f, _c_p, _c_p, _c_p, _c_p, _c_p,
                             _c_p, _c_p, _c_p], _c_i),
    "nerf_linear_fwd": ([_c_p, _c_i, _c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_i, _c_p, _c_p, _c_i, _c_i, _c_i, _c_i,
                         _c_p, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p], _c_i),
    "nerf_linear_fwd_heads": ([_c_p, _c_i, _c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_i, _c_p, _c_p, _c_i, _c_i, _c_i, _c_i,
                               _c_p, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i, _c_p, _c_p, _c_i, _c_p], _c_i),
    "nerf_linear_bwd_data": ([_c_p, _c_i, _c_i, _c_p, _c_p, _c_i, _c_p, _c_i, _c_p, _c_p, _c_i, _c_p, _c_i, _c_i,
                              _c_i, _c_p, _c_p, _c_p, _c_p], _c_i),
    "nerf_linear_bwd_weight": ([_c_p, _c_i, _c_i, _c_p, _c_i, _c_i, _c_i, _c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p,
                                _c_p], _c_i),
    "nerf_linear_bwd_weight_seg": ([_c_p, _c_i, _c_i, _c_p, _c_i, _c_i, _c_p, _c_i, _c_i, _c_i, _c_i, _c_p, _c_i, _c_p,
                                    _c_p, _c_p, _c_p, _c_p], _c_i),
    "nerf_linear_bwd_weight_multi": ([_c_p, _c_i, _c_i, _c_i, _c_p], _c_i),
    "nerf_linear_bwd_weight_jobs": ([_c_p, _c_i, _c_i, _c_i, _c_p], _c_i),
    "nerf_linear_bwd_weight_job_groups": ([_c_p, _c_p, _c_i, _c_i, _c_i, _c_i, _c_p], _c_i),
    "nerf_linear_bwd_weight_splits": ([_c_i, _c_i, _c_i], _c_i),
    "nerf_field_bwd_workspace_bytes": ([_c_i, _c_i], ctypes.c_size_t),
    "nerf_field_backward": ([_c_p, _c_p, _c_p], _c_i),
    "nerf_mlp_chain_bwd": ([_c_p, _c_p], _c_i),
    "nerf_slab_reduce": ([_c_p, _c_i, _c_i, _c_i, _c_i, _c_i, _c_p, _c_p, _c_p, _c_i, _c_p], _c_i),
    "nerf_heads_fwd": ([_c_p, _c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i, _c_p], _c_i),
    "nerf_heads_part_size": ([_c_i, _c_i], _c_i),
    "nerf_heads_bwd": ([_c_p, _c_p, _c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_i, _c_p, _c_i, _c_p, _c_p, _c_p], _c_i),
    "nerf_heads_bwd_mode": ([_c_i, _c_p, _c_p, _c_i, _c_p, _c_i, _c_p, _c_i, _c_i, _c_p, _c_p, _c_i, _c_p, _c_i, _c_p,
                             _c_p, _c_p], _c_i),
    "nerf_heads_reduce": ([_c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_i, _c_p], _c_i),
    "nerf_composite_fwd": ([_c_p, _c_p, _c_i, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p], _c_i),
    "nerf_composite_bwd": ([_c_p, _c_p, _c_i, _c_i, _c_i, _c_p, _c_p, _c_p, _c_i, _c_p], _c_i),
    "nerf_encode_bwd": ([_c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p], _c_i),
    "nerf_pack_weights": ([ctypes.POINTER(PackDesc), _c_i, _c_p], _c_i),
    "nerf_mlp_chain_fwd": ([_c_p, _c_p, _c_p, _c_p, _c_i, ctypes.POINTER(ChainLayer), _c_p], _c_i),
    "nerf_chain_debug_stamps": ([_c_p], _c_i),
    "nerf_chain_stamps_built": ([], _c_i),
    "nerf_mlp_chain_train": ([_c_p, _c_p, _c_p, _c_p, _c_i, ctypes.POINTER(ChainLayer), _c_p, _c_p, _c_p, _c_p, _c_p,
                              _c_p], _c_i),
    "nerf_render_eval_fused": ([_c_p, _c_p, _c_p, _c_i, _c_i, _c_f, _c_f, _c_i, ctypes.POINTER(ChainLayer), _c_p, _c_p,
                                _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p], _c_i),
    "nerf_adam_step": ([_c_p, _c_p, _c_p, _c_p, _c_i64, _c_p, _c_p], _c_i),
    "nerf_chamfer_nn": ([_c_p, _c_i, _c_p, _c_i, _c_p, _c_p], _c_i),
    "nerf_gemm_set_policy": ([_c_i, _c_i], _c_i),
    "nerf_gemm_set_precision": ([_c_i], _c_i),
    "nerf_gemm_get_precision": ([], _c_i),
    "nerf_gemm_debug_ablate": ([_c_i], _c_i),
    "nerf_gemm_debug_stamps": ([_c_p], _c_i),
    "nerf_sample_rays": ([_c_i, _c_i, ctypes.c_uint64, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p], _c_i),
    "nerf_mat4_inv": ([_c_p, _c_i, _c_p, _c_p], _c_i),
    "nerf_pose_c2w": ([_c_p, _c_p, _c_p, _c_p, _c_p], _c_i),
    "nerf_unproject_matrix": ([_c_p, _c_p, _c_p, _c_p, _c_p, _c_p], _c_i),
    "nerf_pose_c2w_bwd": ([_c_p, _c_p, _c_p, _c_p, _c_p, _c_p], _c_i),
    "nerf_mat4_inv_bwd": ([_c_p, _c_p, _c_i, _c_p, _c_p], _c_i),
    "nerf_mat4_mul": ([_c_p, _c_p, _c_i, _c_p, _c_p], _c_i),
    "nerf_mat4_mul_bwd": ([_c_p, _c_p, _c_p, _c_i, _c_p, _c_p, _c_p], _c_i),
    "nerf_unproject_matrix_bwd": ([_c_p, _c_p, _c_p, _c_p, _c_p, _c_p], _c_i),
    "nerf_depth_affine": ([_c_p, _c_i, _c_p, _c_p, _c_i, _c_f, _c_p, _c_p], _c_i),
    "nerf_depth_affine_bwd": ([_c_p, _c_i, _c_p, _c_p, _c_i, _c_f, _c_p, _c_p, _c_p, _c_p], _c_i),
    "nerf_camera_rays": ([_c_p, _c_p, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p], _c_i),
    "nerf_camera_rays_bwd": ([_c_p, _c_p, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p], _c_i),
    "nerf_ray_loss": ([_c_p, _c_p, _c_i, _c_p, _c_p, _c_p, _c_i, _c_i, _c_f, _c_f, _c_p, _c_p, _c_p, _c_p, _c_p,
                       _c_p], _c_i),
    "nerf_ray_loss_bwd": ([_c_p, _c_p, _c_i, _c_p, _c_p, _c_p, _c_i, _c_i, _c_f, _c_f, _c_p, _c_p, _c_p, _c_p,
                           _c_p, _c_p, _c_p, _c_p, _c_p], _c_i),
    "nerf_pair_workspace": ([_c_i, ctypes.POINTER(_c_i), ctypes.POINTER(_c_i64)], _c_i),
    "nerf_pair_forward": ([_c_p, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_f, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p], _c_i),
    "nerf_pair_backward": ([_c_p, _c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_f, _c_p, _c_p, _c_i, _c_p, _c_p, _c_p,
                            _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p], _c_i),
    "nerf_prof_enable": ([_c_i], _c_i),
    "nerf_prof_read_kinds": ([ctypes.POINTER(ProfKind), _c_i], _c_i),
    "nerf_prof_read": ([ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_c_i64),
                        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)], _c_i),
}

EXPORTED_SYMBOLS = tuple(_SIGS)


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise ImportError(
            f"nerf_hip: HIP library not found at {path}; build it with `make -C my-nope-nerf_amd` "
            "(or __graft_entry__.build()). There is no CPU fallback.")
    lib = ctypes.CDLL(path)
    lib.nerf_hip_abi_version.restype = _c_i
    ver = lib.nerf_hip_abi_version()
    if ver != ABI_VERSION:
        # signatures change between ABI versions (v4 added nerf_sample_rays' seed_counter);
        # calling a stale library through these argtypes would pass mismatched arguments
        raise ImportError(f"nerf_hip: {path} has ABI version {ver}, this binding needs {ABI_VERSION}; "
                          "rebuild it with `make -C my-nope-nerf_amd`")
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    return lib


_lib: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        _lib = load_library()
    return _lib


_fns = {}


def _call(name: str, *args):
    fn = _fns.get(name)
    if fn is None:
        fn = _fns[name] = getattr(lib(), name)
    rc = fn(*args)
    if rc != 0:
        msg = lib().nerf_hip_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed ({rc}): {msg}")


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("nerf_hip: tensor must live on the GPU (no CPU fallback)")
    if t.dtype not in (torch.float32, torch.int64, torch.int32, torch.int16, torch.uint8, torch.bool):
        raise RuntimeError(f"nerf_hip: unsupported dtype {t.dtype}")
    return t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_dev = getattr(torch._C, "_cuda_getDevice", None)


def _stream() -> int:
    """The current HIP stream of the current device (the raw handle: constructing a
    torch.cuda.Stream per launch cost ~10 us of host time)."""
    if _raw_stream is not None and _cur_dev is not None:
        return _raw_stream(_cur_dev())
    return torch.cuda.current_stream().cuda_stream


def _ld(t: torch.Tensor) -> int:
    """Row stride (elements) of a 2-D row-major view (columns contiguous)."""
    if t.dim() != 2 or t.stride(1) != 1:
        raise RuntimeError("nerf_hip: expected a 2-D row-major view")
    return t.stride(0)


# --------------------------------------------------------------------------------------
def encode_samples(pts_o, pts_d, view, noise, n_rays, n_samples, n_pad, near, far, z, enc_p, enc_d,
                   enc_p_rmax=None, enc_d_rmax=None, enc_p_cmax=None, enc_d_cmax=None):
    """enc_p_rmax / enc_d_rmax: optional [n_pad] outputs, max |.| per encoding row (the row
    scales GEMM precision mode 2 needs); enc_p_cmax / enc_d_cmax: optional [n_pad/128][64]
    column bounds per 128-row group (its column scales)."""
    _call("nerf_encode_samples", _ptr(pts_o), _ptr(pts_d), _ptr(view), _ptr(noise), n_rays, n_samples,
          n_pad, float(near), float(far), _ptr(z), _ptr(enc_p), _ptr(enc_d), _ptr(enc_p_rmax), _ptr(enc_d_rmax),
          _ptr(enc_p_cmax), _ptr(enc_d_cmax), _stream())


def _split_args(ws):
    """bf16x3 image view [3][K/8][rows][8] (int16, rows may be a slice) -> (ptr, image rows)."""
    if ws is None:
        return None, 0
    if ws.dim() != 4 or ws.shape[0] != 3 or ws.shape[3] != 8 or ws.stride(2) != 8 or ws.stride(3) != 1:
        raise ValueError("split weight image must be a [3][K/8][rows][8] view with contiguous rows")
    return _ptr(ws), ws.stride(1) // 8


def split_image(rows: int, k: int, device) -> "torch.Tensor":
    """Zeroed bf16x3 image buffer for a [rows][k] operand (nerf_pack_desc.dst_s layout); in
    GEMM precision mode 2 the pack writes the fp16 pair form into the same buffer."""
    return torch.zeros(3, k // 8, rows, 8, dtype=torch.int16, device=device)


def linear_fwd(x1, k1, x2, k2, w, bias, y, m, n, relu, mask_out=None, w_split=None, x1_rmax=None, x2_rmax=None,
               y_rmax=None, y_cmax=None, heads=None):
    """mask_out: int32 [m][n/32] ReLU mask bits of y (optional).  w_split: optional split
    image of w (used by GEMM precision modes 1 and 2).  x1_rmax / x2_rmax: max |x| per row of
    each input segment (required in mode 2); y_rmax: optional [m] output, max |y| per row;
    y_cmax: optional [m/128][n] output, max |y| per column and 128-row group (mode 2).
    heads: optional (head_w [nh][n], head_b [nh], raw4 [m][4], raw_col) -- the output heads
    fused into the epilogue (nerf_linear_fwd_heads, mode 2)."""
    wsp, wsr = _split_args(w_split)
    args = (_ptr(x1), _ld(x1), k1, _ptr(x2), _ld(x2) if x2 is not None else 0, k2,
            _ptr(w), wsp, wsr, _ptr(bias), _ptr(y), _ld(y), m, n, int(relu), _ptr(mask_out),
            _ld(mask_out) if mask_out is not None else 0, _ptr(x1_rmax), _ptr(x2_rmax), _ptr(y_rmax), _ptr(y_cmax))
    if heads is None:
        _call("nerf_linear_fwd", *args, _stream())
    else:
        hw, hb, raw4, col = heads
        _call("nerf_linear_fwd_heads", *args, _ptr(hw), hw.shape[0], _ptr(hb), _ptr(raw4), int(col), _stream())


def linear_bwd_data(dy, k, wt, dx, m, n, mask=None, u=None, ldu=1, v=None, wt_split=None, dy_rmax=None,
                    dx_rmax=None, dx_cmax=None):
    """mask: int32 ReLU mask bits [m][words] from linear_fwd(mask_out=...).  dy_rmax / dx_rmax /
    dx_cmax: row and column maxima as x1_rmax / y_rmax / y_cmax of linear_fwd."""
    wsp, wsr = _split_args(wt_split)
    _call("nerf_linear_bwd_data", _ptr(dy), _ld(dy), k, _ptr(wt), wsp, wsr, _ptr(u), int(ldu), _ptr(v), _ptr(mask),
          _ld(mask) if mask is not None else 0, _ptr(dx), _ld(dx), m, n, _ptr(dy_rmax), _ptr(dx_rmax), _ptr(dx_cmax),
          _stream())


def linear_bwd_weight(dy, nout, x, kin, m, splits, slab, ldslab, col0, bslab, dy_cmax=None, x_cmax=None):
    """dy_cmax [m/128][nout] / x_cmax [m/128][kin]: column bounds per 128-row group; with both,
    precision mode 2 runs the fp16 pair kernel."""
    _call("nerf_linear_bwd_weight", _ptr(dy), _ld(dy), nout, _ptr(x), _ld(x), kin, m, splits,
          _ptr(slab), ldslab, col0, _ptr(bslab), _ptr(dy_cmax), _ptr(x_cmax), _stream())


def linear_bwd_weight_seg(dy, nout, x1, k1, x2, k2, m, splits, slab, ldslab, bslab, dy_cmax=None, x1_cmax=None,
                          x2_cmax=None):
    """Weight gradient of a layer whose input is [x1 | x2] (l4, the colour layer): slab columns
    [0, k1) from x1 and [k1, k1 + k2) from x2 -- in mode 2 one launch reading dy once."""
    _call("nerf_linear_bwd_weight_seg", _ptr(dy), _ld(dy), nout, _ptr(x1), _ld(x1), k1, _ptr(x2), _ld(x2), k2, m,
          splits, _ptr(slab), ldslab, _ptr(bslab), _ptr(dy_cmax), _ptr(x1_cmax), _ptr(x2_cmax), _stream())


def linear_bwd_weight_multi(layers, m, splits):
    """Several 256 x 256 weight gradients in one launch (mode 2, TN policy 8): layers is a list of
    (dy, x, slab, bslab, dy_cmax, x_cmax), each as linear_bwd_weight(dy, 256, x, 256, m, splits,
    slab, 256, 0, bslab, dy_cmax, x_cmax) would write it."""
    jobs = (WgradJob * len(layers))()
    for j, (dy, x, slab, bslab, dcm, xcm) in zip(jobs, layers):
        j.dy, j.lddy, j.x, j.ldx = _ptr(dy), _ld(dy), _ptr(x), _ld(x)
        j.slab, j.ldslab, j.bslab, j.dy_cmax, j.x_cmax = _ptr(slab), 256, _ptr(bslab), _ptr(dcm), _ptr(xcm)
    _call("nerf_linear_bwd_weight_multi", ctypes.addressof(jobs), len(layers), m, splits, _stream())


def linear_bwd_weight_jobs(jobs, m, splits, groups=None):
    """Weight gradients of several shapes in one launch of 2 * splits blocks (mode 2, TN policy 8):
    jobs is a list of (dy, nout, x, kin, job_splits, slab, ldslab, col0, bslab, dy_cmax, x_cmax), each
    as linear_bwd_weight(dy, nout, x, kin, m, job_splits, slab, ldslab, col0, bslab, dy_cmax, x_cmax)
    would write it.  groups (a list of block-group ids, one per job): the launch runs max + 1 groups
    of 2 * splits blocks side by side (nerf_linear_bwd_weight_job_groups)."""
    arr = (WgradTileJob * len(jobs))()
    for j, (dy, nout, x, kin, sp, slab, ldslab, col0, bslab, dcm, xcm) in zip(arr, jobs):
        j.dy, j.lddy, j.nout, j.x, j.ldx, j.kin, j.splits = _ptr(dy), _ld(dy), nout, _ptr(x), _ld(x), kin, sp
        j.slab, j.ldslab, j.col0, j.bslab, j.dy_cmax, j.x_cmax = _ptr(slab), ldslab, col0, _ptr(bslab), _ptr(dcm), _ptr(xcm)
    if groups is None:
        _call("nerf_linear_bwd_weight_jobs", ctypes.addressof(arr), len(jobs), m, splits, _stream())
        return
    grp = (ctypes.c_int * len(jobs))(*groups)
    _call("nerf_linear_bwd_weight_job_groups", ctypes.addressof(arr), ctypes.addressof(grp), len(jobs), m, splits,
          max(groups) + 1, _stream())


def bwd_weight_splits(nout, kin, m) -> int:
    return int(lib().nerf_linear_bwd_weight_splits(nout, kin, m))


def slab_reduce(slab, splits, nout, ldslab, nout_ref, kin_ref, bslab, gw, gb, accumulate=False):
    _call("nerf_slab_reduce", _ptr(slab), splits, nout, ldslab, nout_ref, kin_ref, _ptr(bslab), _ptr(gw),
          _ptr(gb), int(accumulate), _stream())


def field_bwd_workspace_bytes(n_pad, ray_grad) -> int:
    return int(lib().nerf_field_bwd_workspace_bytes(n_pad, int(ray_grad)))


def field_backward(args: FieldBwd, side_stream: int):
    """The training backward of the D = 256 field in one call (nerf_field_backward) on the
    current stream + `side_stream` (a raw HIP stream handle)."""
    _call("nerf_field_backward", ctypes.addressof(args), _stream(), side_stream)


def mlp_chain_bwd(args: ChainBwd):
    """dyr and the nine input gradients of the D = 256 field in one launch (nerf_mlp_chain_bwd)."""
    _call("nerf_mlp_chain_bwd", ctypes.addressof(args), _stream())


def heads_fwd(h8, hr, hidden, wd, bd, wc, bc, raw4, n_pad):
    _call("nerf_heads_fwd", _ptr(h8), _ld(h8), _ptr(hr), _ld(hr), hidden, _ptr(wd), _ptr(bd), _ptr(wc),
          _ptr(bc), _ptr(raw4), n_pad, _stream())


def heads_part_size(hidden, n_pad) -> int:
    return int(lib().nerf_heads_part_size(hidden, n_pad))


def heads_bwd(graw4, h8, hr, hidden, wc, dyr, part, n_pad, dyr_rmax=None, dyr_cmax=None, mode=3, hr_mask=None):
    """mode 1: dyr (+ maxima) only; 2: head-weight partials only; 3: both (nerf_heads_bwd_mode).
    hr_mask (mode 1): the colour layer's ReLU bits [n][k] int32 gate dyr instead of hr."""
    if mode == 3 and hr_mask is None:
        _call("nerf_heads_bwd", _ptr(graw4), _ptr(h8), _ld(h8), _ptr(hr), _ld(hr), hidden, _ptr(wc), _ptr(dyr),
              _ld(dyr), _ptr(part), n_pad, _ptr(dyr_rmax), _ptr(dyr_cmax), _stream())
    else:
        _call("nerf_heads_bwd_mode", int(mode), _ptr(graw4), _ptr(h8), _ld(h8) if h8 is not None else 0,
              _ptr(hr), _ld(hr) if hr is not None else 0, _ptr(hr_mask), _ld(hr_mask) if hr_mask is not None else 0,
              hidden, _ptr(wc), _ptr(dyr), _ld(dyr) if dyr is not None else 0, _ptr(part), n_pad, _ptr(dyr_rmax),
              _ptr(dyr_cmax), _stream())


def heads_reduce(part, hidden, n_pad, gwd, gbd, gwc, gbc, accumulate=False):
    _call("nerf_heads_reduce", _ptr(part), hidden, n_pad, _ptr(gwd), _ptr(gbd), _ptr(gwc), _ptr(gbc),
          int(accumulate), _stream())


def composite_fwd(raw4, z, n_rays, n_samples, flags, rgb, dist, alpha):
    _call("nerf_composite_fwd", _ptr(raw4), _ptr(z), n_rays, n_samples, flags, _ptr(rgb), _ptr(dist),
          _ptr(alpha), _stream())


def composite_bwd(raw4, z, n_rays, n_samples, flags, g_rgb, g_dist, graw4, n_pad):
    _call("nerf_composite_bwd", _ptr(raw4), _ptr(z), n_rays, n_samples, flags, _ptr(g_rgb), _ptr(g_dist),
          _ptr(graw4), n_pad, _stream())


def encode_bwd(pts_o, pts_d, view, z, genc_p, genc_d, n_rays, n_samples, g_po, g_pd, g_view, genc_p2=None):
    _call("nerf_encode_bwd", _ptr(pts_o), _ptr(pts_d), _ptr(view), _ptr(z), _ptr(genc_p), _ptr(genc_p2),
          _ptr(genc_d), n_rays, n_samples, _ptr(g_po), _ptr(g_pd), _ptr(g_view), _stream())


def pack_weights(descs: Sequence[PackDesc]):
    arr = (PackDesc * len(descs))(*descs)
    _call("nerf_pack_weights", arr, len(descs), _stream())


def render_eval_fused(pts_o, pts_d, view, R, S, near, far, flags, layers: Sequence[ChainLayer], wd, bd, wc, bc,
                      rgb, dist, alpha, z):
    """The fused per-ray eval render (one launch: samples, encodings, ten linears, heads,
    composite; GEMM precision mode 2, hidden 256, S >= 2 dividing 128)."""
    if len(layers) != 10:
        raise ValueError("render_eval_fused: needs the 10 layer descriptors")
    for t in (pts_o, pts_d, view, wd, bd, wc, bc, rgb, dist, alpha, z):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise RuntimeError("render_eval_fused: float32 contiguous tensors expected")
    arr = (ChainLayer * 10)(*layers)
    _call("nerf_render_eval_fused", _ptr(pts_o), _ptr(pts_d), _ptr(view), int(R), int(S), float(near), float(far),
          int(flags), arr, _ptr(wd), _ptr(bd), _ptr(wc), _ptr(bc), _ptr(rgb), _ptr(dist), _ptr(alpha), _ptr(z),
          _stream())


def mlp_chain_fwd(enc_p, enc_d, enc_p_rmax, enc_d_rmax, n_pad, layers: Sequence[ChainLayer]):
    """All ten field linears in one launch (GEMM precision mode 2, hidden 256 / colour 128)."""
    if len(layers) != 10:
        raise ValueError("mlp_chain_fwd: needs the 10 layer descriptors")
    arr = (ChainLayer * 10)(*layers)
    _call("nerf_mlp_chain_fwd", _ptr(enc_p), _ptr(enc_d), _ptr(enc_p_rmax), _ptr(enc_d_rmax), int(n_pad), arr,
          _stream())


def mlp_chain_train(enc_p, enc_d, enc_p_rmax, enc_d_rmax, n_pad, layers: Sequence[ChainLayer], wd, bd, wc, bc,
                    raw4):
    """The training forward chain (one launch at two waves per SIMD): every layer output,
    ReLU words and column maxima the backward needs, plus raw4 from the in-epilogue heads."""
    if len(layers) != 10:
        raise ValueError("mlp_chain_train: needs the 10 layer descriptors")
    arr = (ChainLayer * 10)(*layers)
    _call("nerf_mlp_chain_train", _ptr(enc_p), _ptr(enc_d), _ptr(enc_p_rmax), _ptr(enc_d_rmax), int(n_pad), arr,
          _ptr(wd), _ptr(bd), _ptr(wc), _ptr(bc), _ptr(raw4), _stream())


def adam_step(param, grad, exp_avg, exp_avg_sq, hyper):
    """hyper: device float32 [16] (model.optim.hyper_block: step, lr, beta1, beta2, eps,
    weight_decay, 1 - beta2, ticket, lr / beta1 / beta2 as doubles, 1 - beta1, flag); the update
    uses step + 1 and stores it back (ticket: zero-initialised counter)."""
    if hyper.numel() < 16 or hyper.dtype != torch.float32:
        raise ValueError("adam_step: hyper needs 16 float32 slots (ABI 13)")
    _call("nerf_adam_step", _ptr(param), _ptr(grad), _ptr(exp_avg), _ptr(exp_avg_sq), param.numel(),
          _ptr(hyper), _stream())


def sample_rays(n_pix, n_rays, seed, width, height, img, idx, pixels=None, rgb=None, status=None, seed_counter=None):
    """seed_counter: optional device int64 [1], mixed into the key and advanced on the device
    (graph replays draw new rays)."""
    _call("nerf_sample_rays", int(n_pix), int(n_rays), int(seed) & 0xFFFFFFFFFFFFFFFF, int(width), int(height),
          _ptr(img), _ptr(idx), _ptr(pixels), _ptr(rgb), _ptr(status), _ptr(seed_counter), _stream())


def mat4_inv(a, out):
    _call("nerf_mat4_inv", _ptr(a), a.numel() // 16, _ptr(out), _stream())


def pose_c2w(r, t, init_c2w, out):
    _call("nerf_pose_c2w", _ptr(r), _ptr(t), _ptr(init_c2w), _ptr(out), _stream())


def unproject_matrix(K, world, scale, M, inverses=None):
    _call("nerf_unproject_matrix", _ptr(K), _ptr(world), _ptr(scale), _ptr(M), _ptr(inverses), _stream())


def pose_c2w_bwd(r, init_c2w, g_c2w, g_r=None, g_t=None):
    _call("nerf_pose_c2w_bwd", _ptr(r), _ptr(init_c2w), _ptr(g_c2w), _ptr(g_r), _ptr(g_t), _stream())


def mat4_inv_bwd(inv_a, g, g_a):
    _call("nerf_mat4_inv_bwd", _ptr(inv_a), _ptr(g), inv_a.numel() // 16, _ptr(g_a), _stream())


def mat4_mul(a, b, c):
    _call("nerf_mat4_mul", _ptr(a), _ptr(b), a.numel() // 16, _ptr(c), _stream())


def mat4_mul_bwd(a, b, g, g_a=None, g_b=None):
    _call("nerf_mat4_mul_bwd", _ptr(a), _ptr(b), _ptr(g), g.numel() // 16, _ptr(g_a), _ptr(g_b), _stream())


def depth_affine(d, scale, shift, shift_first, lo, y):
    _call("nerf_depth_affine", _ptr(d), d.numel(), _ptr(scale), _ptr(shift), int(shift_first), float(lo), _ptr(y),
          _stream())


def depth_affine_bwd(d, scale, shift, shift_first, lo, g, g_scale=None, g_shift=None):
    _call("nerf_depth_affine_bwd", _ptr(d), d.numel(), _ptr(scale), _ptr(shift), int(shift_first), float(lo), _ptr(g),
          _ptr(g_scale), _ptr(g_shift), _stream())


def unproject_matrix_bwd(inverses, g_M, g_K=None, g_world=None, g_scale=None):
    _call("nerf_unproject_matrix_bwd", _ptr(inverses), _ptr(g_M), _ptr(g_K), _ptr(g_world), _ptr(g_scale), _stream())


def camera_rays(M, pixels, depth, n_rays, flags, cam, ray, view, ray_norm, d_src, mask):
    _call("nerf_camera_rays", _ptr(M), _ptr(pixels), _ptr(depth), int(n_rays), int(flags), _ptr(cam), _ptr(ray),
          _ptr(view), _ptr(ray_norm), _ptr(d_src), _ptr(mask), _stream())


def camera_rays_bwd(M, pixels, depth, n_rays, flags, g_cam, g_ray, g_view, g_norm, g_dsrc, gM, g_depth):
    _call("nerf_camera_rays_bwd", _ptr(M), _ptr(pixels), _ptr(depth), int(n_rays), int(flags), _ptr(g_cam),
          _ptr(g_ray), _ptr(g_view), _ptr(g_norm), _ptr(g_dsrc), _ptr(gM), _ptr(g_depth), _stream())


def ray_loss(rgb, rgb_gt, n_rays, depth_pred, depth_gt, mask, n_depth, rgb_l1, w_rgb, w_depth, out, cnt):
    """out: four device scalars (total, l_rgb, l_depth, l2_mean)."""
    _call("nerf_ray_loss", _ptr(rgb), _ptr(rgb_gt), int(n_rays), _ptr(depth_pred), _ptr(depth_gt), _ptr(mask),
          int(n_depth), int(rgb_l1), float(w_rgb), float(w_depth), *[_ptr(o) for o in out], _ptr(cnt), _stream())


def ray_loss_bwd(rgb, rgb_gt, n_rays, depth_pred, depth_gt, mask, n_depth, rgb_l1, w_rgb, w_depth, go, cnt,
                 g_rgb, g_dp, g_dg):
    """go: four upstream scalars (total, l_rgb, l_depth, l2_mean), each a device tensor or None."""
    _call("nerf_ray_loss_bwd", _ptr(rgb), _ptr(rgb_gt), int(n_rays), _ptr(depth_pred), _ptr(depth_gt),
          _ptr(mask), int(n_depth), int(rgb_l1), float(w_rgb), float(w_depth), *[_ptr(g) for g in go], _ptr(cnt),
          _ptr(g_rgb), _ptr(g_dp), _ptr(g_dg), _stream())


def pair_workspace(n_points):
    """-> (chamfer chunks, workspace floats) of nerf_pair_forward at n_points."""
    nc = _c_i()
    fl = _c_i64()
    _call("nerf_pair_workspace", int(n_points), ctypes.byref(nc), ctypes.byref(fl))
    return nc.value, fl.value


def pair_forward(d1, d2, h, w, K, Rt, s1, nl, img1, img2, work, nn, out3):
    _call("nerf_pair_forward", _ptr(d1), _ptr(d2), int(h), int(w), _ptr(K), _ptr(Rt), _ptr(s1), float(nl),
          _ptr(img1), _ptr(img2), _ptr(work), _ptr(nn), _ptr(out3), _stream())


def pair_backward(d1, d2, h, w, K, Rt, s1, nl, img1, img2, rgbs_detach_scale, work, nn, out3, go_pc, go_rgbs,
                  gxy, g_d1, g_d2, g13, part13):
    _call("nerf_pair_backward", _ptr(d1), _ptr(d2), int(h), int(w), _ptr(K), _ptr(Rt), _ptr(s1), float(nl),
          _ptr(img1), _ptr(img2), int(rgbs_detach_scale), _ptr(work), _ptr(nn), _ptr(out3), _ptr(go_pc),
          _ptr(go_rgbs), _ptr(gxy), _ptr(g_d1), _ptr(g_d2), _ptr(g13), _ptr(part13), _stream())


def chamfer_nn(x, y, idx):
    _call("nerf_chamfer_nn", _ptr(x), x.shape[0], _ptr(y), y.shape[0], _ptr(idx), _stream())


def gemm_set_policy(nt: int = 0, tn: int = 0):
    _call("nerf_gemm_set_policy", int(nt), int(tn))


def gemm_set_precision(mode):
    """0 = exact-f32 MFMA, 1 = f32 emulated on bf16 MFMA (3-word split, 6 products),
    2 = f32 emulated on fp16 MFMA (row / column-scaled 2-word split, 3 products; the library
    default, the benchmarked path and the one the fused eval kernel runs).  All three are
    f32-accurate."""
    _call("nerf_gemm_set_precision", int(mode))


def gemm_get_precision():
    return int(lib().nerf_gemm_get_precision())


def prof_enable(on: bool):
    _call("nerf_prof_enable", int(on))


def prof_read_kinds():
    """Per-kind GEMM records since prof_enable (call before prof_read, which resets them):
    {"fwd"|"dx"|"dw"|"dw_narrow"|"chain_fwd"|"chain_bwd": {ms, launches, flops, bytes, mfma_flops,
    exact_f32}}."""
    arr = (ProfKind * len(PROF_KINDS))()
    _call("nerf_prof_read_kinds", arr, len(PROF_KINDS))
    return {name: {f: getattr(arr[i], f) for f, _ in ProfKind._fields_} for i, name in enumerate(PROF_KINDS)}


def prof_read():
    """-> (summed GEMM launch ms, launches, padded FLOPs, union-of-intervals ms)."""
    ms = ctypes.c_double()
    n = _c_i64()
    fl = ctypes.c_double()
    un = ctypes.c_double()
    _call("nerf_prof_read", ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl), ctypes.byref(un))
    return ms.value, n.value, fl.value, un.value

"""The C-ABI library loads and exports every symbol include/nerf_hip.h declares; the
ctypes binding covers all of them; argument checks fail loudly (no GPU needed: these
calls return before any HIP API call)."""
import ctypes
import os
import re

import pytest

from model import _hip

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "nerf_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nerf_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_hip.LIB_PATH):
        pytest.fail(f"library not built at {_hip.LIB_PATH}; run __graft_entry__.build()")
    return _hip.load_library()


def test_every_declared_symbol_is_exported(lib):
    names = _declared()
    assert len(names) >= 18
    for n in names:
        assert hasattr(lib, n), f"{n} declared in nerf_hip.h but not exported"


def test_binding_covers_the_header():
    assert sorted(_hip.EXPORTED_SYMBOLS) == _declared()


def test_abi_version_and_error_path(lib):
    assert lib.nerf_hip_abi_version() == 15
    rc = lib.nerf_linear_fwd(None, 256, 256, None, 0, 0, None, None, 0, None, None, 256, 128, 256, 1, None, 0,
                             None, None, None, None, None)
    assert rc == -1
    assert b"null" in lib.nerf_hip_last_error()
    rc = lib.nerf_linear_bwd_weight(1, 256, 100, 1, 256, 256, 1024, 4, 1, 256, 0, None, None, None, None)
    assert rc == -1 and b"nout" in lib.nerf_hip_last_error()
    rc = lib.nerf_composite_fwd(None, None, 1, 1, 0, None, None, None, None)
    assert rc == -1
    # ray prologue: sampler size limits, camera rays without outputs
    rc = lib.nerf_sample_rays(100, 80, 1, 10, 10, None, 1, None, None, None, None, None)
    assert rc == -1 and b"2*n_rays" in lib.nerf_hip_last_error()
    rc = lib.nerf_sample_rays(10 ** 6, 5000, 1, 1000, 1000, None, 1, None, None, None, None, None)
    assert rc == -1 and b"n_rays" in lib.nerf_hip_last_error()
    rc = lib.nerf_camera_rays(1, 1, None, 4, 1, None, 1, None, 1, 1, None, None)
    assert rc == -1 and b"cam" in lib.nerf_hip_last_error()
    # several weight gradients in one launch: 1..8 layers, each job checked before any launch
    import ctypes
    from model import _hip
    jobs = (_hip.WgradJob * 9)()
    rc = lib.nerf_linear_bwd_weight_multi(ctypes.addressof(jobs), 9, 131072, 128, None)
    assert rc == -1 and b"layers" in lib.nerf_hip_last_error()
    rc = lib.nerf_linear_bwd_weight_multi(ctypes.addressof(jobs), 0, 131072, 128, None)
    assert rc == -1
    rc = lib.nerf_linear_bwd_weight_multi(None, 2, 131072, 128, None)
    assert rc == -1
    tjobs = (_hip.WgradTileJob * 9)()
    rc = lib.nerf_linear_bwd_weight_jobs(ctypes.addressof(tjobs), 9, 131072, 128, None)
    assert rc == -1 and b"jobs" in lib.nerf_hip_last_error()
    rc = lib.nerf_linear_bwd_weight_jobs(None, 2, 131072, 128, None)
    assert rc == -1


def test_ops_refuse_cpu_tensors(lib):
    import torch
    x = torch.zeros(128, 64)
    with pytest.raises(RuntimeError, match="GPU"):
        _hip.linear_fwd(x, 64, None, 0, torch.zeros(64, 64), None, torch.zeros(128, 64), 128, 64, 1)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(ImportError, match="no CPU fallback"):
        _hip.load_library(str(tmp_path / "nope.so"))


def test_chain_image_descriptor_checks(lib):
    """ABI 13 chain images (nerf_pack_desc dst_cs / dst_cts): rejected outside precision mode 2
    or with perm_k not a multiple of 32 -- argument checks only, no launch."""
    src = ctypes.c_void_p(16)
    old = lib.nerf_gemm_get_precision()
    try:
        lib.nerf_gemm_set_precision(2)
        d = _hip.PackDesc(src, src, None, 256, 256, 256, 0, 0, src, None, 256, src, None, 48)
        assert lib.nerf_pack_weights(ctypes.byref(d), 1, None) == -1
        assert b"perm_k" in lib.nerf_hip_last_error()
        lib.nerf_gemm_set_precision(0)
        d = _hip.PackDesc(src, src, None, 256, 256, 256, 0, 0, None, None, 256, src, None, 256)
        assert lib.nerf_pack_weights(ctypes.byref(d), 1, None) == -1
        assert b"mode 2" in lib.nerf_hip_last_error()
    finally:
        lib.nerf_gemm_set_precision(old)

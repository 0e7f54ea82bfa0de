import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "my-nope-nerf_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the nerf_hip C-ABI)")


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(params=[0, 1, 2], ids=["f32mfma", "bf16x6", "f16x3"])
def gemm_precision(request, dev):
    """Run a GPU test under every GEMM arithmetic mode (nerf_gemm_set_precision)."""
    from model import _hip
    old = _hip.gemm_get_precision()
    _hip.gemm_set_precision(request.param)
    yield request.param
    _hip.gemm_set_precision(old)


@pytest.fixture(autouse=True)
def _restore_gemm_state(request):
    """Every GPU test leaves the process-wide GEMM precision and tile policy as it found them
    (the library default is precision mode 2, the fp16 pair)."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    import torch
    if not torch.cuda.is_available():
        yield
        return
    from model import _hip
    old = _hip.gemm_get_precision()
    yield
    _hip.gemm_set_precision(old)
    _hip.gemm_set_policy(0, 0)

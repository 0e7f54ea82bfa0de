"""The native field backward (nerf_field_backward, csrc/field_bwd.cpp) against the Python
schedule it replaces (FieldRunner.backward with NERF_NATIVE_BWD=0).  With the per-layer
input gradients (NERF_BWD_CHAIN=0) it runs the same kernels in the same order, so every
parameter gradient and every ray gradient must be bit-identical; with the input-gradient
chain (nerf_mlp_chain_bwd, the default) the input gradients accumulate in another MFMA order
(16x16x32 tiles, K in chain order), so the gradients agree to 1e-5 relative L2 per tensor.
Training-size batches (Np >= 65536, where the native path runs), with and without ray
gradients (pose learning), from the composite backward and from a given graw4
(eval_points); the per-layer schedule also under a tail of 0 and 3 deferred weight gradients
(tail_main applies to it only), and the chain under both weight-gradient schedules
(NERF_WGRAD_SCHED 1 / 2 / 3; 3 also with NERF_WGRAD_GROUPS 0 / 1 besides its default 2)."""
import os

import pytest
import torch

from model import _hip
from model.field import eval_points, render_field
from model.official_nerf import OfficialStaticNerf
from tests.helpers import make_cfg

pytestmark = pytest.mark.gpu


@pytest.fixture
def h16(dev):
    old = _hip.gemm_get_precision()
    _hip.gemm_set_precision(2)
    yield
    _hip.gemm_set_precision(old)


def _net(dev, seed):
    torch.manual_seed(seed)
    return OfficialStaticNerf(make_cfg(hidden=256, S=128)).to(dev)


def _rays(R, S, seed):
    g = torch.Generator().manual_seed(seed)
    o = (torch.rand(R, 3, generator=g) - 0.5) * 4
    d = torch.nn.functional.normalize(torch.rand(R, 3, generator=g) - 0.5, dim=-1)
    return o, d, torch.rand(R, S, generator=g)


def _grads(net, fn, native, env=None):
    env = dict(env or {})
    old = {k: os.environ.get(k) for k in ("NERF_NATIVE_BWD", *env)}
    os.environ["NERF_NATIVE_BWD"] = "1" if native else "0"
    os.environ.update(env)
    try:
        net.zero_grad(set_to_none=True)
        extra = fn()
        torch.cuda.synchronize()
        return [p.grad.clone() for p in net.parameters()] + [t.grad.clone() for t in extra]
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _agree(a, b, chain):
    assert torch.isfinite(a).all()
    if chain == "0":
        assert torch.equal(a, b)
    else:
        scale = b.norm().item()
        assert (a - b).norm().item() <= 1e-5 * scale + 1e-30, (a - b).norm().item() / max(scale, 1e-30)
        assert (a - b).abs().max().item() <= 1e-4 * b.abs().max().item() + 1e-30


@pytest.mark.parametrize("chain,sched", [("0", "1"), ("1", "1"), ("1", "2"), ("1", "3"), ("1", "3g0"), ("1", "3g1")])
@pytest.mark.parametrize("ray_grad,R,S,tail", [(False, 1024, 128, None), (True, 1024, 128, None),
                                               (False, 600, 128, "0"), (True, 520, 128, "3")])
def test_native_backward_bit_identical(dev, h16, ray_grad, R, S, tail, chain, sched):
    if chain == "1" and tail is not None:
        pytest.skip("tail_main applies to the per-layer schedule only (nerf_field_bwd)")
    net = _net(dev, seed=R)
    o, d, noise = _rays(R, S, seed=R + 1)
    runner = net.hip_runner()

    def fn():
        oo = o.to(dev).requires_grad_(ray_grad)
        dd = d.to(dev).requires_grad_(ray_grad)
        rgb, dist, _, _ = render_field(net, oo, dd, -dd, noise.to(dev), 0.01, 10.0, S, 0)
        (rgb.square().sum() + 0.1 * dist.sum()).backward()
        return [oo, dd] if ray_grad else []

    env = {"NERF_TAIL_MAIN": tail} if tail is not None else {}
    env["NERF_BWD_CHAIN"] = chain
    env["NERF_WGRAD_SCHED"] = sched[0]   # the chain's weight-gradient schedules (field_bwd.cpp)
    if len(sched) > 1:                   # schedule 3's block groups: none / the second launch (default: both)
        env["NERF_WGRAD_GROUPS"] = sched[2:]
    g_native = _grads(net, fn, True, env)
    g_python = _grads(net, fn, False, env)
    n_pad = (R * S + 127) // 128 * 128
    assert n_pad >= 65536 and runner.native_backward(n_pad)
    for a, b in zip(g_native, g_python):
        _agree(a, b, chain)


@pytest.mark.parametrize("chain", ["0", "1"])
def test_native_backward_from_raw_heads(dev, h16, chain):
    """eval_points (FieldRawFn): the backward starts from a given graw4, no composite."""
    net = _net(dev, seed=3)
    n = 70000
    g = torch.Generator().manual_seed(4)
    p = ((torch.rand(n, 3, generator=g) - 0.5) * 3).to(dev)
    v = torch.nn.functional.normalize(torch.rand(n, 3, generator=g) - 0.5, dim=-1).to(dev)

    def fn():
        pp = p.clone().requires_grad_(True)
        vv = v.clone().requires_grad_(True)
        raw = eval_points(net, pp, vv)
        (raw[:, 0].square().sum() + raw[:, 1:].sum()).backward()
        return [pp, vv]

    g_native = _grads(net, fn, True, {"NERF_BWD_CHAIN": chain})
    g_python = _grads(net, fn, False, {"NERF_BWD_CHAIN": chain})
    for a, b in zip(g_native, g_python):
        _agree(a, b, chain)


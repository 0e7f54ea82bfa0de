"""Fused layer chain (nerf_mlp_chain_fwd) vs one launch per layer at the cfg2 shape
(1024 rays x 128 samples, hidden 256), GEMM precision mode 2, plus the chain's per-block
phase cycles (nerf_chain_debug_stamps).

    python scripts/chain_bench.py
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from model import _hip  # noqa: E402
from model.official_nerf import OfficialStaticNerf  # noqa: E402
from model.synthetic import make_cfg  # noqa: E402


def main():
    dev = torch.device("cuda")
    _hip.gemm_set_precision(2)
    torch.manual_seed(0)
    net = OfficialStaticNerf(make_cfg(hidden=256, S=128)).to(dev)
    R, S = 1024, 128
    o = (torch.rand(R, 3, device=dev) - 0.5) * 4
    d = torch.nn.functional.normalize(torch.rand(R, 3, device=dev) - 0.5, dim=-1)
    noise = torch.rand(R, S, device=dev)
    runner = net.hip_runner()

    def fwd(keep=True):
        return runner.forward(o, d, -d, noise, 0.01, 10.0, S, 0, keep=keep)

    if "--fused" in sys.argv:
        fused_phases(dev, net, runner)
        return
    for chain in ("1", "0", "1"):
        os.environ["NERF_CHAIN"] = chain
        for keep in (True, False):
            for _ in range(3):
                fwd(keep)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                fwd(keep)
            e.record()
            torch.cuda.synchronize()
            print(f"chain={chain} keep={keep}: forward {s.elapsed_time(e) / 10 * 1e3:8.1f} us", flush=True)
    os.environ["NERF_CHAIN"] = "1"
    Np = R * S
    for keep in (True, False):
        buf = torch.zeros((Np // 128) * 6, dtype=torch.int64, device=dev)
        _hip.lib().nerf_chain_debug_stamps(ctypes.c_void_p(buf.data_ptr()))
        fwd(keep)
        torch.cuda.synchronize()
        _hip.lib().nerf_chain_debug_stamps(None)
        st = buf.cpu().numpy().reshape(-1, 6).astype(np.float64)
        med = np.median(st, axis=0)
        if keep:   # k_mlp_chain_train2 (two waves per SIMD)
            print(f"keep=True: training chain phase cycles per block (median over {len(st)} blocks, wave 0): "
                  f"{f2_phases(med)}", flush=True)
        else:      # k_mlp_chain_fwd<false> (one wave per SIMD)
            print(f"keep=False: chain phase cycles per block (median over {len(st)} blocks, wave 0): dma wait "
                  f"{med[0]:.0f}  barrier {med[1]:.0f}  mfma section {med[2]:.0f}  epilogue {med[3]:.0f}  total "
                  f"{med[4]:.0f}", flush=True)


def f2_phases(med):
    """k_render_fused2 / k_mlp_chain_train2 stamps: k-step waits, barriers, prologue, layer
    epilogues, total, tail; the rest of the total is the k-steps' MFMA sections."""
    mma = med[4] - med[0] - med[1] - med[2] - med[3] - med[5]
    return (f"k-step waits {med[0]:.0f}  barriers {med[1]:.0f}  prologue {med[2]:.0f}  epilogues {med[3]:.0f}  "
            f"MFMA sections {mma:.0f}  tail {med[5]:.0f}  total {med[4]:.0f}")


def fused_phases(dev, net, runner):
    """Per-block phase cycles of the fused per-ray eval kernel at the cfg4 frame size."""
    R, S = 116748, 128
    o = (torch.rand(R, 3, device=dev) - 0.5) * 4
    d = torch.nn.functional.normalize(torch.rand(R, 3, device=dev) - 0.5, dim=-1)
    fn = lambda: runner.render_eval_fused(o, d, -d, 0.01, 10.0, S, 0)   # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        fn()
    e.record()
    torch.cuda.synchronize()
    nb = R * S // 128
    buf = torch.zeros(nb * 6, dtype=torch.int64, device=dev)
    _hip.lib().nerf_chain_debug_stamps(ctypes.c_void_p(buf.data_ptr()))
    fn()
    torch.cuda.synchronize()
    _hip.lib().nerf_chain_debug_stamps(None)
    st = buf.cpu().numpy().reshape(-1, 6).astype(np.float64)
    med = np.median(st, axis=0)
    if os.environ.get("NERF_FUSED_V1") == "1":
        print(f"fused eval (one wave per SIMD): {s.elapsed_time(e) / 3:.2f} ms/frame; phase cycles per block (median "
              f"over {len(st)} blocks, wave 0): dma wait {med[0]:.0f}  barrier {med[1]:.0f}  mfma section "
              f"{med[2]:.0f}  epilogue {med[3]:.0f}  total {med[4]:.0f}", flush=True)
    else:
        print(f"fused eval (k_render_fused2): {s.elapsed_time(e) / 3:.2f} ms/frame; phase cycles per block (median "
              f"over {len(st)} blocks, wave 0): {f2_phases(med)}", flush=True)


if __name__ == "__main__":
    main()

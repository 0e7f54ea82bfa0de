"""Standalone timing of the f16x3 NT GEMMs at the cfg2 layer shape (131072 x 256 x 256):
forward (bias, ReLU, mask, row / column maxima) and input gradient (mask); prints one JSON
line.  Environment knobs of the kernels (NERF_NT_STAGGER ...) apply per process.

    python scripts/nt_bench.py [--iters 30]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch  # noqa: E402

from model import _hip  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--ablate", type=int, default=0, help="nerf_gemm_debug_ablate mask (1: no epilogue stores)")
    ap.add_argument("--stamps", action="store_true", help="per-block phase clocks of one launch of each kernel")
    args = ap.parse_args()
    dev = torch.device("cuda")
    _hip.gemm_set_precision(2)
    M, D = 131072, 256
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(M, D, device=dev, generator=g) - 0.5
    W = (torch.rand(D, D, device=dev, generator=g) - 0.5) * 0.1
    b = torch.rand(D, device=dev, generator=g)
    y = torch.empty(M, D, device=dev)
    mask = torch.empty(M, D // 32, device=dev, dtype=torch.int32)
    ws, wts = _hip.split_image(D, D, dev), _hip.split_image(D, D, dev)
    Wp, Wt = torch.zeros(D, D, device=dev), torch.zeros(D, D, device=dev)
    _hip.pack_weights([_hip.PackDesc(W.data_ptr(), Wp.data_ptr(), Wt.data_ptr(), D, D, D, D, D, ws.data_ptr(),
                                     wts.data_ptr())])
    x_rm = x.abs().amax(1)
    y_rm, y_cm = torch.empty(M, device=dev), torch.empty(M // 128, D, device=dev)
    dx = torch.empty(M, D, device=dev)
    fwd = lambda: _hip.linear_fwd(x, D, None, 0, Wp, b, y, M, D, True, mask_out=mask, w_split=ws, x1_rmax=x_rm,
                                  y_rmax=y_rm, y_cmax=y_cm)
    fwd()
    bwd = lambda: _hip.linear_bwd_data(y, D, Wt, dx, M, D, mask=mask, wt_split=wts, dy_rmax=y_rm, dx_rmax=x_rm,
                                       dx_cmax=y_cm)
    if args.stamps:
        stamps(dev, M, {"fwd": fwd, "dx": bwd})
        return
    _hip.lib().nerf_gemm_debug_ablate(args.ablate)
    t_f = min(timeit(fwd, args.iters) for _ in range(3))
    t_b = min(timeit(bwd, args.iters) for _ in range(3))
    _hip.lib().nerf_gemm_debug_ablate(0)
    print(json.dumps({"fwd_us": t_f, "dx_us": t_b, "ablate": args.ablate, "stagger_fwd": os.environ.get("NERF_NT_STAGGER", "0"),
                      "stagger_bwd": os.environ.get("NERF_NT_STAGGER_BWD", "0")}))


def stamps(dev, M, fns):
    """Phase clocks (s_memtime / s_memrealtime at kernel start, after the prologue, after the
    main loop, after the epilogue's stores drained) of every block of one launch: per-phase
    cycles, and how the phases of co-running blocks overlap in time."""
    import ctypes
    import numpy as np
    nb = M // 128
    for name, fn in fns.items():
        for _ in range(10):
            fn()
        buf = torch.zeros(nb * 10 * 2, dtype=torch.int64, device=dev)
        _hip.lib().nerf_gemm_debug_stamps(ctypes.c_void_p(buf.data_ptr()))
        fn()
        torch.cuda.synchronize()
        _hip.lib().nerf_gemm_debug_stamps(None)
        st = buf.cpu().numpy().reshape(nb, 10, 2).astype(np.float64)
        cyc = np.diff(st[:, :4, 0], axis=1)
        rt = st[:, :4, 1]
        clk = (st[:, 3, 0] - st[:, 0, 0]) / ((st[:, 3, 1] - st[:, 0, 1]) / 100e6)
        t0 = rt[:, 0].min()
        rt = (rt - t0) / 100.0                      # us since the first block started
        # fraction of the launch during which >= 1 / all resident blocks are in the main loop
        grid = np.arange(0.0, rt[:, 3].max(), 0.05)
        inmain = ((rt[:, 1][None, :] <= grid[:, None]) & (grid[:, None] < rt[:, 2][None, :])).sum(1)
        alive = ((rt[:, 0][None, :] <= grid[:, None]) & (grid[:, None] < rt[:, 3][None, :])).sum(1)
        print(json.dumps({
            "kernel": name, "blocks": nb, "clock_ghz": round(float(np.median(clk)) / 1e9, 3),
            "cycles_median": {"prologue": float(np.median(cyc[:, 0])), "mainloop": float(np.median(cyc[:, 1])),
                              "epilogue_incl_store_drain": float(np.median(cyc[:, 2]))},
            "epilogue_parts_median": ({"loop": float(np.median(st[:, 4, 0] - st[:, 2, 0])),
                                       "maxima": float(np.median(st[:, 5, 0] - st[:, 4, 0])),
                                       "post": float(np.median(st[:, 9, 0] - st[:, 5, 0])),
                                       "drain": float(np.median(st[:, 3, 0] - st[:, 9, 0]))}
                                      if (st[:, 4, 0] > 0).all() else None),
            "block_us_median": round(float(np.median(rt[:, 3] - rt[:, 0])), 2),
            "span_us": round(float(rt[:, 3].max()), 2),
            "start_us_quartiles": np.percentile(rt[:, 0], [25, 50, 75, 100]).round(2).tolist(),
            "mean_blocks_alive": round(float(alive.mean()), 1),
            "mean_blocks_in_mainloop": round(float(inmain.mean()), 1)}))


if __name__ == "__main__":
    main()

"""Exact-f32 GEMM launches for the clock / MFMA-busy PMC pass.

Runs the exact-f32 MFMA kernels of one field layer (131072 x 256 x 256 per launch at the cfg2
shape: forward NT, input-gradient NT, weight-gradient TN + slab reduce) back to back for ~2 s so
the chip settles at its loaded clock, then a few more launches of each; under
``rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES ... --kernel-trace``
every dispatch carries its counters and its duration (scripts/f32_clock_summary.py reduces
them: effective clock = GRBM_GUI_ACTIVE / 8 XCDs / duration, MFMA busy against the
instructions the launch must issue).  Prints the un-profiled per-launch times as one JSON line.

    python scripts/f32_clock.py [--seconds 2]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch  # noqa: E402

from model import _hip  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--rows", type=int, default=4 * 131072, help="rows per launch (longer dispatches: the "
                    "GRBM clock estimate reads high below ~0.3 ms)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    _hip.load_library()
    _hip.gemm_set_precision(0)
    M, D = args.rows, 256
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(M, D, device=dev, generator=g) - 0.5            # random operands: the loaded clock
    W = (torch.rand(D, D, device=dev, generator=g) - 0.5) * 0.1
    Wt = W.t().contiguous()
    b = torch.rand(D, device=dev, generator=g)
    y = torch.empty(M, D, device=dev)
    mask = torch.empty(M, D // 32, device=dev, dtype=torch.int32)
    dx = torch.empty(M, D, device=dev)
    splits = _hip.bwd_weight_splits(D, D, M)
    slab = torch.empty(splits * D * D, device=dev)
    bslab = torch.empty(splits * D, device=dev)
    gw, gb = torch.empty(D, D, device=dev), torch.empty(D, device=dev)
    fns = {
        "fwd": lambda: _hip.linear_fwd(x, D, None, 0, W, b, y, M, D, True, mask_out=mask),
        "dx": lambda: _hip.linear_bwd_data(y, D, Wt, dx, M, D, mask=mask),
        "dw": lambda: _hip.linear_bwd_weight(y, D, x, D, M, splits, slab, D, 0, bslab),
        "reduce": lambda: _hip.slab_reduce(slab, splits, D, D, D, D, bslab, gw, gb),
    }
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.seconds:
        for f in fns.values():
            f()
        torch.cuda.synchronize()
    us = {k: min(timeit(f, 5) for _ in range(2)) for k, f in fns.items()}
    fl = 2.0 * M * D * D
    print(json.dumps({"rows": M, "us": us, "tflops": {k: fl / us[k] / 1e6 for k in ("fwd", "dx", "dw")},
                      "precision": "exact f32 (v_mfma_f32_32x32x2_f32)"}))


if __name__ == "__main__":
    main()

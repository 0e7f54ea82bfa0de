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
    t_f = min(timeit(fwd, args.iters) for _ in range(3))
    t_b = min(timeit(bwd, args.iters) for _ in range(3))
    print(json.dumps({"fwd_us": t_f, "dx_us": t_b, "stagger_fwd": os.environ.get("NERF_NT_STAGGER", "0"),
                      "stagger_bwd": os.environ.get("NERF_NT_STAGGER_BWD", "0")}))


if __name__ == "__main__":
    main()

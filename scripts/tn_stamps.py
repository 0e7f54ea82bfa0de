"""Per-phase cycles of the weight-gradient TN main loop (policy 7, 131072 x 256 x 256) from a
diagnostic build (make BUILD=build_tst LIB=lib/ab/tst.so EXTRA=-DNERF_TN_STAMPS=1, run with
NERF_HIP_LIB pointing at it): wave 0 of every block, mean over blocks.

    NERF_HIP_LIB=my-nope-nerf_amd/lib/ab/tst.so python scripts/tn_stamps.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
import torch  # noqa: E402

from model import _hip  # noqa: E402

PHASES = ["fragment_reads", "split_next_tile", "load_issue", "mfma", "barrier", "prologue", "epilogue", "total"]


def main():
    dev = torch.device("cuda")
    _hip.load_library()
    _hip.gemm_set_precision(2)
    M, D = 131072, 256
    g = torch.Generator(device=dev).manual_seed(0)
    dy = torch.rand(M, D, device=dev, generator=g) - 0.5
    x = torch.rand(M, D, device=dev, generator=g) - 0.5
    dy_cm = dy.abs().view(M // 128, 128, D).amax(1)
    x_cm = x.abs().view(M // 128, 128, D).amax(1)
    sp = _hip.bwd_weight_splits(D, D, M)
    slab = torch.empty(sp * D * D, device=dev)
    bslab = torch.empty(sp * D, device=dev)
    buf = torch.zeros(2 * sp * 8, dtype=torch.int64, device=dev)
    run = lambda: _hip.linear_bwd_weight(dy, D, x, D, M, sp, slab, D, 0, bslab, dy_cmax=dy_cm, x_cmax=x_cm)  # noqa
    run()
    torch.cuda.synchronize()
    _hip.lib().nerf_gemm_debug_stamps(buf.data_ptr())
    run()
    torch.cuda.synchronize()
    _hip.lib().nerf_gemm_debug_stamps(None)
    s = buf.view(-1, 8).double()
    mean = s.mean(0).tolist()
    out = {p: {"cycles": mean[i], "frac_of_total": mean[i] / mean[7]} for i, p in enumerate(PHASES)}
    out["blocks"] = s.shape[0]
    out["k_tiles_per_block"] = M // sp // 16
    print(json.dumps(out))


if __name__ == "__main__":
    main()

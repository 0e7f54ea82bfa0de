"""Where a weight-gradient (TN policy 7) launch's time goes: one 131072 x 256 x 256 layer timed
standalone, also without the bias column sums (nerf_gemm_debug_ablate TN bit 4, shifted by 4;
results are wrong while set) and, with a library built with -DNERF_TN_ABLATE=1 (NERF_HIP_LIB),
without the operand split (one RNE fp16 word per value).

    python scripts/tn_ablation.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch  # noqa: E402

from gemm_bench import timeit  # noqa: E402
from model import _hip  # noqa: E402


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
    out = {}
    for name, mask in (("production", 0), ("no_bias_sums", 4), ("production_again", 0)):
        _hip.lib().nerf_gemm_debug_ablate(mask << 4)
        out[name] = timeit(lambda: _hip.linear_bwd_weight(dy, D, x, D, M, sp, slab, D, 0, bslab, dy_cmax=dy_cm,
                                                            x_cmax=x_cm), iters=30)
    _hip.lib().nerf_gemm_debug_ablate(0)
    out["lib"] = os.environ.get("NERF_HIP_LIB", "default")
    print(json.dumps(out))


if __name__ == "__main__":
    main()

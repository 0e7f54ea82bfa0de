"""Weight-gradient GEMM (k_gemm_tn_*) + slab reduce at the production shapes vs split count.

    python scripts/dw_bench.py [--x6|--h16]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
import torch  # noqa: E402

from model import _hip  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda")
    _hip.gemm_set_precision(2 if "--h16" in sys.argv else 1 if "--x6" in sys.argv else 0)
    M = 131072
    g = torch.Generator(device=dev).manual_seed(0)
    for nout, kin in ((256, 256), (256, 64), (128, 256), (128, 64)):
        dy = torch.rand(M, nout, device=dev, generator=g) - 0.5
        x = torch.rand(M, kin, device=dev, generator=g) - 0.5
        gw, gb = torch.empty(nout, kin, device=dev), torch.empty(nout, device=dev)
        dy_cm = dy.abs().view(M // 128, 128, nout).amax(1)
        x_cm = x.abs().view(M // 128, 128, kin).amax(1)
        best = _hip.bwd_weight_splits(nout, kin, M)
        for sp in (16, 32, 64, 128, 256, 512):
            slab = torch.empty(sp * nout * kin, device=dev)
            bslab = torch.empty(sp * nout, device=dev)
            t_g = min(timeit(lambda: _hip.linear_bwd_weight(dy, nout, x, kin, M, sp, slab, kin, 0, bslab,
                                                              dy_cmax=dy_cm, x_cmax=x_cm))
                      for _ in range(3))
            t_r = min(timeit(lambda: _hip.slab_reduce(slab, sp, nout, kin, nout, kin, bslab, gw, gb))
                      for _ in range(3))
            fl = 2.0 * M * nout * kin
            print(f"dW {nout}x{kin} splits {sp:4d}{' (default)' if sp == best else '          '}: gemm {t_g:7.1f} us "
                  f"({fl / t_g / 1e6:6.1f} TF/s)  reduce {t_r:6.1f} us  sum {t_g + t_r:7.1f} us", flush=True)


if __name__ == "__main__":
    main()

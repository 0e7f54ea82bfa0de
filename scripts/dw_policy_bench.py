"""Weight gradient of one 131072 x 256 x 256 layer (fp16 pair) + its slab reduce, per TN tile
policy (3: 256x256 tiles, 256 splits; 7: XCD-paired 256x128 tiles of 8 waves, 128 splits, the
colour layer as one 128x256 tile), standalone and beside an input-gradient NT on a
second stream (the step's situation).

    python scripts/dw_policy_bench.py
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
    _hip.load_library()
    _hip.gemm_set_precision(2)
    for nout, kin, pols in ((256, 256, (3, 7)), (256, 64, (3, 7)), (128, 256, (3, 7)), (128, 64, (3, 7))):
        shape(dev, nout, kin, pols)
    _hip.gemm_set_policy(0, 0)


def shape(dev, nout, kin, pols):
    M = 131072
    g = torch.Generator(device=dev).manual_seed(0)
    dy = torch.rand(M, nout, device=dev, generator=g) - 0.5
    x = torch.rand(M, kin, device=dev, generator=g) - 0.5
    gw, gb = torch.empty(nout, kin, device=dev), torch.empty(nout, device=dev)
    dy_cm = dy.abs().view(M // 128, 128, nout).amax(1)
    x_cm = x.abs().view(M // 128, 128, kin).amax(1)
    ref = None
    for pol in pols:
        _hip.gemm_set_policy(0, pol)
        sp = _hip.bwd_weight_splits(nout, kin, M)
        slab = torch.empty(sp * nout * kin, device=dev)
        bslab = torch.empty(sp * nout, device=dev)
        t_g = min(timeit(lambda: _hip.linear_bwd_weight(dy, nout, x, kin, M, sp, slab, kin, 0, bslab,
                                                          dy_cmax=dy_cm, x_cmax=x_cm)) for _ in range(3))
        t_r = min(timeit(lambda: _hip.slab_reduce(slab, sp, nout, kin, nout, kin, bslab, gw, gb)) for _ in range(3))
        torch.cuda.synchronize()
        if ref is None:
            ref = gw.clone()
        err = ((gw - ref).norm() / ref.norm()).item()
        slab_mb = sp * nout * kin * 4 / 1e6
        print(f"{nout}x{kin} policy {pol}: splits {sp:4d}  gemm {t_g:7.1f} us  reduce {t_r:6.1f} us  sum {t_g + t_r:7.1f} us  "
              f"slab {slab_mb:5.1f} MB  rel-diff vs first {err:.2e}", flush=True)


if __name__ == "__main__":
    main()

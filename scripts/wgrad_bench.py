"""Weight-gradient kernels of one 131072-row layer (fp16 pair, GEMM precision mode 2),
standalone: TN policy 7 (the 8-wave kernels of gemm_x6.hip) against policy 8 (the MFMA +
load-wave kernels of wgrad.hip), per shape, with the slab reduce; the policy-8 slabs are
checked bit-identical to policy 7's.

    python scripts/wgrad_bench.py            # timings (us per launch, median of 3 x 20)
    python scripts/wgrad_bench.py --loop N   # N back-to-back policy-8 launches of the 256 x 256
                                             # layer only (for rocprofv3 --pmc passes)
    python scripts/wgrad_bench.py --lib my-nope-nerf_amd/lib/ab/x.so ...   # a diagnostic build
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
if "--lib" in sys.argv:   # a diagnostic build in place of the tree's library (read at import)
    os.environ["NERF_HIP_LIB"] = os.path.join(ROOT, sys.argv[sys.argv.index("--lib") + 1])
import torch  # noqa: E402

from model import _hip  # noqa: E402

M = 131072


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return 1e3 * a.elapsed_time(b) / n


def operands(dev, nout, kin):
    g = torch.Generator(device=dev).manual_seed(nout + kin)
    dy = torch.rand(M, nout, device=dev, generator=g) - 0.5
    x = torch.rand(M, kin, device=dev, generator=g) - 0.5
    return dy, x, dy.abs().view(M // 128, 128, nout).amax(1), x.abs().view(M // 128, 128, kin).amax(1)


def shape(dev, nout, kin, check=True):
    dy, x, dy_cm, x_cm = operands(dev, nout, kin)
    gw, gb = torch.empty(nout, kin, device=dev), torch.empty(nout, device=dev)
    out = {}
    for pol in (7, 8):
        _hip.gemm_set_policy(0, pol)
        sp = _hip.bwd_weight_splits(nout, kin, M)
        slab = torch.empty(sp * nout * kin, device=dev)
        bslab = torch.empty(sp * nout, device=dev)
        t_g = sorted(timeit(lambda: _hip.linear_bwd_weight(dy, nout, x, kin, M, sp, slab, kin, 0, bslab,
                                                             dy_cmax=dy_cm, x_cmax=x_cm)) for _ in range(3))[1]
        t_r = sorted(timeit(lambda: _hip.slab_reduce(slab, sp, nout, kin, nout, kin, bslab, gw, gb))
                     for _ in range(3))[1]
        torch.cuda.synchronize()
        out[pol] = slab.clone()
        mb = 4 * M * (nout + kin) / 1e6
        print(f"{nout}x{kin} policy {pol}: splits {sp:4d}  gemm {t_g:7.1f} us ({mb / t_g:5.2f} TB/s algorithmic)  "
              f"reduce {t_r:6.1f} us", flush=True)
    _hip.gemm_set_policy(0, 0)
    if check:
        assert torch.equal(out[7], out[8]), "policy 8 slabs differ from policy 7"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loop", type=int, default=0)
    ap.add_argument("--lib", default=None, help="library path relative to the repo root (diagnostic builds)")
    ap.add_argument("--shapes", default="256x256,256x64,128x256,128x64")
    ap.add_argument("--no-check", dest="check", action="store_false",
                    help="skip the policy 7 / 8 bit-identity check (diagnostic builds via NERF_HIP_LIB)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    _hip.load_library()
    _hip.gemm_set_precision(2)
    if args.loop:
        dy, x, dy_cm, x_cm = operands(dev, 256, 256)
        sp = _hip.bwd_weight_splits(256, 256, M)
        slab, bslab = torch.empty(sp * 256 * 256, device=dev), torch.empty(sp * 256, device=dev)
        for _ in range(args.loop):
            _hip.linear_bwd_weight(dy, 256, x, 256, M, sp, slab, 256, 0, bslab, dy_cmax=dy_cm, x_cmax=x_cm)
        torch.cuda.synchronize()
        return
    for sh in args.shapes.split(","):
        nout, kin = (int(v) for v in sh.split("x"))
        shape(dev, nout, kin, args.check)


if __name__ == "__main__":
    main()

"""GEMM tile-policy A/B at the production shapes (one process, interleaved rounds).

    python scripts/gemm_bench.py
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))

import torch  # noqa: E402

from model import _hip  # noqa: E402


def timeit(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us


def main():
    dev = torch.device("cuda")
    M, D = 131072, 256
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(M, D, device=dev, generator=g) - 0.5
    enc = torch.rand(M, 64, device=dev, generator=g) - 0.5
    W = (torch.rand(D, D, device=dev, generator=g) - 0.5) * 0.1
    W4 = (torch.rand(D, D + 64, device=dev, generator=g) - 0.5) * 0.1
    b = torch.rand(D, device=dev, generator=g)
    y = torch.empty(M, D, device=dev)
    mask = torch.empty(M, D // 32, device=dev, dtype=torch.int32)
    dy = torch.rand(M, D, device=dev, generator=g) - 0.5
    u = torch.rand(M, 4, device=dev, generator=g)
    # split images of W (forward B operand) and of W as the transposed backward operand, in
    # both split forms (mode 1 bf16x3, mode 2 fp16 pair: the pack writes the current mode's)
    imgs = {}
    for mode in (1, 2):
        _hip.gemm_set_precision(mode)
        ws, wts = _hip.split_image(D, D, dev), _hip.split_image(D, D, dev)
        Wp, Wt = torch.zeros(D, D, device=dev), torch.zeros(D, D, device=dev)
        _hip.pack_weights([_hip.PackDesc(W.data_ptr(), Wp.data_ptr(), Wt.data_ptr(), D, D, D, D, D, ws.data_ptr(),
                                         wts.data_ptr())])
        ws4 = _hip.split_image(D, D + 64, dev)
        W4p, W4t = torch.zeros(D, D + 64, device=dev), torch.zeros(D + 64, D, device=dev)
        _hip.pack_weights([_hip.PackDesc(W4.data_ptr(), W4p.data_ptr(), W4t.data_ptr(), D, D + 64, D + 64, D + 64, D,
                                         ws4.data_ptr(), None)])
        imgs[mode] = (ws, wts, ws4)
    _hip.gemm_set_precision(0)
    im = lambda i: imgs[max(1, _hip.gemm_get_precision())][i]
    # row maxima of the A operands (mode 2 only; the other modes ignore them)
    x_rm, enc_rm, dy_rm = x.abs().amax(1), enc.abs().amax(1), dy.abs().amax(1)
    x_cm, dy_cm = x.abs().view(M // 128, 128, D).amax(1), dy.abs().view(M // 128, 128, D).amax(1)
    y_rm = torch.empty(M, device=dev)
    cases = {}
    # split images are passed everywhere; the exact-f32 mode ignores them
    cases["fwd 256x256"] = (lambda: _hip.linear_fwd(x, D, None, 0, W, b, y, M, D, 1, mask_out=mask, w_split=im(0),
                                                    x1_rmax=x_rm, y_rmax=y_rm), 2 * M * D * D)
    cases["fwd skip 320"] = (lambda: _hip.linear_fwd(x, D, enc, 64, W4, b, y, M, D, 1, w_split=im(2), x1_rmax=x_rm,
                                                     x2_rmax=enc_rm, y_rmax=y_rm), 2 * M * D * (D + 64))
    cases["bwd-data mask+u"] = (lambda: _hip.linear_bwd_data(dy, D, W, y, M, D, mask=mask, u=u, ldu=4, v=b,
                                                             wt_split=im(1), dy_rmax=dy_rm, dx_rmax=y_rm),
                                2 * M * D * D)
    for sp in (64, 128, 256):
        slab = torch.empty(sp * D * D, device=dev)
        bslab = torch.empty(sp * D, device=dev)
        cases[f"dW splits={sp}"] = ((lambda sp=sp, slab=slab, bslab=bslab:
                                     _hip.linear_bwd_weight(dy, D, x, D, M, sp, slab, D, 0, bslab, dy_cmax=dy_cm,
                                                            x_cmax=x_cm)), 2 * M * D * D)
    slab = torch.rand(256 * D * D, device=dev, generator=g)
    bslab = torch.rand(256 * D, device=dev, generator=g)
    gw, gb = torch.empty(D, D, device=dev), torch.empty(D, device=dev)
    cases["slab_reduce 256"] = (lambda: _hip.slab_reduce(slab, 256, D, D, D, D, bslab, gw, gb), 0)
    if "--x6" in sys.argv:
        _hip.gemm_set_precision(1)
    if "--h16" in sys.argv:
        _hip.gemm_set_precision(2)
    if "--stamps" in sys.argv:   # per-block phase clocks of the split-bf16 NT kernel
        import numpy as np
        for name in ("fwd 256x256", "bwd-data mask+u"):
            fn, fl = cases[name]
            for _ in range(20):
                fn()
            buf = torch.zeros((M // 128) * 10 * 2, dtype=torch.int64, device=dev)   # 128-row tiles: M/128 blocks
            _hip.lib().nerf_gemm_debug_stamps(ctypes.c_void_p(buf.data_ptr()))
            fn()
            torch.cuda.synchronize()
            _hip.lib().nerf_gemm_debug_stamps(None)
            st = buf.cpu().numpy().reshape(-1, 10, 2).astype(np.float64)
            sub = st[:, [9, 4, 5, 6, 7, 8], 0]
            d = np.median(np.diff(sub, axis=1), axis=0)
            print(f"  iteration 5 (cycles): issue+frag reads {d[0]:.0f}  split+row0 {d[1]:.0f}  rest MFMA issue "
                  f"{d[2]:.0f}  dma wait {d[3]:.0f}  barrier {d[4]:.0f}")
            clk = (st[:, 3, 0] - st[:, 0, 0]) / ((st[:, 3, 1] - st[:, 0, 1]) / 100e6)
            ph = np.diff(st[:, :4, 0], axis=1)
            t0 = st[:, 0, 1].min()
            start = (st[:, 0, 1] - t0) / 100.0
            end = (st[:, 3, 1] - t0) / 100.0
            print(f"{name}: blocks {len(st)}  clock median {np.median(clk) / 1e9:.2f} GHz  "
                  f"cycles median prologue {np.median(ph[:, 0]):.0f} mainloop {np.median(ph[:, 1]):.0f} "
                  f"epilogue {np.median(ph[:, 2]):.0f}  block us median {np.median(end - start):.1f} "
                  f"span {end.max():.1f} us  start quartiles {np.percentile(start, [25, 50, 75, 100]).round(1)}")
        return
    quick = "--quick" in sys.argv
    if quick:   # one launch per case at the default policy (for PMC collection)
        for name, (fn, fl) in cases.items():
            fn()
        torch.cuda.synchronize()
        return
    if "--ablate" in sys.argv:
        for pol in (2, 3):
            _hip.gemm_set_policy(pol, 3)
            for ab in (0, 1, 2, 3, 4, 7):
                _hip.lib().nerf_gemm_debug_ablate(ab)
                for name in ("fwd 256x256", "bwd-data mask+u"):
                    fn, fl = cases[name]
                    us = min(timeit(fn) for _ in range(3))
                    print(f"ablate={ab} policy {pol} {name:18s}: {us:8.1f} us {fl / us / 1e6:6.1f} TF/s")
        _hip.gemm_set_policy(0, 0)
        for ab in (0, 16, 32, 64, 128, 16 + 32 + 64, 16 + 32 + 64 + 128):
            _hip.lib().nerf_gemm_debug_ablate(ab)
            fn, fl = cases["dW splits=256"]
            us = min(timeit(fn) for _ in range(3))
            print(f"ablate={ab} dW splits=256: {us:8.1f} us {fl / us / 1e6:6.1f} TF/s")
        _hip.lib().nerf_gemm_debug_ablate(0)
        return
    if "--prec" in sys.argv:   # exact-f32 MFMA vs split-bf16 vs fp16 pair, default tile policy
        res = {}
        for rnd in range(3):
            for prec in (0, 1, 2):
                _hip.gemm_set_precision(prec)
                for name, (fn, fl) in cases.items():
                    res.setdefault((name, prec), []).append(timeit(fn))
        _hip.gemm_set_precision(0)
        for (name, prec), v in sorted(res.items()):
            fl = cases[name][1]
            best = min(v)
            print(f"{name:22s} precision {prec}: {best:8.1f} us  {fl / best / 1e6:6.1f} TF/s (f32-equivalent)"
                  + (f"  {4 * 257 * D * D / best / 1e3:6.0f} GB/s" if fl == 0 else ""))
        return
    res = {}
    for rnd in range(3):
        for pol in (1, 2, 3):
            _hip.gemm_set_policy(pol, 0)
            for name, (fn, fl) in cases.items():
                us = timeit(fn)
                res.setdefault((name, pol), []).append(us)
    for (name, pol), v in sorted(res.items()):
        fl = cases[name][1]
        best = min(v)
        print(f"{name:22s} policy {pol}: {best:8.1f} us  {fl / best / 1e6:6.1f} TF/s  (rounds {['%.0f' % t for t in v]})")
    _hip.gemm_set_policy(0, 0)


if __name__ == "__main__":
    main()

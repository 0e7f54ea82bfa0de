"""Does splitting the rows of a layer chain over two streams desynchronise the launches?

Four dependent f16x3 forward layers (131072 x 256 x 256, bias + ReLU + mask + maxima, as in
training) timed three ways:
  single  one stream, full M per launch (the production forward);
  dual    rows [0, M/2) on stream 1 and [M/2, M) on stream 2, each stream its own chain;
  dual_o  as dual, stream 2 starting one half-layer behind stream 1 (event after s1's layer 0).
Prints one JSON line of microseconds per 4-layer chain.

    python scripts/dual_stream_bench.py [--iters 20] [--layers 4]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))

import torch  # noqa: E402

from model import _hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--layers", type=int, default=4)
    args = ap.parse_args()
    dev = torch.device("cuda")
    _hip.gemm_set_precision(2)
    M, D, L = 131072, 256, args.layers
    H = M // 2
    g = torch.Generator(device=dev).manual_seed(0)
    acts = [torch.rand(M, D, device=dev, generator=g) - 0.5] + [torch.empty(M, D, device=dev) for _ in range(L)]
    rmax = [a.abs().amax(1) if i == 0 else torch.empty(M, device=dev) for i, a in enumerate(acts)]
    cmax = [torch.empty(M // 128, D, device=dev) for _ in range(L + 1)]
    masks = [torch.empty(M, D // 32, device=dev, dtype=torch.int32) for _ in range(L)]
    Ws, bs, imgs = [], [], []
    for _ in range(L):
        W = (torch.rand(D, D, device=dev, generator=g) - 0.5) * 0.2
        ws, wts = _hip.split_image(D, D, dev), _hip.split_image(D, D, dev)
        Wp, Wt = torch.zeros(D, D, device=dev), torch.zeros(D, D, device=dev)
        _hip.pack_weights([_hip.PackDesc(W.data_ptr(), Wp.data_ptr(), Wt.data_ptr(), D, D, D, D, D, ws.data_ptr(),
                                         wts.data_ptr())])
        Ws.append(Wp)
        imgs.append(ws)
        bs.append(torch.rand(D, device=dev, generator=g) * 0.1)

    def layer(l, r0, r1):
        x, y = acts[l][r0:r1], acts[l + 1][r0:r1]
        _hip.linear_fwd(x, D, None, 0, Ws[l], bs[l], y, r1 - r0, D, True, mask_out=masks[l][r0:r1],
                        w_split=imgs[l], x1_rmax=rmax[l][r0:r1], y_rmax=rmax[l + 1][r0:r1],
                        y_cmax=cmax[l + 1][r0 // 128:r1 // 128])

    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    main = torch.cuda.current_stream(dev)

    def single():
        for l in range(L):
            layer(l, 0, M)

    def dual(offset):
        ev0 = torch.cuda.Event()
        s1.wait_stream(main)
        s2.wait_stream(main)
        with torch.cuda.stream(s1):
            for l in range(L):
                layer(l, 0, H)
                if l == 0:
                    ev0.record(s1)
        with torch.cuda.stream(s2):
            if offset:
                s2.wait_event(ev0)
            for l in range(L):
                layer(l, H, M)
        main.wait_stream(s1)
        main.wait_stream(s2)

    def timeit(fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        torch.cuda.synchronize()
        s.record()
        for _ in range(args.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / args.iters * 1e3

    single()
    ref = acts[L].clone()
    dual(False)
    torch.cuda.synchronize()
    same = bool(torch.equal(ref, acts[L]))
    res = {"layers": L, "rows": M, "dual_bitwise_equal": same}
    for name, fn in (("single", single), ("dual", lambda: dual(False)), ("dual_o", lambda: dual(True))):
        res[name + "_us"] = round(min(timeit(fn) for _ in range(3)), 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

"""The head-weight / bias partials (nerf_heads_bwd_mode 2) of the D = 256 field at the
training batch (131072 samples), standalone: the 16-byte-load kernel (k_heads_wgrad256, rows
16-byte aligned) against the dword form (k_heads_bwd<4, 2, 2>, reached with a padded h8
leading dimension), plus the partial reduce; the two agree to f32 rounding.

    python scripts/heads_bench.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
import torch  # noqa: E402

from model import _hip  # noqa: E402

N = 131072


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


def main():
    dev = torch.device("cuda")
    _hip.load_library()
    g = torch.Generator(device=dev).manual_seed(0)
    graw = torch.randn(N, 4, device=dev, generator=g)
    h8p = torch.rand(N, 258, device=dev, generator=g)          # ld 258: the dword kernel
    h8 = h8p[:, :256].contiguous()                              # ld 256: the 16-byte kernel
    hr = torch.rand(N, 128, device=dev, generator=g)
    wc = torch.randn(3, 128, device=dev, generator=g)
    part = torch.empty(_hip.heads_part_size(256, N), device=dev)
    out = {}
    for name, h in (("16-byte loads", h8), ("dword loads", h8p[:, :256])):
        t = sorted(timeit(lambda: _hip.heads_bwd(graw, h, hr, 256, wc, None, part, N, mode=2)) for _ in range(3))[1]
        gwd, gbd = torch.empty(256, device=dev), torch.empty(1, device=dev)
        gwc, gbc = torch.empty(3, 128, device=dev), torch.empty(3, device=dev)
        tr = sorted(timeit(lambda: _hip.heads_reduce(part, 256, N, gwd, gbd, gwc, gbc)) for _ in range(3))[1]
        torch.cuda.synchronize()
        out[name] = torch.cat([gwd, gbd, gwc.flatten(), gbc])
        mb = 4 * N * (256 + 128 + 4) / 1e6
        print(f"{name}: partials {t:7.1f} us ({mb / t:5.2f} TB/s of h8 + hr + graw4)  reduce {tr:5.1f} us", flush=True)
    a, b = out["16-byte loads"], out["dword loads"]
    print("max rel diff", ((a - b).abs().max() / b.abs().max()).item())


if __name__ == "__main__":
    main()

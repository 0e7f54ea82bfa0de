"""Composite kernel roofline at large ray counts (HBM bound): algorithmic bytes
fwd = 24 B/sample (raw4 16 + z 4 read, alpha 4 written) + 16 B/ray; bwd = 36 B/sample
(raw4 16 + z 4 read, graw4 16 written) + 16 B/ray read."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
import torch  # noqa: E402

from model import _hip  # noqa: E402

PEAK = 8000.0   # GB/s (MI355X HBM3E spec)


def main():
    dev = torch.device("cuda")
    S = 128
    for R in (1024, 116748, 1 << 20):
        N = R * S
        Np = (N + 127) // 128 * 128
        g = torch.Generator(device=dev).manual_seed(0)
        raw4 = torch.randn(Np, 4, device=dev, generator=g)
        z = torch.sort(torch.rand(R, S, device=dev, generator=g) * 10, 1)[0].reshape(-1)
        z = torch.cat([z, torch.zeros(Np - N, device=dev)])
        rgb, dist, alpha = torch.empty(R, 3, device=dev), torch.empty(R, device=dev), torch.empty(R, S, device=dev)
        grgb, gd = torch.randn(R, 3, device=dev), torch.randn(R, device=dev)
        graw = torch.empty(Np, 4, device=dev)
        for name, fn, nbytes in (
                ("fwd", lambda: _hip.composite_fwd(raw4, z, R, S, 0, rgb, dist, alpha), 24 * N + 16 * R),
                ("bwd", lambda: _hip.composite_bwd(raw4, z, R, S, 0, grgb, gd, graw, Np), 36 * N + 16 * R)):
            fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            it = 20
            s.record()
            for _ in range(it):
                fn()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / it * 1e3
            gbs = nbytes / us / 1e3
            print(f"composite_{name} R={R:8d} S={S}: {us:9.1f} us  {gbs:7.0f} GB/s  {100 * gbs / PEAK:5.1f} % of 8 TB/s")


if __name__ == "__main__":
    main()

"""Benchmark of the full NoPe-NeRF training step (BASELINE.json configs[2], config 3 of
SURVEY.md section 8(d)) on its own: the same measurement bench.py reports as "full_cfg3"
(bench.cfg3_line), with more steps.  Prints one JSON line.

    python scripts/bench_full.py [--steps K --warmup W] [--mode both|eager|graph]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    import bench
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--gemm-precision", choices=["f32", "bf16x6", "f16x3"], default="f16x3")
    ap.add_argument("--mode", choices=["both", "eager", "graph"], default="both",
                    help="eager enqueue, hipGraph replay of the two views' captured train_steps, or both "
                         "(default; value = the faster, both reported)")
    args = ap.parse_args()
    from model import _hip
    dev = torch.device("cuda", 0)
    _hip.load_library()
    _hip.gemm_set_precision(bench.PRECISION[args.gemm_precision])
    modes = ["eager", "graph"] if args.mode == "both" else [args.mode]
    out = bench.cfg3_line(dev, args.steps, args.warmup, modes)
    out["gemm_arithmetic"] = args.gemm_precision
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""A/B of eager enqueue vs hipGraph replay of bench.py's cfg2 train step (one GPU),
interleaved over rounds; prints ms/step per mode (median of rounds).

    python scripts/graph_ab.py [--steps 30 --rounds 3]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    from model import _hip
    _hip.load_library()
    _hip.gemm_set_precision(2)
    dev = torch.device("cuda", 0)
    cfg = bench.make_cfg()
    data, c2w = bench.synthetic_scene(dev)
    res = {}
    for mode in ("eager", "graph"):
        trainer, _ = bench.build_trainer(dev, c2w, cfg)
        if mode == "graph":
            trainer.enable_graph_rng()
        step = lambda i: trainer.train_step(data, it=i, epoch=0, scheduling_start=0)  # noqa: E731
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for i in range(3):
                step(i)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if mode == "graph":
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                out = step(0)
            run = lambda i: (g.replay(), out)[1]  # noqa: E731
        else:
            run = step
        res[mode] = (run, [])
    for _ in range(args.rounds):
        for mode, (run, times) in res.items():
            for i in range(3):
                run(i)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.steps):
                ld = run(i)
            torch.cuda.synchronize()
            times.append(1e3 * (time.perf_counter() - t0) / args.steps)
            if not torch.isfinite(ld["loss"]).item():
                raise RuntimeError(f"{mode}: non-finite loss")
    print(json.dumps({m: {"ms_per_step_median": statistics.median(t), "rounds": t} for m, (_, t) in res.items()}))


if __name__ == "__main__":
    main()

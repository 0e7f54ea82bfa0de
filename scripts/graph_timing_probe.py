"""Probe: does bench.py's graph-replay timing loop (an event recorded behind every replay) cost
the replays time, and does that depend on the head-reduce placement (NERF_HEADS_PLACE)?  For
each placement, one trainer and one captured cfg2 step (bench.measure_graph's recipe); K replays
timed with and without the per-replay events, interleaved over rounds; the work is checked by
the loss staying finite and the field's parameters moving between timed sets.

    python scripts/graph_timing_probe.py --rounds 3 --steps 30 [--places 5 1]
"""
from __future__ import annotations

import argparse
import json
import math
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
    ap.add_argument("--places", nargs="+", default=["5", "1"])
    args = ap.parse_args()
    from model import _hip
    _hip.load_library()
    _hip.gemm_set_precision(2)
    dev = torch.device("cuda", 0)
    cfg = bench.make_cfg()
    data, c2w = bench.synthetic_scene(dev)
    setups = {}
    for hp in args.places:
        os.environ["NERF_HEADS_PLACE"] = hp
        tr, net = bench.build_trainer(dev, c2w, cfg)
        tr.enable_graph_rng()
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for i in range(3):
                tr.train_step(data, it=i, epoch=0, scheduling_start=0)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = tr.train_step(data, it=0, epoch=0, scheduling_start=0)
        setups[hp] = (g, out, net)
    os.environ.pop("NERF_HEADS_PLACE", None)
    res = {hp: {"no_events": [], "events": []} for hp in args.places}
    checks = {hp: [] for hp in args.places}
    for _ in range(args.rounds):
        for hp in args.places:
            g, out, net = setups[hp]
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            w0 = net.layers0[0].weight.detach().double().sum().item()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                g.replay()
            torch.cuda.synchronize()
            res[hp]["no_events"].append(1e3 * (time.perf_counter() - t0) / args.steps)
            w1 = net.layers0[0].weight.detach().double().sum().item()
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
            t0 = time.perf_counter()
            evs[0].record()
            for i in range(args.steps):
                g.replay()
                evs[i + 1].record()
            torch.cuda.synchronize()
            res[hp]["events"].append(1e3 * (time.perf_counter() - t0) / args.steps)
            res[hp].setdefault("event_median", []).append(
                statistics.median(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)))
            loss = float(out["loss"].detach())
            checks[hp].append({"loss": loss, "finite": math.isfinite(loss), "weights_moved": w1 != w0})
    print(json.dumps({hp: {k: {"median": statistics.median(v), "rounds": v} for k, v in r.items()} | {"checks": checks[hp]}
                      for hp, r in res.items()}, indent=1))


if __name__ == "__main__":
    main()

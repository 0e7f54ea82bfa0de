"""A/B of backward-schedule environment settings on the cfg2 train step replayed as a hipGraph
(bench.py's graph mode) AND eager, settings interleaved over rounds.  The native backward reads
its NERF_* knobs while the step is enqueued, so each setting gets its own trainer and its own
captured graph.

    python scripts/graph_env_ab.py --rounds 3 --steps 30 default NERF_HEADS_PLACE=1
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

KEYS = ("NERF_HEADS_PLACE", "NERF_WGRAD_BATCH1", "NERF_WGRAD_SCHED", "NERF_BWD_CHAIN", "NERF_WGRAD_GROUPS")


def env_of(name):
    # (a "#tag" suffix names a repeat of a setting: "default#2" checks the harness's own spread)
    name = name.split("#", 1)[0]
    return {} if name == "default" else dict(kv.split("=", 1) for kv in name.split(","))


def set_env(env):
    for k in KEYS:
        os.environ.pop(k, None)
    os.environ.update(env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("settings", nargs="+")
    args = ap.parse_args()
    from model import _hip
    _hip.load_library()
    _hip.gemm_set_precision(2)
    dev = torch.device("cuda", 0)
    cfg = bench.make_cfg()
    data, c2w = bench.synthetic_scene(dev)
    runs = {}
    for name in args.settings:
        set_env(env_of(name))
        tr, _ = bench.build_trainer(dev, c2w, cfg)
        tr_g, _ = bench.build_trainer(dev, c2w, cfg)
        tr_g.enable_graph_rng()
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for i in range(3):
                tr_g.train_step(data, it=i, epoch=0, scheduling_start=0)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            tr_g.train_step(data, it=0, epoch=0, scheduling_start=0)
        runs[name] = (tr, g)
    res = {n: {"eager": [], "graph": []} for n in args.settings}
    it = 0
    for _ in range(args.rounds):
        for name in args.settings:
            tr, g = runs[name]
            set_env(env_of(name))
            for _ in range(3):
                tr.train_step(data, it=it, epoch=0, scheduling_start=0)
                it += 1
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                tr.train_step(data, it=it, epoch=0, scheduling_start=0)
                it += 1
            torch.cuda.synchronize()
            res[name]["eager"].append(1e3 * (time.perf_counter() - t0) / args.steps)
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                g.replay()
            torch.cuda.synchronize()
            res[name]["graph"].append(1e3 * (time.perf_counter() - t0) / args.steps)
    set_env({})
    print(json.dumps({n: {m: {"ms_per_step_median": statistics.median(v), "rounds": v} for m, v in r.items()}
                      for n, r in res.items()}, indent=1))


if __name__ == "__main__":
    main()

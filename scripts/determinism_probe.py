"""Probe: are the cfg2 train step's results independent of the head-reduce placement
(NERF_HEADS_PLACE 5, the default, forks k_heads_reduce to the side stream; 1 keeps it on the
caller's stream)?  The placement moves no arithmetic, so with the same seeds the two must give
bit-identical losses step after step; a difference points at a missing stream dependency.  Each
placement trains one trainer eagerly and one as replays of a captured step (bench.measure_graph's
recipe), every run from the same seeds; the per-step losses and the field parameters' checksums
are compared within each mode.

    python scripts/determinism_probe.py --steps 150 [--places 5 1]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def checksum(net):
    return [float(p.detach().double().sum()) for p in net.parameters()]


def run_eager(dev, data, c2w, cfg, steps):
    torch.cuda.manual_seed(7)
    tr, net = bench.build_trainer(dev, c2w, cfg)
    torch.cuda.manual_seed(7)
    losses = []
    for i in range(steps):
        out = tr.train_step(data, it=i, epoch=0, scheduling_start=0)
        losses.append(out["loss"].detach().clone())
    torch.cuda.synchronize()
    return [float(x) for x in losses], checksum(net)


def run_graph(dev, data, c2w, cfg, steps):
    torch.cuda.manual_seed(7)
    tr, net = bench.build_trainer(dev, c2w, cfg)
    tr.enable_graph_rng()
    torch.cuda.manual_seed(7)
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
    losses = []
    for _ in range(steps):
        g.replay()
        losses.append(out["loss"].detach().clone())
    torch.cuda.synchronize()
    return [float(x) for x in losses], checksum(net)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--places", nargs="+", default=["5", "1"])
    ap.add_argument("--modes", nargs="+", default=["graph", "eager"])
    args = ap.parse_args()
    from model import _hip
    _hip.load_library()
    _hip.gemm_set_precision(2)
    dev = torch.device("cuda", 0)
    cfg = bench.make_cfg()
    data, c2w = bench.synthetic_scene(dev)
    report = {}
    for mode in args.modes:
        runs = {}
        for hp in args.places:
            os.environ["NERF_HEADS_PLACE"] = hp
            runs[hp] = (run_graph if mode == "graph" else run_eager)(dev, data, c2w, cfg, args.steps)
        os.environ.pop("NERF_HEADS_PLACE", None)
        base_l, base_c = runs[args.places[0]]
        rep = {}
        for hp, (ls, cs) in runs.items():
            first = next((i for i, (a, b) in enumerate(zip(ls, base_l)) if a != b), None)
            rep[hp] = {"loss_first": ls[0], "loss_last": ls[-1], "loss_max": max(ls),
                       "finite": all(math.isfinite(v) for v in ls),
                       "first_step_differing_from_" + args.places[0]: first,
                       "params_equal_" + args.places[0]: cs == base_c,
                       "losses_every_10": ls[::10]}
        report[mode] = rep
        print(json.dumps({mode: {hp: {k: v for k, v in r.items() if k != "losses_every_10"} for hp, r in rep.items()}}),
              flush=True)
    print(json.dumps(report, indent=1))


if __name__ == "__main__":
    main()

"""A/B of GEMM tile policies / backward-schedule settings on the real cfg2 training step (bench.py's workload), one
trainer, settings interleaved over rounds; prints ms/step per setting (median of rounds).

    python scripts/step_ab.py [--steps 20 --rounds 3]
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

# name -> (nt policy, tn policy, env overrides); 0 = default
SETTINGS = {
    "default": (0, 0, {}),
    "tail1": (0, 0, {"NERF_TAIL_MAIN": "1"}),
    "tail3": (0, 0, {"NERF_TAIL_MAIN": "3"}),
    "tn3": (0, 3, {}),
    "heads_joint": (0, 0, {"NERF_HEADS_SIDE": "0"}),
    "chain": (0, 0, {"NERF_CHAIN": "1"}),
    "per_layer": (0, 0, {"NERF_CHAIN": "0"}),
    "dw_two_launch": (0, 0, {"NERF_DW_SEG": "0"}),
    "python_bwd": (0, 0, {"NERF_NATIVE_BWD": "0"}),
    "wgrad2": (0, 0, {"NERF_WGRAD_SCHED": "2"}),
    "wgrad3": (0, 0, {"NERF_WGRAD_SCHED": "3"}),
    "heads_before": (0, 0, {"NERF_HEADS_PLACE": "1"}),
    "heads_after": (0, 0, {"NERF_HEADS_PLACE": "2"}),
    "heads_part": (0, 0, {"NERF_HEADS_PLACE": "3"}),
    "wgrad1": (0, 0, {"NERF_WGRAD_SCHED": "1"}),
    "heads_reduce_side": (0, 0, {"NERF_HEADS_PLACE": "5"}),
    "batch1_main": (0, 0, {"NERF_WGRAD_BATCH1": "1"}),
}
ENV_KEYS = ("NERF_TAIL_MAIN", "NERF_HEADS_SIDE", "NERF_CHAIN", "NERF_DW_SEG", "NERF_NATIVE_BWD", "NERF_WGRAD_SCHED",
            "NERF_HEADS_PLACE", "NERF_WGRAD_BATCH1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--settings", nargs="+", default=list(SETTINGS))
    args = ap.parse_args()
    from model import _hip
    _hip.load_library()
    _hip.gemm_set_precision(2)
    dev = torch.device("cuda", 0)
    cfg = bench.make_cfg()
    data, c2w = bench.synthetic_scene(dev)
    trainer, _ = bench.build_trainer(dev, c2w, cfg)
    it = 0
    res = {k: [] for k in args.settings}
    trainers = {name: (bench.build_trainer(dev, c2w, cfg)[0] if name != "default" else trainer)
                for name in args.settings}
    for _ in range(args.rounds):
        for name in args.settings:
            trainer = trainers[name]
            nt, tn, env = SETTINGS[name]
            for k in ENV_KEYS:
                os.environ.pop(k, None)
            os.environ.update(env)
            _hip.gemm_set_policy(nt, tn)
            for _ in range(3):
                trainer.train_step(data, it=it, epoch=0, scheduling_start=0)
                it += 1
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                ld = trainer.train_step(data, it=it, epoch=0, scheduling_start=0)
                it += 1
            torch.cuda.synchronize()
            res[name].append(1e3 * (time.perf_counter() - t0) / args.steps)
            if not torch.isfinite(ld["loss"]).item():
                raise RuntimeError(f"{name}: non-finite loss")
    _hip.gemm_set_policy(0, 0)
    print(json.dumps({k: {"ms_per_step_median": statistics.median(v), "rounds": v} for k, v in res.items()}))


if __name__ == "__main__":
    main()

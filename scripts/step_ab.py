"""A/B of GEMM tuning knobs on the real cfg2 training step (bench.py's workload), one
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

# name -> (nt policy, tn policy, dW target blocks, non-temporal NT stores); 0 = default
SETTINGS = {
    "default": (0, 0, 0, 0),
    "side_hi": (0, 0, 0, 0),
    "old_default": (0, 0, 0, 0),
    "side2": (0, 0, 0, 0),
    "tail2": (0, 0, 0, 0),
    "tail3": (0, 0, 0, 0),
    "tail4": (0, 0, 0, 0),
    "side2_tail2": (0, 0, 0, 0),
    "tside2": (0, 0, 0, 0),
    "tside3": (0, 0, 0, 0),
    "tside4": (0, 0, 0, 0),
    "tail1": (0, 0, 0, 0),
    "tail2_ts1": (0, 0, 0, 0),
    "tail2_ts2": (0, 0, 0, 0),
    "tail1_ts2": (0, 0, 0, 0),
    "store_nt": (0, 0, 0, 1),
    "store_sc1": (0, 0, 0, 2),
    "tn128_b256": (0, 1, 256, 0),
    "tn128_b512": (0, 1, 512, 0),
    "tn128_b1024": (0, 1, 1024, 0),
    "tn256_b128": (0, 0, 128, 0),
    "tn_pair": (0, 4, 0, 0),
    "tn_quad": (0, 5, 0, 0),
    "tn_pair8": (0, 7, 0, 0),
    "seg2_splits": (0, 0, 0, 0),
    "tn_narrow8": (0, 8, 0, 0),
    "tn3": (0, 3, 0, 0),
}


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
    trainers = {}
    for name in args.settings:
        # side_hi: the weight-gradient side stream at high priority (a trainer of its own: the
        # stream is created on the first backward)
        os.environ["NERF_SIDE_PRIORITY"] = "-1" if name == "side_hi" else "0"
        trainers[name] = bench.build_trainer(dev, c2w, cfg)[0] if name != "default" else trainer
        trainers[name].train_step(data, it=0, epoch=0, scheduling_start=0)
    os.environ.pop("NERF_SIDE_PRIORITY", None)
    # backward schedule (field.py): weight-gradient side streams / layers whose dW runs on main
    SCHED = {"old_default": ("1", "0", "0"), "side2": ("2", "0", "0"), "tail2": ("1", "2", "0"), "tail3": ("1", "3", "0"), "tail4": ("1", "4", "0"),
             "side2_tail2": ("2", "2", "0"), "tside2": ("1", "0", "2"), "tside3": ("1", "0", "3"),
             "tside4": ("1", "0", "4"), "tail1": ("1", "1", "0"), "tail2_ts1": ("1", "2", "1"),
             "tail2_ts2": ("1", "2", "2"), "tail1_ts2": ("1", "1", "2")}
    for _ in range(args.rounds):
        for name in args.settings:
            trainer = trainers[name]
            if name in SCHED:
                (os.environ["NERF_SIDE_STREAMS"], os.environ["NERF_TAIL_MAIN"],
                 os.environ["NERF_TAIL_SIDE"]) = SCHED[name]
            else:   # the library defaults
                for k in ("NERF_SIDE_STREAMS", "NERF_TAIL_MAIN", "NERF_TAIL_SIDE"):
                    os.environ.pop(k, None)
            if name == "seg2_splits":
                os.environ["NERF_SEG2_SPLITS"] = "1"
            else:
                os.environ.pop("NERF_SEG2_SPLITS", None)
            nt, tn, blocks, snt = SETTINGS[name]
            _hip.gemm_set_policy(nt, tn)
            _hip.gemm_set_dw_blocks(blocks)
            _hip.gemm_set_store_hint(snt)
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
    _hip.gemm_set_dw_blocks(0)
    _hip.gemm_set_store_hint(0)
    print(json.dumps({k: {"ms_per_step_median": statistics.median(v), "rounds": v} for k, v in res.items()}))


if __name__ == "__main__":
    main()

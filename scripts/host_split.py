"""Host (enqueue) time of the cfg2 train step split by phase: FieldRunner.forward and
FieldRunner.backward (the autograd engine runs the latter on its device thread) are wrapped
with perf_counter; the rest of train_step is the remainder.  No GPU sync inside the timed
steps, so the numbers are the host's own cost, not the GPU's.

    python scripts/host_split.py [--steps 40]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    args = ap.parse_args()
    from model import _hip, field
    _hip.load_library()
    _hip.gemm_set_precision(2)
    acc = {"forward": 0.0, "backward": 0.0}
    for name in acc:
        orig = getattr(field.FieldRunner, name)

        def wrap(self, *a, _o=orig, _n=name, **k):
            t = time.perf_counter()
            r = _o(self, *a, **k)
            acc[_n] += time.perf_counter() - t
            return r
        setattr(field.FieldRunner, name, wrap)
    dev = torch.device("cuda", 0)
    cfg = bench.make_cfg()
    data, c2w = bench.synthetic_scene(dev)
    trainer, _ = bench.build_trainer(dev, c2w, cfg)
    for i in range(5):
        trainer.train_step(data, it=i, epoch=0, scheduling_start=0)
    torch.cuda.synchronize()
    for k in acc:
        acc[k] = 0.0
    t0 = time.perf_counter()
    for i in range(args.steps):
        trainer.train_step(data, it=5 + i, epoch=0, scheduling_start=0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    n = args.steps
    print(json.dumps({"enqueue_ms_per_step": 1e3 * (t1 - t0) / n, "drained_ms_per_step": 1e3 * (t2 - t0) / n,
                      "field_forward_host_ms": 1e3 * acc["forward"] / n,
                      "field_backward_host_ms": 1e3 * acc["backward"] / n,
                      "rest_host_ms": 1e3 * (t1 - t0 - acc["forward"] - acc["backward"]) / n}))


if __name__ == "__main__":
    main()

"""Which Python lines launch the small torch kernels of a training step (fills, device copies,
elementwise adds)?  torch.profiler with stacks over a few eager steps; prints, per op, the
self device time per step and the top frames of the repo's code that issued it.

    python scripts/glue_sources.py [--full]     (--full: config 3, else config 2)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda")
    from model import _hip
    _hip.load_library()
    _hip.gemm_set_precision(2)
    if "--full" in sys.argv:
        import bench_full as bf
        trainer, datas = bf.setup(dev)
        step = lambda it: trainer.train_step(datas[it % 2], it=it + 1, epoch=0, scheduling_start=0)  # noqa: E731
    else:
        cfg = bench.make_cfg()
        data, c2w = bench.synthetic_scene(dev)
        trainer, _ = bench.build_trainer(dev, c2w, cfg)
        step = lambda it: trainer.train_step(data, it=it, epoch=0, scheduling_start=0)  # noqa: E731
    for i in range(5):
        step(i)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    n = 4
    with torch.profiler.profile(activities=acts, with_stack=True) as prof:
        for i in range(n):
            step(5 + i)
        torch.cuda.synchronize()
    rows = prof.key_averages(group_by_stack_n=6)
    keep = [r for r in rows if r.self_device_time_total > 0 and r.key.startswith("aten::")]
    keep.sort(key=lambda r: -r.self_device_time_total)
    for r in keep[:30]:
        stack = [f for f in r.stack if "torch/" not in f and "<built-in" not in f][:4] or list(r.stack)[:4]
        print(f"{r.self_device_time_total / n:8.1f} us/step {r.count / n:5.1f}/step  {r.key}")
        for f in stack:
            print(f"            {f}")


if __name__ == "__main__":
    main()

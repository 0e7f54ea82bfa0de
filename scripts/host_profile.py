"""Host-side (Python / ctypes enqueue) profile of the training step (cfg2 or cfg3 shape)."""
import cProfile
import os
import pstats
import sys
import time

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
        trainer, datas = bench.cfg3_setup(dev)
        step = lambda it: trainer.train_step(datas[it % 2], it=it + 1, epoch=0, scheduling_start=0)
    else:
        cfg = bench.make_cfg()
        data, c2w = bench.synthetic_scene(dev)
        trainer, net = bench.build_trainer(dev, c2w, cfg)
        step = lambda it: trainer.train_step(data, it=it, epoch=0, scheduling_start=0)
    if "--same-thread" in sys.argv:
        # the autograd engine runs CUDA backwards on a worker thread, invisible to cProfile;
        # run them on this thread so FieldRunner.backward's host time shows up
        torch.autograd.set_multithreading_enabled(False)
    for i in range(5):
        step(i)
    torch.cuda.synchronize()
    if "--plain" in sys.argv:
        # no profiler: host enqueue time per step vs the drained (GPU-inclusive) time
        t0 = time.perf_counter()
        for i in range(40):
            step(5 + i)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"plain: enqueue {1e3 * (t1 - t0) / 40:.3f} ms/step, drained {1e3 * (t2 - t0) / 40:.3f} ms/step")
        return
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for i in range(20):
        step(5 + i)
    pr.disable()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"enqueue {1e3 * (t1 - t0) / 20:.3f} ms/step (profiled), drained {1e3 * (t2 - t0) / 20:.3f} ms/step")
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)
    pstats.Stats(pr).sort_stats("cumulative").print_stats(60)


if __name__ == "__main__":
    main()

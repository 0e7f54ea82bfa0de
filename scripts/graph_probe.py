"""Probe: capture Trainer.train_step in a hipGraph (torch.cuda.graph) and compare eager vs
replay step time, plus loss agreement after identical numbers of steps."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda")
    from model import _hip
    _hip.load_library()
    _hip.gemm_set_precision(2 if "--h16" in sys.argv else 1 if "--x6" in sys.argv else 0)
    cfg = bench.make_cfg()
    data, c2w = bench.synthetic_scene(dev)
    trainer, net = bench.build_trainer(dev, c2w, cfg)
    torch.cuda.manual_seed(1000)

    def step():
        return trainer.train_step(data, it=0, epoch=0, scheduling_start=0)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / 20
    host = []
    for _ in range(20):                     # host enqueue time of one step (GPU drained first)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        step()
        host.append(time.perf_counter() - t1)
    torch.cuda.synchronize()
    host.sort()
    print(f"eager: {eager * 1e3:.3f} ms/step  host enqueue median {host[10] * 1e3:.3f} ms/step", flush=True)
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g):
            out = step()
    except Exception as e:  # report and stop
        print("capture failed:", type(e).__name__, str(e)[:2000], flush=True)
        raise
    print("captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    rep = (time.perf_counter() - t0) / 20
    print(f"graph replay: {rep * 1e3:.3f} ms/step  loss {out['loss'].item():.5f}", flush=True)


if __name__ == "__main__":
    main()

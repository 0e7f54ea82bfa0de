"""hipGraph capture of the training step (cfg2 and cfg3 shapes, GEMM precision mode 2):
replays draw new rays (device seed counter), advance Adam, and track the eager step's
losses (GPU only)."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

pytestmark = pytest.mark.gpu


def _capture(step, warm=3):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warm):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = step()
    return g, out


def test_graph_replay_cfg2_trains_on_fresh_rays(dev):
    import bench
    from model import _hip
    old = _hip.gemm_get_precision()
    _hip.gemm_set_precision(2)
    try:
        cfg = bench.make_cfg()
        data, c2w = bench.synthetic_scene(dev)
        trainer, net = bench.build_trainer(dev, c2w, cfg)
        trainer.enable_graph_rng()
        g, out = _capture(lambda: trainer.train_step(data, it=0, epoch=0, scheduling_start=0))
        losses, ctrs = [], []
        w0 = net.layers0[0].weight.detach().clone()
        for _ in range(30):
            g.replay()
            losses.append(out["loss"].item())
            ctrs.append(trainer.seed_counter.item())
        assert ctrs == sorted(set(ctrs)) and ctrs[-1] - ctrs[0] == 29      # one draw per replay
        assert len(set(round(x, 7) for x in losses)) > 20                   # new rays every step
        assert all(torch.isfinite(torch.tensor(losses)))
        assert sum(losses[-5:]) < sum(losses[:5])                           # it trains
        assert not torch.equal(net.layers0[0].weight.detach(), w0)
    finally:
        _hip.gemm_set_precision(old)

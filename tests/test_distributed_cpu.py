"""Multi-process data parallelism on the CPU (gloo, world_size 2): the Trainer's flat
gradient all-reduce averages exactly, and per-rank ray shards reproduce the single-
process gradient of the concatenated batch."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import model as mdl
from oracle import nerf_oracle as orc
from tests.helpers import make_cfg, synthetic_rays


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    net = orc.OracleNerf(hidden_dim=16)
    R, S = 32, 8
    b = synthetic_rays(R=R, S=S, H=30, W=40, seed=7)
    lo, hi = rank * R // world, (rank + 1) * R // world
    out = orc.render_nope_nerf(net, b["pixels"][:, lo:hi], b["depth"][:, lo:hi], b["K"], b["w2c"], b["scale"],
                               {"num_points": S}, noise=b["noise"][:, lo:hi])
    gt = torch.full((1, hi - lo, 3), 0.5)
    # per-rank mean over its own rays; the average over ranks = the mean over all rays
    loss = ((out["rgb"] - gt) ** 2).sum() / (hi - lo)
    loss.backward()
    cfg = make_cfg(hidden=16)
    tr = mdl.Trainer(net, None, cfg["training"], device=torch.device("cpu"))
    assert tr.world_size == world
    tr.allreduce_grads()
    q.put((rank, [p.grad.clone().numpy() for p in net.parameters()]))  # by value, not shared memory
    dist.barrier()
    dist.destroy_process_group()


def test_ray_sharded_gradients_equal_full_batch():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(0)
    net = orc.OracleNerf(hidden_dim=16)
    R, S = 32, 8
    b = synthetic_rays(R=R, S=S, H=30, W=40, seed=7)
    out = orc.render_nope_nerf(net, b["pixels"], b["depth"], b["K"], b["w2c"], b["scale"], {"num_points": S},
                               noise=b["noise"])
    loss = ((out["rgb"] - 0.5) ** 2).sum() / R
    loss.backward()
    for g0, g1, p in zip(res[0], res[1], net.parameters()):
        g0, g1 = torch.from_numpy(g0), torch.from_numpy(g1)
        assert torch.allclose(g0, g1)                       # every rank holds the same average
        assert torch.allclose(g0, p.grad, atol=1e-6, rtol=1e-4)


def _render_worker(rank, world, port, q, n_rays):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from model.render_dist import render_frame_sharded, tile_bounds
    torch.manual_seed(0)
    net = orc.OracleNerf(hidden_dim=16)
    b = synthetic_rays(R=n_rays, S=8, H=30, W=40, seed=11)
    seen = []

    def tile(start, end):                   # the CPU restatement stands in for the HIP renderer
        seen.append((start, end))
        with torch.no_grad():
            o = orc.render_nope_nerf(net, b["pixels"][:, start:end], b["depth"][:, start:end], b["K"], b["w2c"],
                                     b["scale"], {"num_points": 8}, noise=None, eval_=True)
        return o["rgb"].reshape(-1, 3), o["depth_pred"].reshape(-1)

    rgb, depth = render_frame_sharded(tile, n_rays, torch.device("cpu"))
    assert seen == [tile_bounds(n_rays, rank, world)[:2]]     # one contiguous tile per rank
    q.put((rank, rgb.numpy(), depth.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_full_frame_render_sharded_all_gather():
    """config 4: contiguous ray tiles per rank (last one padded) + one all-gather give
    every rank the frame the single-process render produces (uneven split: 3 ranks)."""
    world, n_rays = 3, 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_render_worker, args=(r, world, port, q, n_rays)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, rgb, depth = q.get(timeout=120)
        res[r] = (torch.from_numpy(rgb), torch.from_numpy(depth))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(0)
    net = orc.OracleNerf(hidden_dim=16)
    b = synthetic_rays(R=n_rays, S=8, H=30, W=40, seed=11)
    with torch.no_grad():
        o = orc.render_nope_nerf(net, b["pixels"], b["depth"], b["K"], b["w2c"], b["scale"], {"num_points": 8},
                                 noise=None, eval_=True)
    for r in range(world):
        assert res[r][0].shape == (n_rays, 3)
        assert torch.allclose(res[r][0], o["rgb"].reshape(-1, 3), atol=1e-6)
        assert torch.allclose(res[r][1], o["depth_pred"].reshape(-1), atol=1e-5)
        assert torch.equal(res[r][0], res[0][0])

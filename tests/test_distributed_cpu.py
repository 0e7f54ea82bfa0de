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


def _missing_grad_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(4, 3), torch.nn.Linear(3, 2))
    cfg = make_cfg(hidden=16)
    tr = mdl.Trainer(net, None, cfg["training"], device=torch.device("cpu"))
    ps = tr.bucket_params()
    # parameter 0: only rank 0 has a gradient; parameter 2: no rank has one; rest: all
    for i, p in enumerate(ps):
        if i == 2 or (i == 0 and rank == 1):
            p.grad = None
        else:
            p.grad = torch.full_like(p, float(10 * rank + i))
    tr.allreduce_grads()
    q.put((rank, [None if p.grad is None else p.grad.clone().numpy() for p in ps]))
    dist.barrier()
    dist.destroy_process_group()


def test_allreduce_fixed_layout_with_missing_gradient():
    """A rank without a gradient for some parameter still sends the same bucket size (no
    hang, zeros counted in the average); a parameter no rank has a gradient for stays None
    on every rank (torch Adam skips it everywhere alike)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_missing_grad_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        g = res[r]
        assert g[2] is None
        assert torch.allclose(torch.from_numpy(g[0]), torch.full(g[0].shape, 0.0 / 2))      # (0 + missing) / 2
        assert torch.allclose(torch.from_numpy(g[1]), torch.full(g[1].shape, (1 + 11) / 2))
        assert torch.allclose(torch.from_numpy(g[3]), torch.full(g[3].shape, (3 + 13) / 2))


def test_bench_launcher_spawns_ranks():
    """`bench.py --gpus 2` without WORLD_SIZE launches its own two ranks (a child
    torch.distributed.run) and reports n_gpus from the process group; --plumbing swaps the
    GPU step for a CPU gloo check of the fixed-layout gradient all-reduce."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--plumbing", "--gpus", "2"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["plumbing"] and line["n_gpus"] == 2 and line["world_size"] == 2
    assert line["bucket_elems"] > 595_000            # NeRF (595 844) + pose + distortion parameters
    # the N > 1 attribution fields bench.py prints under RCCL (rank_attribution), from the same code
    assert line["allreduce_ms_per_step"] > 0 and line["multi_gpu"]["world_size"] == 2
    mg = line["multi_gpu"]
    assert len(mg["per_rank"]) == 2 and mg["allreduce_ms_per_step_min"] <= mg["allreduce_ms_per_step"]
    assert mg["rays_per_s_per_rank_min"] <= mg["rays_per_s_per_rank_max"]
    assert mg["compute_ms_per_step_min"] <= mg["compute_ms_per_step_max"]
    bad = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--plumbing", "--gpus", "3"],
                         capture_output=True, text=True, timeout=120, env=dict(env, WORLD_SIZE="2"), cwd=root)
    assert bad.returncode != 0 and "WORLD_SIZE" in bad.stderr


def _inplace_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = make_cfg(hidden=64, S=16)
    torch.manual_seed(0)
    net = mdl.OfficialStaticNerf(cfg)
    model = mdl.get_model(mdl.Renderer(net, cfg["rendering"]), cfg)
    pose = mdl.LearnPose(2, True, True, cfg)
    distn = mdl.Learn_Distortion(2, True, True, cfg)
    tr = mdl.Trainer(model, None, cfg["training"], device=torch.device("cpu"), pose_param_net=pose,
                     distortion_net=distn)
    flat = tr._bucket_buffer(torch.device("cpu"))
    runner = net.hip_runner()
    assert runner.grad_buffer is not None and runner.grad_buffer.data_ptr() == flat.data_ptr()
    field = runner.param_list()
    # what FieldRunner.backward does: the field gradients are views of grad_buffer in
    # param_list() order (autograd hands them on as param.grad); the pose / distortion
    # gradients are ordinary autograd tensors
    off = 0
    for i, p in enumerate(field):
        p.grad = runner.grad_buffer[off:off + p.numel()].view_as(p)
        p.grad.fill_(float(rank + i))
        off += p.numel()
    ptrs = [p.grad.data_ptr() for p in field]
    extra = [p for p in tr.bucket_params() if all(p is not f for f in field)]
    for i, p in enumerate(extra):
        p.grad = torch.full_like(p, float(100 * rank + i))
    tr.allreduce_grads()
    base, end = flat.data_ptr(), flat.data_ptr() + flat.numel() * 4
    ok_inplace = [p.grad.data_ptr() == ptr for p, ptr in zip(field, ptrs)]      # reduced where they lie
    ok_views = [base <= p.grad.data_ptr() < end for p in extra]                  # no copy back: bucket views
    vals = [float(p.grad.flatten()[0]) for p in field] + [float(p.grad.flatten()[0]) for p in extra]
    q.put((rank, ok_inplace, ok_views, vals, len(field)))
    dist.barrier()
    dist.destroy_process_group()


def test_allreduce_in_place_on_field_gradient_buffer():
    """The NeRF field's gradients are written by the runner into the Trainer's persistent
    bucket and all-reduced there: after allreduce_grads every field p.grad still points at
    the same storage (no torch.cat, no copy back), the pose / distortion gradients are views
    of the same bucket, and every value is the average over the ranks."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_inplace_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, rest) for r, *rest in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        ok_inplace, ok_views, vals, n_field = res[r]
        assert all(ok_inplace) and all(ok_views)
        for i, v in enumerate(vals[:n_field]):
            assert v == (0 + i + 1 + i) / 2
        for i, v in enumerate(vals[n_field:]):
            assert v == (i + 100 + i) / 2

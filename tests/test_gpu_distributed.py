"""The HIP training step under a process group, on the
one GPU of the box: two ranks (gloo carries the collective; RCCL needs one GPU per rank)
each render half of a ray batch through the full HIP path -- NeRF forward / backward, pose
and distortion learning -- and average their gradients with Trainer.allreduce_grads.  The
averaged gradients must equal the single-process gradients of the whole batch, and one
HipAdam / Adam step later the parameters must be identical on both ranks."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

H, W, FX = 40, 56, 50.0
R, S, D = 256, 32, 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(dev):
    import model as mdl
    from model.optim import HipAdam
    from tests.helpers import camera_K, make_cfg, rigid_c2w
    cfg = make_cfg(hidden=D, S=S)
    t = cfg["training"]
    t["n_training_points"] = R
    t["pc_weight"], t["rgb_s_weight"] = [0.0, 0.0], [0.0, 0.0]
    g = torch.Generator().manual_seed(5)
    yy, xx = torch.meshgrid(torch.linspace(0, 1, H), torch.linspace(0, 1, W), indexing="ij")
    img = torch.stack([0.5 + 0.4 * torch.sin(5 * xx + yy), 0.5 + 0.3 * torch.cos(4 * yy), 0.2 + 0.6 * xx * yy])
    depth = 1.5 + 4.0 * torch.rand(1, H, W, generator=g)       # no holes: every rank masks 0 rays
    c2w = torch.stack([rigid_c2w(3, 0.2), rigid_c2w(4, 0.2)])
    data = {"img": img.unsqueeze(0).to(dev), "img.idx": torch.tensor([0]), "img.depth": depth.to(dev),
            "img.depth_mask": torch.ones(1, H, W, dtype=torch.bool), "img.camera_mat": camera_K(H, W, FX, FX).to(dev),
            "img.scale_mat": torch.eye(4).unsqueeze(0).to(dev), "img.pose_gt": c2w[0:1].to(dev)}
    torch.manual_seed(42)
    net = mdl.OfficialStaticNerf(cfg)
    model = mdl.get_model(mdl.Renderer(net, cfg["rendering"], device=dev), cfg, device=dev)
    opt = HipAdam(model.parameters(), lr=1e-3)
    pose = mdl.LearnPose(2, True, True, cfg, init_c2w=c2w.to(dev)).to(dev)
    with torch.no_grad():
        pose.r.copy_(0.01 * torch.randn(2, 3, generator=g))
        pose.t.copy_(0.02 * torch.randn(2, 3, generator=g))
    opt_pose = torch.optim.Adam(pose.parameters(), lr=1e-3)
    distn = mdl.Learn_Distortion(2, True, True, cfg).to(dev)
    with torch.no_grad():
        distn.global_scales.copy_(torch.tensor([[1.1], [0.95]]))
    opt_dist = torch.optim.Adam(distn.parameters(), lr=1e-3)
    tr = mdl.Trainer(model, opt, t, device=dev, optimizer_pose=opt_pose, pose_param_net=pose,
                     optimizer_distortion=opt_dist, distortion_net=distn)
    gi = torch.Generator().manual_seed(9)
    ray_idx = torch.randperm(H * W, generator=gi)[:R]
    noise = torch.rand(1, R, S, generator=gi)
    return tr, data, ray_idx, noise


def _grads(tr):
    return [None if p.grad is None else p.grad.detach().cpu().clone().numpy() for p in tr.bucket_params()]


def _rank(rank, world, port, q):
    try:
        _rank_body(rank, world, port, q)
    except BaseException:                    # report instead of leaving the parent waiting
        import traceback
        q.put((rank, "error", traceback.format_exc()))
        raise


def _rank_body(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    tr, data, ray_idx, noise = _setup(dev)
    assert tr.world_size == world and tr.rank == rank
    lo, hi = rank * R // world, (rank + 1) * R // world
    tr.inject = (ray_idx[lo:hi], noise[:, lo:hi])
    tr.n_training_points = hi - lo
    tr.train_step(data, it=0, epoch=0, scheduling_start=0)       # backward + all-reduce + optimiser steps
    grads = _grads(tr)
    params = [p.detach().cpu().clone().numpy() for p in tr.bucket_params()]
    q.put((rank, grads, params))
    dist.barrier()
    dist.destroy_process_group()


def test_hip_train_step_under_process_group_matches_full_batch(dev):
    from model import _hip
    _hip.load_library()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    import time
    res, t0 = {}, time.time()
    while len(res) < world:
        try:
            r, g, pr = q.get(timeout=5)
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f"a rank exited with {dead} before reporting"
            assert time.time() - t0 < 240, "ranks did not report within 240 s"
            continue
        assert g != "error", f"rank {r} failed:\n{pr}"
        res[r] = (g, pr)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0

    # single process, the whole batch: same parameters, rays and noise
    tr, data, ray_idx, noise = _setup(dev)
    tr.inject = (ray_idx, noise)
    ld = tr.compute_loss(data, it=0, epoch=0, scheduling_start=0)
    ld["loss"].backward()
    full = _grads(tr)
    for i, (g0, g1, gf) in enumerate(zip(res[0][0], res[1][0], full)):
        assert (g0 is None) == (g1 is None) == (gf is None), i
        if gf is None:
            continue
        g0, g1, gf = torch.from_numpy(g0).double(), torch.from_numpy(g1).double(), torch.from_numpy(gf).double()
        assert torch.equal(g0, g1), i                       # every rank holds the same average
        # the per-rank GEMM reductions split the sample sum differently than one launch
        rel = ((g0 - gf).norm() / gf.norm().clamp_min(1e-30)).item()
        assert rel < 2e-3, (i, rel)
    for p0, p1 in zip(res[0][1], res[1][1]):                # replicated optimiser: identical parameters
        assert (p0 == p1).all()

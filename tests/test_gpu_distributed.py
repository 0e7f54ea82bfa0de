"""The HIP path under a process group, on the one GPU of the box:
two ranks (gloo carries the collectives; RCCL needs one GPU per rank) each run their share
of the work through the full HIP path; and the gradient all-reduce on RCCL itself with one rank.

* config 5 (training): each rank renders half of a ray batch -- NeRF forward / backward, pose
  and distortion learning -- and Trainer.allreduce_grads averages the gradients in place on
  its persistent bucket.  The averaged gradients must equal the single-process HIP gradients
  of the whole batch AND the oracle's full-batch gradients (compute_loss_full), the NeRF
  gradients must be views of the Trainer's bucket, and one optimiser step later the
  parameters must be identical on both ranks.  Cases: 256 x 32 at D = 64, and the bench shape
  1024 x 128 at D = 256 on a 188 x 621 image.
* config 4 (render): model.render_dist.render_image cuts a 188 x 621 frame into one ray tile per
  rank, renders each tile with the fused per-ray eval kernel (D = 256, S = 128) and all-gathers
  (rgb, depth); every rank's frame must be bit-identical to the single-process render."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CASES = {   # name: (H, W, fx, rays, samples, hidden)
    "small": (40, 56, 50.0, 256, 32, 64),
    "cfg5": (188, 621, 362.5, 1024, 128, 256),
}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(dev, case):
    import model as mdl
    from model.optim import HipAdam
    from tests.helpers import camera_K, make_cfg, rigid_c2w
    H, W, FX, R, S, D = CASES[case]
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
    return tr, data, ray_idx, noise, cfg, (net, pose, distn, c2w)


def _grads(tr):
    return [None if p.grad is None else p.grad.detach().cpu().clone().numpy() for p in tr.bucket_params()]


def _spawn(target, world, *args, timeout=300):
    """Start `world` ranks, collect one report per rank; on any failure the ranks are killed
    (a rank blocked on a full result pipe would otherwise keep the test process from exiting)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args, daemon=True) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    import time
    res, t0 = {}, time.time()
    try:
        while len(res) < world:
            try:
                r, *payload = q.get(timeout=5)
            except queue.Empty:
                dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
                assert not dead, f"a rank exited with {dead} before reporting"
                assert time.time() - t0 < timeout, f"ranks did not report within {timeout} s"
                continue
            is_err = isinstance(payload[0], str) and payload[0] == "error"
            assert not is_err, f"rank {r} failed:\n{payload[1]}"
            res[r] = payload
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    return res


def _run_rank(rank, world, port, q, body_name, *args, backend="gloo"):
    """Rank entry point (module level: spawn pickles it by name): joins the gloo (or, one rank per
    GPU, the nccl = RCCL) group on 127.0.0.1, runs the named body, reports a traceback instead of
    leaving the parent waiting."""
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        dist.init_process_group(backend, rank=rank, world_size=world,
                                **({"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}))
        globals()[body_name](rank, world, q, *args)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        import traceback
        q.put((rank, "error", traceback.format_exc()))
        raise


def _train_body(rank, world, q, case):
    dev = torch.device("cuda:0")
    tr, data, ray_idx, noise, _, _ = _setup(dev, case)
    assert tr.world_size == world and tr.rank == rank
    R = ray_idx.numel()
    lo, hi = rank * R // world, (rank + 1) * R // world
    tr.inject = (ray_idx[lo:hi], noise[:, lo:hi])
    tr.n_training_points = hi - lo
    tr.train_step(data, it=0, epoch=0, scheduling_start=0)       # backward + all-reduce + optimiser steps
    grads = _grads(tr)
    # the NeRF gradients were reduced where the HIP backward wrote them: views of the bucket
    flat = tr._flat
    runner = tr.model.renderer.model.hip_runner()
    base, end = flat.data_ptr(), flat.data_ptr() + 4 * flat.numel()
    in_bucket = all(base <= p.grad.data_ptr() < end for p in runner.param_list())
    params = [p.detach().cpu().clone().numpy() for p in tr.bucket_params()]
    q.put((rank, grads, params, in_bucket))



def _run_rank_rccl(rank, world, port, q, body_name, *args):
    _run_rank(rank, world, port, q, body_name, *args, backend="nccl")


def _rccl_body(rank, world, q, case):
    """The data-parallel gradient path on RCCL itself (one rank: the box has one GPU): the HIP
    backward writes the NeRF gradients into the Trainer's bucket, allreduce_grads runs the ONE
    in-place RCCL all-reduce on it, and every gradient must come back bit-identical (a sum over
    one rank, times 1.0) as a view of the bucket."""
    dev = torch.device("cuda:0")
    tr, data, ray_idx, noise, _, _ = _setup(dev, case)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    tr.inject = (ray_idx, noise)
    tr._bucket_buffer(dev)                      # as train_step does under a process group
    runner = tr.model.renderer.model.hip_runner()
    runner.release_grad_buffer()
    for _, o in tr._modules_and_optims():
        if o is not None:
            o.zero_grad()
    ld = tr.compute_loss(data, it=0, epoch=0, scheduling_start=0)
    ld["loss"].backward()
    flat = tr._flat
    base, end = flat.data_ptr(), flat.data_ptr() + 4 * flat.numel()
    written_in_place = all(base <= p.grad.data_ptr() < end for p in runner.param_list())
    before = _grads(tr)
    tr.allreduce_grads()
    torch.cuda.synchronize()
    after = _grads(tr)
    views = all(p.grad is None or base <= p.grad.data_ptr() < end for p in tr.bucket_params())
    q.put((rank, before, after, written_in_place, views))


@pytest.mark.parametrize("case", list(CASES))
def test_allreduce_grads_on_rccl(dev, case):
    res = _spawn(_run_rank_rccl, 1, "_rccl_body", case)
    before, after, written_in_place, views = res[0]
    assert written_in_place, "the HIP backward did not write the NeRF gradients into the bucket"
    assert views, "a gradient is not a view of the all-reduce bucket"
    assert len(before) == len(after)
    for i, (b, a) in enumerate(zip(before, after)):
        assert (b is None) == (a is None), i
        if b is not None:
            assert (b == a).all(), i


def _nrel(a, b):
    a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("case", list(CASES))
def test_hip_train_step_under_process_group_matches_full_batch(dev, case):
    from model import _hip
    from oracle import nerf_oracle as orc
    _hip.load_library()
    world = 2
    res = _spawn(_run_rank, world, "_train_body", case)
    for r in range(world):
        assert res[r][2], f"rank {r}: NeRF gradients are not views of the all-reduce bucket"

    # single process, the whole batch: same parameters, rays and noise
    tr, data, ray_idx, noise, cfg, (net, pose, distn, c2w) = _setup(dev, case)
    o_net = orc.OracleNerf(hidden_dim=net.hidden_dim)
    o_net.load_state_dict({k: v.cpu() for k, v in net.state_dict().items()})
    o_pose = {"r": pose.r.detach().cpu().clone().requires_grad_(True),
              "t": pose.t.detach().cpu().clone().requires_grad_(True), "init_c2w": c2w.clone()}
    o_dist = {"scales": distn.global_scales.detach().cpu().clone().requires_grad_(True),
              "shifts": distn.global_shifts.detach().cpu().clone().requires_grad_(True), "fix_scaleN": True}
    tr.inject = (ray_idx, noise)
    ld = tr.compute_loss(data, it=0, epoch=0, scheduling_start=0)
    ld["loss"].backward()
    full = _grads(tr)
    # the oracle's full-batch gradients (CPU restatement of training.py:214-416)
    cpu_data = {k: (v.cpu() if torch.is_tensor(v) else v) for k, v in data.items()}
    lo = orc.compute_loss_full(o_net, o_pose, o_dist, cpu_data, cfg["training"], cfg["rendering"], epoch=0,
                               scheduling_start=0, ray_idx=ray_idx, noise=noise)
    lo["loss"].backward()
    assert abs(float(ld["loss"]) - float(lo["loss"])) <= 1e-4 * abs(float(lo["loss"])) + 1e-6
    oracle = [p.grad for p in o_net.parameters()] + [o_pose["r"].grad, o_pose["t"].grad, o_dist["scales"].grad,
                                                     o_dist["shifts"].grad]
    assert len(oracle) == len(full)
    for i, (g0, g1, gf, go) in enumerate(zip(res[0][0], res[1][0], full, oracle)):
        assert (g0 is None) == (g1 is None) == (gf is None), i
        if gf is None:
            continue
        g0, g1, gf = torch.from_numpy(g0).double(), torch.from_numpy(g1).double(), torch.from_numpy(gf).double()
        assert torch.equal(g0, g1), i                       # every rank holds the same average
        # the per-rank GEMM reductions split the sample sum differently than one launch
        assert _nrel(g0, gf) < 2e-3, (i, _nrel(g0, gf))
        if go is None:                                      # e.g. the fixed last camera scale
            assert float(g0.abs().max()) == 0.0, i
            continue
        assert _nrel(g0, go) < 2e-3, (i, "vs oracle", _nrel(g0, go))
    for p0, p1 in zip(res[0][1], res[1][1]):                # replicated optimiser: identical parameters
        assert (p0 == p1).all()


# ---------------------------------------------------------------------------- config 4
FRAME = (188, 621, 362.5, 128, 256)     # H, W, fx, samples, hidden


def _frame_setup(dev):
    import model as mdl
    from tests.helpers import camera_K, make_cfg, rigid_c2w
    H, W, FX, S, D = FRAME
    cfg = make_cfg(hidden=D, S=S)
    torch.manual_seed(42)
    net = mdl.OfficialStaticNerf(cfg)
    rnd = mdl.Renderer(net, cfg["rendering"], device=dev)
    c2w = rigid_c2w(6, 0.2)
    K = camera_K(H, W, FX, FX).to(dev)
    w2c = torch.inverse(c2w).unsqueeze(0).to(dev)
    from model.common import arange_pixels
    pix = arange_pixels((H, W), 1, device=dev)[1]
    return rnd, net, pix, K, w2c, torch.eye(4).unsqueeze(0).to(dev), cfg


def _render_body(rank, world, q):
    from model import _hip
    from model.render_dist import render_image
    dev = torch.device("cuda:0")
    rnd, net, pix, K, w2c, sc, _ = _frame_setup(dev)
    assert net.hip_runner().use_fused_eval(FRAME[3])        # the north-star per-ray kernel renders the tiles
    assert _hip.gemm_get_precision() == 2                   # the library default
    rgb, depth = render_image(rnd, pix, K, w2c, sc)
    q.put((rank, rgb.cpu().numpy(), depth.cpu().numpy()))



def test_full_frame_render_sharded_under_process_group_is_bit_identical(dev):
    world = 2
    res = _spawn(_run_rank, world, "_render_body")
    from model.render_dist import render_image
    rnd, _, pix, K, w2c, sc, _ = _frame_setup(dev)
    rgb, depth = render_image(rnd, pix, K, w2c, sc)        # no process group: the whole frame in one call
    H, W = FRAME[:2]
    assert rgb.shape == (H * W, 3) and depth.shape == (H * W,)
    for r in range(world):
        assert torch.equal(torch.from_numpy(res[r][0]), rgb.cpu()), r
        assert torch.equal(torch.from_numpy(res[r][1]), depth.cpu()), r


def test_full_frame_render_matches_oracle_on_ray_subset(dev):
    """config 4 at its full size: one 188 x 621 frame (116 748 rays x 128 samples, D = 256)
    through render_image (the fused per-ray eval kernel, one launch), every ray finite, and a
    seeded 2048-ray subset elementwise within 1e-4 of the oracle's eval render of those rays
    (rays are independent, so the subset's oracle render is the frame's)."""
    from model.render_dist import render_image
    from oracle import nerf_oracle as orc
    from tests.helpers import assert_elementwise
    rnd, net, pix, K, w2c, sc, cfg = _frame_setup(dev)
    rgb, depth = render_image(rnd, pix, K, w2c, sc)
    H, W = FRAME[:2]
    assert rgb.shape == (H * W, 3) and depth.shape == (H * W,)
    assert bool(torch.isfinite(rgb).all()) and bool(torch.isfinite(depth).all())
    assert float(rgb.min()) >= 0.0 and float(rgb.max()) <= 1.0
    sub = torch.randperm(H * W, generator=torch.Generator().manual_seed(17))[:2048]
    ref = orc.OracleNerf(hidden_dim=FRAME[4])
    ref.load_state_dict({k: v.cpu() for k, v in net.state_dict().items()})
    with torch.no_grad():
        o = orc.render_nope_nerf(ref, pix[:, sub].cpu(), torch.ones(1, sub.numel(), 1), K.cpu(), w2c.cpu(), sc.cpu(),
                                 cfg["rendering"], noise=None, eval_=True)
    assert_elementwise(rgb[sub.to(dev)], o["rgb"].reshape(-1, 3), what="rgb (frame subset)")
    assert_elementwise(depth[sub.to(dev)], o["depth_pred"].reshape(-1), what="depth (frame subset)")

"""Benchmark: training rays/s of the NoPe-NeRF render path at 1024 rays x 128 samples.

Workload (BASELINE.json configs[1], config 2 of SURVEY.md section 8(d)): a V_KITTI-shaped
synthetic scene (188x621 image, fx = fy = 362.5, depth prior U[1,8] with ~5 % holes, a
fixed camera pose), hidden width 256, 1024 rays per GPU per step, 128 stratified samples
per ray.  One step = Trainer.train_step: ray sampling (randperm on device), ray
generation, fused HIP render forward, rgb-L2 + depth-L1 loss, fused HIP backward,
gradient all-reduce over RCCL (N > 1), Adam.  Inputs are resident in HBM.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (N > 1)

Rank 0 prints ONE JSON line.  Extra objects: "roofline" (the field-MLP GEMM family,
timed live with hipEvents around every GEMM launch of the timed steps), "cpu_baseline"
(the oracle CPU restatement of the same step on this host's cores, bounded sample) and
"alt_gemm" (the same workload with the other GEMM arithmetics).  The GEMMs compute f32
products on the exact-f32 MFMA (f32), as a 3-word bf16 split with six MFMA products
accumulated in f32 (bf16x6), or as a row-scaled 2-word fp16 split with three products
(f16x3, default; forward, input gradient and weight gradient).  All three are f32-accurate
(tests/test_gpu_kernels.py::test_split_accuracy); the exact-f32
number of the same run is "value_exact_f32".

Execution (--exec, default auto): on one GPU the K steps are timed twice -- enqueued eagerly
from Python, and as one captured hipGraph of the whole step replayed K times (new rays every
replay from the sampler's device step counter) -- and "value" is the faster; "execution",
"ms_per_step_eager" and "ms_per_step_graph" say which and give both.  Both are the full step
(nothing is cached or skipped); the graph only removes the host's ~1.9 ms (fast core) to
> 3 ms (slow core) of Python enqueue per step from the timed region, which on a slow host
is longer than the GPU's step.  N > 1 runs eager.

"roofline" names the GEMM kind with the most time per step (per_kind lists all of them)
and prices it against BOTH ceilings: its MFMA work at the dense MFMA rate of the
arithmetic that ran, and its algorithmic HBM bytes at 8 TB/s; "bound" is the ceiling
with the larger ideal time.  "roofline.dominant_kernel" prices the longest single in-step
kernel (the training forward chain) the same way, so that the figure stays comparable
across rounds whichever kind has the most time per step.

    python bench.py --gpus N     (N > 1 without WORLD_SIZE: spawns N ranks itself)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "training rays/sec at 1024 rays×128 samples; PSNR parity (±0.1 dB) vs ref"
H, W, FOCAL = 188, 621, 362.5
RAYS, SAMPLES, HIDDEN = 1024, 128, 256
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
BF16_MFMA_PEAK_TFLOPS = 2516.6  # 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz (v_mfma_f32_32x32x16_bf16, dense)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_cfg():
    from model.synthetic import make_cfg as mk
    cfg = mk(hidden=HIDDEN, S=SAMPLES)
    t = cfg["training"]
    t["n_training_points"] = RAYS
    t["pc_weight"] = [0.0, 0.0]        # config 2: pure render path (rgb l2 + depth l1)
    t["rgb_s_weight"] = [0.0, 0.0]
    return cfg


def synthetic_scene(dev, seed=0):
    """V_KITTI-shaped data dict (dataset.py:281-364 keys), resident on the GPU."""
    from model.synthetic import vkitti_scene
    return vkitti_scene(dev, seed, H, W, FOCAL)


def build_trainer(dev, c2w, cfg):
    import model as mdl
    from model.optim import HipAdam
    torch.manual_seed(42)                                   # train.py:23-24
    net = mdl.OfficialStaticNerf(cfg)
    renderer = mdl.Renderer(net, cfg["rendering"], device=dev)
    nn_model = mdl.get_model(renderer, cfg, device=dev)
    opt = HipAdam(nn_model.parameters(), lr=cfg["training"]["learning_rate"])
    pose = mdl.LearnPose(1, False, False, cfg, init_c2w=c2w.unsqueeze(0).to(dev)).to(dev)
    trainer = mdl.Trainer(nn_model, opt, cfg["training"], device=dev, pose_param_net=pose)
    return trainer, net


def algorithmic_gemm_flops(net, n_samples, split=False):
    """FP32 FLOPs of the field GEMMs one train step needs (reference shapes, no padding):
    forward and weight-gradient of every Linear, input-gradient of every Linear except
    the first and except the encoding columns (poses fixed).  split: (forward + input
    gradient, weight gradient) separately."""
    D = net.hidden_dim
    layers = [net.layers0[0], net.layers0[2], net.layers0[4], net.layers0[6], net.layers1[0], net.layers1[2],
              net.layers1[4], net.layers1[6], net.fc_feature, net.rgb_layers[0]]
    nt = tn = 0
    for i, lin in enumerate(layers):
        out_f, in_f = lin.weight.shape
        nt += 2 * n_samples * out_f * in_f               # forward
        tn += 2 * n_samples * out_f * in_f               # dW
        if i > 0:
            in_x = D if lin in (net.layers1[0], net.rgb_layers[0]) else in_f
            nt += 2 * n_samples * out_f * in_x           # dX
    return (nt, tn) if split else nt + tn


PRECISION = {"f32": 0, "bf16x6": 1, "f16x3": 2}
DEFAULT_GEMM = "f16x3"          # the library default (nerf_gemm_get_precision() == 2; tests/test_host_logic.py)
DTYPE = {"f32": "f32", "bf16x6": "f32 (bf16x6 emulation)", "f16x3": "f32 (f16x3 emulation)"}
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
KIND_NAMES = {
    "fwd": "forward NT (nerf_linear_fwd)",
    "dx": "input-gradient NT (nerf_linear_bwd_data)",
    "dw": "weight-gradient TN (f16x3 default: every layer's, as the two nerf_linear_bwd_weight_job_groups launches "
          "of TN schedule 3, each two block groups at half the splits -- [colour f, l_f, l7 | colour enc_d, l6, l5] "
          "and [l4 h3, l3, l0 | l4 enc_p, l2, l1]; other modes: the 256-output layers; algorithmic bytes: dy once "
          "per layer + x + dW, the split-K slabs excluded)",
    "dw_narrow": "narrow weight-gradient TN (l0 over enc_p; the colour layer over [f | enc_d] in one launch)",
    "chain_fwd": "training forward chain (nerf_mlp_chain_train: ten linears + heads, every output saved, one launch)",
    "chain_bwd": "input-gradient chain (nerf_mlp_chain_bwd: dyr + nine input gradients, every dy saved, one launch)",
}
KERNEL = {
    "f16x3": {"fwd": "k_gemm_nt_x6<128,256,2,2,0,true,true,2> (fp16 pair, 3 products)",
              "dx": "k_gemm_nt_x6<128,256,2,2,1,true,true,2> (fp16 pair, 3 products)",
              "dw": "k_wgrad_jobs<3> + k_wgrad_jobs<6> (a job list of 256x128 / 128x256 / 128x64 / 256x64 tiles "
                    "on 256 XCD-paired blocks, 4 MFMA + 4 load waves; fp16 pair, 3 products)",
              "dw_narrow": "k_wgrad_one<256,64> + k_wgrad_seg<128,256,1,64> (4 waves; fp16 pair, 3 products)",
              "chain_fwd": "k_mlp_chain_train2 (8 waves x 16 rows, 16x16x32 f16 MFMA; fp16 pair, 3 products)",
              "chain_bwd": "k_mlp_chain_bwd (8 waves x 16 rows, 16x16x32 f16 MFMA; fp16 pair, 3 products)"},
    "bf16x6": {"fwd": "k_gemm_nt_x6<256,256,2,2,0,true> (bf16x3 split, 6 products)",
               "dx": "k_gemm_nt_x6<256,256,2,2,1,true> (bf16x3 split, 6 products)",
               "dw": "k_gemm_tn_x6<256,128,4,2,false,1,2> (XCD-paired column tiles; bf16x3 split, 6 products)",
               "dw_narrow": "k_gemm_tn_x6<128,64|128,2,2,false> (bf16x3 split, 6 products)"},
    "f32": {"fwd": "k_gemm_nt<256,256,2,4,0> (f32 MFMA 32x32x2)", "dx": "k_gemm_nt<256,256,2,4,1> (f32 MFMA 32x32x2)",
            "dw": "k_gemm_tn<256,256,2,4> (f32 MFMA 32x32x2)",
            "dw_narrow": "k_gemm_tn<128,64|128,...> (f32 MFMA 32x32x2)"},
}


def kind_roofline(rec):
    """Both ceilings of one GEMM kind from its live hipEvent records (per-launch averages):
    MFMA -- the launches' MFMA work (f32 FLOPs x products per f32 product) at the dense
    MFMA rate of the arithmetic that ran; HBM -- their algorithmic bytes at 8 TB/s.  The
    binding ceiling is the one with the larger ideal time."""
    if rec["launches"] == 0 or rec["ms"] <= 0:
        return None
    n = rec["launches"]
    us = 1e3 * rec["ms"] / n
    peak_rate = FP32_MFMA_PEAK_TFLOPS if rec["exact_f32"] else BF16_MFMA_PEAK_TFLOPS
    t_mfma_us = rec["mfma_flops"] / n / (peak_rate * 1e12) * 1e6
    t_hbm_us = rec["bytes"] / n / (HBM_PEAK_GBS * 1e9) * 1e6
    products = rec["mfma_flops"] / rec["flops"] if rec["flops"] else 1.0
    return {"launches_per_step": None, "avg_launch_us": us,
            "gflop_per_launch": rec["flops"] / n / 1e9, "mbytes_per_launch": rec["bytes"] / n / 1e6,
            "products_per_f32_product": products,
            "mfma": {"achieved_tflops_f32eq": rec["flops"] / n / (us * 1e-6) / 1e12,
                     "peak_tflops_f32eq": peak_rate / products, "frac": t_mfma_us / us},
            "hbm": {"achieved_gbs": rec["bytes"] / n / (us * 1e-6) / 1e9, "peak_gbs": HBM_PEAK_GBS,
                    "frac": t_hbm_us / us},
            "binding": "hbm" if t_hbm_us >= t_mfma_us else "mfma"}


def lscpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(budget_s=20.0):
    """The oracle (CPU restatement of the reference step) on this host's cores."""
    from oracle import nerf_oracle as orc
    threads = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():      # the box's CPU share
        threads = min(threads, int(os.environ["OMP_NUM_THREADS"]))
    threads = max(1, threads)
    torch.set_num_threads(threads)
    torch.manual_seed(42)                                   # the GPU run's NeRF init (build_trainer)
    net = orc.OracleNerf(hidden_dim=HIDDEN)
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    data, c2w = synthetic_scene(torch.device("cpu"))        # the GPU run's scene
    g = torch.Generator().manual_seed(3)
    ray_idx = torch.randperm(H * W, generator=g)[:RAYS]
    noise = torch.rand(1, RAYS, SAMPLES, generator=g)

    def step():
        orc.train_step_render(net, opt, data["img"], data["img.depth"].unsqueeze(1), data["img.camera_mat"], c2w,
                              data["img.scale_mat"], ray_idx, noise, {"num_points": SAMPLES})

    step()                                                  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        step()
        n += 1
        el = time.perf_counter() - t0
        if el > budget_s or n >= 20:
            break
    return {"value": RAYS * n / el, "unit": "rays/s", "cores": threads, "kind": "port", "cpu_model": lscpu_model(),
            "sample": f"oracle train step (torch CPU fp32) on the GPU run's synthetic scene and NeRF init, "
                      f"{RAYS} rays x {SAMPLES} samples, D={HIDDEN}, one fixed ray draw and noise (seed 3), "
                      f"{n} timed steps after 1 warm-up ({el:.1f} s)"}


def render_frame_line(dev, frames=3, warmup=1):
    """The cfg4 workload beside the headline (1 GPU): one 188x621 frame x 128 samples through the
    reference caller's path (render_dist.render_image -> Renderer -> the fused per-ray eval
    kernel, samples + encodings + ten linears + heads + composite in one launch), with its MFMA
    roofline: 2 x 593 408 f32-equivalent FLOP per sample against the fp16-pair
    peak.  A few frames, ~0.2 s."""
    from model.common import arange_pixels
    from model.official_nerf import OfficialStaticNerf
    from model.render_dist import render_image
    from model.rendering import Renderer
    from model.synthetic import camera_K, make_cfg as pkg_cfg, rigid_c2w
    H, W = 188, 621
    cfg = pkg_cfg(hidden=HIDDEN, S=SAMPLES)
    torch.manual_seed(42)
    net = OfficialStaticNerf(cfg).to(dev)
    rnd = Renderer(net, cfg["rendering"], device=dev)
    K = camera_K(H, W, 362.5, 362.5).to(dev)
    w2c = torch.inverse(rigid_c2w(0)).unsqueeze(0).to(dev)
    scale = torch.eye(4, device=dev).unsqueeze(0)
    pix = arange_pixels((H, W), 1, device=dev)[1]
    for _ in range(warmup):
        render_image(rnd, pix, K, w2c, scale)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(frames):
        rgb, _ = render_image(rnd, pix, K, w2c, scale)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / frames
    if not bool(torch.isfinite(rgb).all()):
        raise RuntimeError("render: non-finite frame")
    flops = 2.0 * 593408 * H * W * SAMPLES
    peak = BF16_MFMA_PEAK_TFLOPS / 3
    ach = flops / el / 1e12
    return {"metric": "full-frame eval render rays/s (config 4: 188x621, 128 samples/ray, D=256)",
            "value": H * W / el, "unit": "rays/s", "ms_per_frame": 1e3 * el, "frames": frames,
            "kernel": "k_render_fused2 (nerf_render_eval_fused: samples, encodings, ten linears, heads, composite)",
            "roofline": {"bound": "mfma", "achieved": ach, "peak": peak, "unit": "TFLOP/s",
                         "frac": ach / peak, "flop_basis": "f32-equivalent (fp16-pair: 3 fp16 products per f32 product, peak = dense fp16 / 3)"}}


def cfg3_setup(dev, capturable=False):
    """Trainer with pose + distortion learning and the image-pair terms (config 3, reference
    training.py:214-416) on the two-view synthetic scene -> (trainer, [data view 0, view 1]).
    capturable: the pose / distortion Adams keep their step counts on the device (graphs)."""
    import model as mdl
    from model.optim import HipAdam
    from model.synthetic import make_cfg as pkg_cfg, vkitti_pair_scene
    cfg = pkg_cfg(hidden=HIDDEN, S=SAMPLES)
    t = cfg["training"]
    t["n_training_points"] = RAYS
    t["annealing_epochs"], t["scheduling_start"] = 2000, 0      # default.yaml:139: rgb l1 in the early epochs
    datas, c2w = vkitti_pair_scene(dev, H, W, FOCAL)
    torch.manual_seed(42)
    net = mdl.OfficialStaticNerf(cfg)
    renderer = mdl.Renderer(net, cfg["rendering"], device=dev)
    nn_model = mdl.get_model(renderer, cfg, device=dev)
    opt = HipAdam(nn_model.parameters(), lr=1e-3)
    pose = mdl.LearnPose(2, True, True, cfg, init_c2w=c2w.clone()).to(dev)
    distn = mdl.Learn_Distortion(2, True, True, cfg).to(dev)
    # train.py:100, :118; torch's fused Adam (the same update as the default multi-tensor
    # path, fewer launches), capturable in graphs
    opt_pose = torch.optim.Adam(pose.parameters(), lr=5e-4, capturable=capturable, fused=True)
    opt_dist = torch.optim.Adam(distn.parameters(), lr=5e-4, capturable=capturable, fused=True)
    tr = mdl.Trainer(nn_model, opt, t, device=dev, optimizer_pose=opt_pose, pose_param_net=pose,
                     optimizer_distortion=opt_dist, distortion_net=distn)
    return tr, datas


def cfg3_measure(dev, graph, steps, warmup):
    """The cfg3 step, eager or replaying one captured hipGraph per view (the two cameras
    alternate: both branches of training.py:329-358) -> dict: seconds for `steps` timed steps,
    median per-step GPU milliseconds (hipEvents at the step boundaries), median host enqueue
    milliseconds per step, last loss dict."""
    tr, datas = cfg3_setup(dev, capturable=graph)

    def one(i):
        return tr.train_step(datas[i % 2], it=i + 1, epoch=0, scheduling_start=0)

    if graph:
        tr.enable_graph_rng()                 # the ray draw keys on a device counter: new rays every replay
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for i in range(max(warmup, 2)):
                one(i)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        graphs, outs = [], []
        # a replay re-runs the captured step: iteration-dependent schedules (the loss annealing
        # of training.py) stay at the captured it, which is the eager run's first timed it
        for v in range(2):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                outs.append(tr.train_step(datas[v], it=warmup + 1 + v, epoch=0, scheduling_start=0))
            graphs.append(g)

        def one(i):  # noqa: F811
            graphs[i % 2].replay()
            return outs[i % 2]

    for i in range(warmup):
        one(i)
    torch.cuda.synchronize()
    host = []
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(steps):
        th = time.perf_counter()
        ld = one(warmup + i)
        host.append(time.perf_counter() - th)
        evs[i + 1].record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    gpu = statistics.median(evs[i].elapsed_time(evs[i + 1]) for i in range(steps))
    return {"s": el, "gpu_ms_median": gpu, "host_ms_median": 1e3 * statistics.median(host), "ld": ld}


def cfg3_line(dev, steps, warmup, modes=("eager", "graph")):
    """BASELINE configs[2] beside the headline: the full NoPe-NeRF step -- joint pose +
    depth-distortion learning, rgb + depth + point-cloud (chamfer, 7 285 points) + reprojection
    (rgb_s) losses, 188x621, 1024 rays x 128 samples, D = 256 -- eager and as graph replays,
    with the host enqueue time per step against the GPU time per step."""
    runs = {}
    for mode in modes:
        m = cfg3_measure(dev, mode == "graph", steps, warmup)
        ld = m["ld"]
        runs[mode] = {"value": RAYS * steps / m["s"], "ms_per_step": 1e3 * m["s"] / steps,
                      "gpu_ms_per_step_median": m["gpu_ms_median"],
                      # host time to enqueue one step: a replay enqueues one graph launch
                      "host_ms_per_step_median": m["host_ms_median"],
                      "host_over_gpu": m["host_ms_median"] / m["gpu_ms_median"],
                      "losses": {k: float(ld[k].detach()) for k in ("loss", "loss_rgb", "loss_depth", "loss_pc",
                                                                    "loss_rgb_s")}}
        if not all(math.isfinite(v) for v in runs[mode]["losses"].values()):
            raise RuntimeError(f"cfg3 {mode}: non-finite loss {runs[mode]['losses']}")
    best = max(runs, key=lambda k: runs[k]["value"])
    r = runs[best]
    return {"metric": "full NoPe-NeRF training rays/sec (config 3: pose + distortion + pc + rgb_s losses)",
            "value": r["value"], "unit": "rays/s", "ms_per_step": r["ms_per_step"], "steps": steps,
            "warmup": warmup, "execution": {"eager": "eager", "graph": "graph replay"}[best],
            "data": "synthetic two-view V_KITTI-shaped scene (model.synthetic.vkitti_pair_scene)",
            "config": {"workload": "config 3: 188x621, 1024 rays x 128 samples, D=256, pose + distortion learned, "
                                   "pc chamfer 7285 points, rgb_s reprojection, cameras alternating",
                       "graph_note": "graph replays keep iteration-dependent schedules at the captured it "
                                     "(warmup + 1, + 2 per camera); eager advances it every step"},
            "runs": runs}


def rank_attribution(world, steps, el_s, allreduce_ms, dev):
    """N > 1: what each rank spent of the K timed steps, gathered from every rank -- the
    all-reduce milliseconds (hipEvents around dist.all_reduce in Trainer.allreduce_grads,
    training.py; they include the wait for the slowest rank), the rest of the step
    ("compute"), and each rank's own rays/s -- so a scaling shortfall splits into
    communication and compute spread."""
    t = torch.tensor([el_s, allreduce_ms], dtype=torch.float64, device=dev)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    per = [(float(x[0]), float(x[1])) for x in parts]
    ar = [a / steps for _, a in per]
    comp = [(1e3 * s - a) / steps for s, a in per]
    rps = [RAYS * steps / s for s, _ in per]
    return {"world_size": world, "allreduce_ms_per_step": max(ar), "allreduce_ms_per_step_min": min(ar),
            "compute_ms_per_step_max": max(comp), "compute_ms_per_step_min": min(comp),
            "rays_per_s_per_rank_min": min(rps), "rays_per_s_per_rank_max": max(rps),
            "per_rank": [{"rank": i, "ms_per_step": 1e3 * s / steps, "allreduce_ms_per_step": a / steps}
                         for i, (s, a) in enumerate(per)]}


def spawn_ranks(n, argv, script=None):
    """--gpus N > 1 without a launcher: run this script under torch.distributed.run as a
    CHILD process (N ranks, one per GPU, rendezvous on 127.0.0.1) and return its exit
    code.  Called before anything touches the GPU; the parent never initialises HIP."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")       # dmabuf IPC only on this driver
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", script or os.path.abspath(__file__)] + list(argv)
    log(f"bench: launching {n} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd, env=env)


def init_ranks(args):
    """(world, rank, local, device) from the launcher's env; refuses a --gpus that
    disagrees with WORLD_SIZE."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank per GPU")
    if args.plumbing:
        if world > 1:
            dist.init_process_group("gloo")
        return world, rank, local, torch.device("cpu")
    if world > 1 and os.environ.get("NERF_BENCH_SHARED_GPU") == "1":
        # rehearsal of the N-rank measurement path on a one-GPU box: every rank on cuda:0, the
        # collectives on gloo (RCCL refuses two ranks on one GPU); its numbers are not a
        # measurement (the ranks share the GPU) and the line says so
        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
        return world, rank, 0, torch.device("cuda", 0)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local, torch.device("cuda", local)


def plumbing(args, world, rank):
    """CPU check of the multi-rank path (gloo): the launcher, the rank env and the
    Trainer's fixed-layout gradient all-reduce on the real model / pose / distortion
    parameter set, with rank 1 missing a gradient.  Prints a JSON line that says it is
    a plumbing check, not a measurement."""
    import model as mdl
    cfg = make_cfg()
    torch.manual_seed(0)
    net = mdl.OfficialStaticNerf(cfg)
    pose = mdl.LearnPose(2, True, True, cfg)
    dist_net = mdl.Learn_Distortion(2, True, True, cfg)
    tr = mdl.Trainer(net, None, cfg["training"], device=torch.device("cpu"), pose_param_net=pose,
                     distortion_net=dist_net)
    params = tr.bucket_params()
    steps = max(1, args.steps if args.steps < 30 else 3)
    tr.time_collectives(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        for i, p in enumerate(params):
            p.grad = None if (rank == 1 and i == 0) else torch.full_like(p, float(rank + 1 + i))
        if world > 1:
            tr.allreduce_grads()
    el = time.perf_counter() - t0
    for i, p in enumerate(params):
        ranks_with = [r for r in range(world) if not (r == 1 and i == 0)]
        want = sum(r + 1 + i for r in ranks_with) / world
        if p.grad is None or not torch.allclose(p.grad, torch.full_like(p, want)):
            raise RuntimeError(f"plumbing: parameter {i} not averaged over the ranks")
    att = rank_attribution(world, steps, el, tr.collective_ms(), torch.device("cpu")) if world > 1 else None
    if world > 1:
        dist.barrier()
    if rank == 0:
        out = {"plumbing": True, "n_gpus": world, "world_size": dist.get_world_size() if world > 1 else 1,
               "steps": steps, "bucket_params": len(params), "bucket_elems": sum(p.numel() for p in params),
               "allreduce_s": el, "data": "CPU gloo plumbing check of the launcher and gradient all-reduce; "
                                          "not a measurement"}
        if att is not None:
            out["allreduce_ms_per_step"] = att["allreduce_ms_per_step"]
            out["multi_gpu"] = att
        print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--gemm-precision", choices=list(PRECISION), default=DEFAULT_GEMM,
                    help="GEMM arithmetic: f32 emulated by a row-scaled 2-word fp16 split (f16x3, default), by a "
                         "3-word bf16 split (bf16x6), or the exact-f32 MFMA (f32); all f32-accurate")
    ap.add_argument("--exec", dest="exec_mode", choices=["auto", "eager", "graph"], default="auto",
                    help="auto (1 GPU): time the step eager AND as one replayed hipGraph, report the faster; "
                         "N > 1 runs eager (RCCL capture is not exercised on this pool)")
    ap.add_argument("--no-alt", dest="alt", action="store_false",
                    help="skip timing the other GEMM arithmetics (reported as alt_gemm)")
    ap.add_argument("--no-cfg3", dest="cfg3", action="store_false",
                    help="skip the config-3 line (full NoPe-NeRF step, eager and graph; 1 GPU)")
    ap.add_argument("--cfg3-steps", type=int, default=20)
    ap.add_argument("--plumbing", action="store_true",
                    help="CPU gloo check of the rank launcher + gradient all-reduce (tests), no GPU")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world, rank, local, dev = init_ranks(args)
    if args.plumbing:
        plumbing(args, world, rank)
        if world > 1:
            dist.destroy_process_group()
        return
    world = dist.get_world_size() if world > 1 else 1
    from model import _hip
    _hip.load_library()

    cfg = make_cfg()
    data, c2w = synthetic_scene(dev)
    medians = {}      # median per-step milliseconds (hipEvents at the step boundaries) per timed pass
    attributions = {}  # N > 1: per-rank all-reduce / compute split of the timed pass (rank_attribution)

    def measure(precision, with_hooks=True):
        """W warm-up + K timed train steps with the GEMMs in `precision` (0 exact-f32 MFMA,
        1 split-bf16, 2 fp16 pair); returns (max-over-ranks seconds, last loss dict, GEMM
        hook stats, per-kind records, net, seconds of the instrumented pass)."""
        _hip.gemm_set_precision(precision)
        trainer, net = build_trainer(dev, c2w, cfg)
        torch.cuda.manual_seed(1000 + rank)                 # each rank samples its own rays

        def one(it):
            return trainer.train_step(data, it=it, epoch=0, scheduling_start=0)

        def timed(it0, hooks):
            """K steps between barrier + synchronize; hooks: hipEvent pairs around every GEMM
            launch (they serialise neighbouring launches a little, so `value` is timed without
            them and the roofline in a second, instrumented pass of the same K steps)."""
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            _hip.prof_enable(hooks)
            trainer.time_collectives(world > 1 and not hooks)   # hipEvents around the all-reduce
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
            t0 = time.perf_counter()
            evs[0].record()
            for i in range(args.steps):
                ld = one(it0 + i)
                evs[i + 1].record()           # step boundaries on the launch stream (no host sync)
            torch.cuda.synchronize()
            t_local = time.perf_counter() - t0       # this rank's own time, before the barrier
            if world > 1:
                dist.barrier()
            t1 = time.perf_counter()
            kinds = _hip.prof_read_kinds() if hooks else None
            stats = _hip.prof_read() if hooks else None
            _hip.prof_enable(False)
            el = t1 - t0
            med = statistics.median(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps))
            if world > 1 and not hooks:
                timed.attribution = rank_attribution(world, args.steps, t_local, trainer.collective_ms(), dev)
            trainer.time_collectives(False)
            if world > 1:
                t = torch.tensor([el, med], device=dev, dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                el, med = t[0].item(), t[1].item()
            timed.median_ms = med
            return el, ld, stats, kinds

        for i in range(args.warmup):
            one(i)
        timed.attribution = None
        el, ld, _, _ = timed(args.warmup, False)
        medians[precision] = timed.median_ms
        attributions[precision] = timed.attribution
        if with_hooks:
            el_h, _, stats, kinds = timed(args.warmup + args.steps, True)
        else:
            el_h = stats = kinds = None
        return el, ld, stats, kinds, net, el_h

    def measure_graph(precision):
        """The same K steps as ONE captured hipGraph replayed (1 GPU): the ray sampler keys on a
        device step counter (Trainer.enable_graph_rng), so every replay trains on new rays, and
        the whole step -- sampling, render fwd + bwd, loss, Adam -- is in the graph.  The step's
        host enqueue (~1.9 ms on a fast host core, > 3 ms on a slow one) drops out of the timed
        region.  Returns (seconds for K replays, loss dict) or None if capture is not possible."""
        _hip.gemm_set_precision(precision)
        trainer, _ = build_trainer(dev, c2w, cfg)
        trainer.enable_graph_rng()
        step = lambda i: trainer.train_step(data, it=i, epoch=0, scheduling_start=0)  # noqa: E731
        try:
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                for i in range(3):
                    step(i)
            torch.cuda.current_stream(dev).wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                out = step(0)
        except RuntimeError as exc:    # capture unsupported here: eager only
            log(f"graph capture failed ({exc}); eager timing only")
            return None
        for _ in range(args.warmup):
            g.replay()
        torch.cuda.synchronize()
        # the timed K replays carry no per-replay events (an event behind every replay cost
        # ~0.02 ms per step: profiles/r06/graph_timing_probe.json); the per-replay median comes
        # from a second, untimed pass
        t0 = time.perf_counter()
        for i in range(args.steps):
            g.replay()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        evs[0].record()
        for i in range(args.steps):
            g.replay()
            evs[i + 1].record()
        torch.cuda.synchronize()
        medians["graph"] = statistics.median(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps))
        if not math.isfinite(out["loss"].detach().item()):
            raise RuntimeError("graph replay: non-finite loss")
        return el, out

    main_prec = PRECISION[args.gemm_precision]
    elapsed, ld, (gemm_ms, gemm_launches, _, gemm_union_ms), kinds, net, elapsed_hooks = measure(main_prec)
    elapsed_eager = elapsed
    graph = None
    if world == 1 and args.exec_mode in ("auto", "graph"):
        graph = measure_graph(main_prec)
        if graph is not None and (args.exec_mode == "graph" or graph[0] < elapsed):
            elapsed, ld = graph
    execution = "graph replay" if (graph is not None and elapsed == graph[0]) else "eager"
    if args.exec_mode == "graph" and execution != "graph replay":
        raise RuntimeError("--exec graph: capture failed")
    alt = None
    if args.alt:
        # the other GEMM arithmetics on the same workload, reported beside the headline
        alt = []
        for name, prec in PRECISION.items():
            if prec == main_prec:
                continue
            el2, ld2, _, _, _, _ = measure(prec, with_hooks=False)
            alt.append({"gemm_arithmetic": name, "dtype": DTYPE[name], "value": world * RAYS / (el2 / args.steps),
                        "ms_per_step": 1e3 * el2 / args.steps, "final_loss": ld2["loss"].detach().item()})
        _hip.gemm_set_precision(main_prec)
    loss = ld["loss"].detach().item()
    psnr = -10.0 * math.log10(max(ld["l2_mean"].detach().item(), 1e-10))
    if not math.isfinite(loss):
        raise RuntimeError(f"non-finite loss {loss}")

    if rank == 0:
        ms = 1e3 * elapsed / args.steps
        # per-kind rooflines (MFMA and HBM ceilings, per-launch averages of the live records)
        per_kind = {}
        for k, rec in kinds.items():
            r = kind_roofline(rec)
            if r is not None:
                r["launches_per_step"] = rec["launches"] / args.steps
                r["ms_per_step"] = rec["ms"] / args.steps
                r["what"] = KIND_NAMES[k]
                r["kernel"] = KERNEL[args.gemm_precision][k]
                per_kind[k] = r
        dom = max(per_kind, key=lambda k: per_kind[k]["ms_per_step"])
        d = per_kind[dom]
        bound = d["binding"]
        ach, peak, unit = ((d["hbm"]["achieved_gbs"], HBM_PEAK_GBS, "GB/s") if bound == "hbm" else
                           (d["mfma"]["achieved_tflops_f32eq"], d["mfma"]["peak_tflops_f32eq"], "TFLOP/s"))
        tpath = next((q for q in (os.path.join(ROOT, "profiles", r, "gemm_traffic.json")
                                  for r in ("r06", "r05", "r04")) if os.path.exists(q)), "")
        tkinds = json.load(open(tpath)).get("kinds", {}) if tpath and args.gemm_precision == "f16x3" else {}

        def kind_traffic(k):
            # HBM bytes per launch of kind k from the committed rocprofv3 PMC passes (FETCH_SIZE x2 +
            # WRITE_SIZE, the guide's gfx950 correction): the mean over the kind's launches, as
            # per_kind's algorithmic bytes are
            kd = tkinds.get(k)
            if not kd:
                return None, None
            return kd["bytes_per_launch"], (
                f"{os.path.relpath(tpath, ROOT)}: mean over {kd['launches_profiled']} profiled launches of the "
                f"kind's kernels ({kd['read_bytes_per_launch'] / 1e6:.1f} MB read, "
                f"{kd['write_bytes_per_launch'] / 1e6:.1f} MB written per launch)")

        traffic, traffic_note = kind_traffic(dom)
        # the longest single in-step kernel (the training forward chain since round 4), priced
        # against its own binding ceiling: comparable across rounds whichever kind has the most
        # time per step
        dk = max(per_kind, key=lambda k: per_kind[k]["avg_launch_us"])
        dkr = per_kind[dk]
        dk_hbm = dkr["binding"] == "hbm"
        dk_traffic, dk_note = kind_traffic(dk)
        dominant = {"kind": dk, "kernel": dkr["kernel"], "bound": dkr["binding"],
                    "avg_launch_us": dkr["avg_launch_us"],
                    "achieved": dkr["hbm"]["achieved_gbs"] if dk_hbm else dkr["mfma"]["achieved_tflops_f32eq"],
                    "peak": HBM_PEAK_GBS if dk_hbm else dkr["mfma"]["peak_tflops_f32eq"],
                    "unit": "GB/s" if dk_hbm else "TFLOP/s",
                    "frac": dkr["hbm"]["frac"] if dk_hbm else dkr["mfma"]["frac"],
                    "algorithmic_mbytes_per_launch": dkr["mbytes_per_launch"],
                    "gflop_per_launch": dkr["gflop_per_launch"],
                    "traffic": dk_traffic, "traffic_note": dk_note}
        nt_fl, tn_fl = algorithmic_gemm_flops(net, RAYS * SAMPLES, split=True)
        fam_ms = sum(rec["ms"] for rec in kinds.values())
        fam_mfma = sum(rec["mfma_flops"] for rec in kinds.values())
        roof = {"bound": bound, "kernel": d["kernel"], "what": d["what"],
                "achieved": ach, "peak": peak, "unit": unit, "frac": ach / peak, "traffic": traffic,
                "flop_basis": ("f32-equivalent: algorithmic f32 products; the fp16-pair kernels issue 3 fp16 MFMA "
                               "products per f32 product, so the peak is the dense fp16 MFMA peak / 3"
                               if bound == "mfma" else None),
                "traffic_note": traffic_note,
                "other_ceiling": ({"mfma_frac": d["mfma"]["frac"], "mfma_achieved_tflops_f32eq":
                                   d["mfma"]["achieved_tflops_f32eq"], "mfma_peak_tflops_f32eq":
                                   d["mfma"]["peak_tflops_f32eq"]} if bound == "hbm" else
                                  {"hbm_frac": d["hbm"]["frac"], "hbm_achieved_gbs": d["hbm"]["achieved_gbs"]}),
                "dominant_kernel": dominant,
                "per_kind": per_kind,
                "family": {"gemm_ms_per_step": gemm_ms / args.steps, "union_ms_per_step": gemm_union_ms / args.steps,
                           "launches_per_step": gemm_launches / args.steps,
                           "algorithmic_gflop_per_step": (nt_fl + tn_fl) / 1e9,
                           "mfma_frac_per_launch": (fam_mfma / (BF16_MFMA_PEAK_TFLOPS * 1e12 if
                                                                args.gemm_precision != "f32" else
                                                                FP32_MFMA_PEAK_TFLOPS * 1e12)) / (fam_ms * 1e-3)},
                "timing": "per-kind hipEvent pairs around every GEMM launch on its own stream, second timed "
                          "pass of the same K steps (ms_per_step of that pass: %.3f)" % (1e3 * elapsed_hooks /
                                                                                          args.steps)}
        render = render_frame_line(dev) if world == 1 and args.gemm_precision == "f16x3" else None
        full = None
        if world == 1 and args.cfg3:
            log("timing config 3 (the full NoPe-NeRF step) ...")
            full = cfg3_line(dev, args.cfg3_steps, 3)
            _hip.gemm_set_precision(main_prec)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            log("timing the CPU baseline (oracle) ...")
            cpu = cpu_baseline(args.cpu_budget)
        exact = next((a for a in (alt or []) if a["gemm_arithmetic"] == "f32"), None)
        out = {"metric": METRIC, "value": world * RAYS / (elapsed / args.steps), "unit": "rays/s",
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
               "execution": execution,
               "ms_per_step_median": medians["graph" if execution == "graph replay" else main_prec],
               "ms_per_step_eager": 1e3 * elapsed_eager / args.steps,
               "ms_per_step_graph": 1e3 * graph[0] / args.steps if graph is not None else None,
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
               "dtype": DTYPE[args.gemm_precision], "gemm_arithmetic": args.gemm_precision,
               "value_exact_f32": exact["value"] if exact else None,
               "ms_per_step_exact_f32": exact["ms_per_step"] if exact else None,
               "data": "synthetic (V_KITTI-shaped scene, random-init NeRF D=256; no dataset offline)",
               "config": {"workload": "config 2: V_KITTI scene-1 shape 188x621, 1024 rays x 128 samples per GPU, "
                                      "poses fixed, full train_step (render fwd+bwd, rgb-l2+depth-l1, Adam)",
                          "global_batch": world * RAYS, "seq_len": SAMPLES, "hidden_dim": HIDDEN,
                          "parallelism": f"dp{world}"},
               "final_loss": loss, "train_psnr_last_step": psnr,
               "roofline": roof, "cpu_baseline": cpu, "alt_gemm": alt, "render_cfg4": render, "full_cfg3": full}
        if os.environ.get("NERF_BENCH_SHARED_GPU") == "1" and world > 1:
            out["rehearsal"] = ("NERF_BENCH_SHARED_GPU: every rank on one GPU over gloo -- a check of the "
                                "N-rank path, not a measurement")
        att = attributions.get(main_prec)
        if att is not None:
            out["world_size"] = world
            out["allreduce_ms_per_step"] = att["allreduce_ms_per_step"]
            out["multi_gpu"] = att
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

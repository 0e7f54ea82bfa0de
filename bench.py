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
accumulated in f32 (bf16x6), or -- forward and backward-data GEMMs -- as a row-scaled
2-word fp16 split with three products (f16x3; its weight gradients as bf16x6).  All three
are f32-accurate (tests/test_gpu_kernels.py::test_split_accuracy).
"""
from __future__ import annotations

import argparse
import json
import math
import os
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
    from tests.helpers import make_cfg as mk
    cfg = mk(hidden=HIDDEN, S=SAMPLES)
    t = cfg["training"]
    t["n_training_points"] = RAYS
    t["pc_weight"] = [0.0, 0.0]        # config 2: pure render path (rgb l2 + depth l1)
    t["rgb_s_weight"] = [0.0, 0.0]
    return cfg


def synthetic_scene(dev, seed=0):
    """V_KITTI-shaped data dict (dataset.py:281-364 keys), resident on the GPU."""
    from tests.helpers import camera_K, rigid_c2w
    g = torch.Generator().manual_seed(seed)
    yy, xx = torch.meshgrid(torch.linspace(0, 1, H), torch.linspace(0, 1, W), indexing="ij")
    img = torch.stack([0.5 + 0.4 * torch.sin(6 * xx + 2 * yy), 0.5 + 0.4 * torch.cos(5 * yy),
                       0.3 + 0.3 * xx * yy], 0).unsqueeze(0)
    img = (img + 0.02 * torch.rand(img.shape, generator=g)).clamp(0, 1)
    depth = 1.0 + 7.0 * torch.rand(1, H, W, generator=g)
    holes = torch.rand(1, H, W, generator=g) < 0.05
    depth[holes] = 0.0
    c2w = rigid_c2w(seed)
    data = {"img": img, "img.idx": torch.tensor([0]), "img.depth": depth, "img.depth_mask": ~holes,
            "img.camera_mat": camera_K(H, W, FOCAL, FOCAL), "img.scale_mat": torch.eye(4).unsqueeze(0),
            "img.pose_gt": c2w.unsqueeze(0)}
    for k, v in list(data.items()):
        if k not in ("img.idx", "img.depth_mask"):
            data[k] = v.to(dev)
    return data, c2w


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


def gemm_peak(mode, nt_flops, tn_flops):
    """f32-equivalent MFMA peak of the GEMM family in arithmetic `mode`: the dense MFMA rate
    divided by the products per f32 product (f32: 1 on the f32 MFMA; bf16x6: 6; f16x3: 3 for
    forward / input gradient, 6 for the weight gradients), weighted by the FLOPs each runs."""
    if mode == "f32":
        return FP32_MFMA_PEAK_TFLOPS
    if mode == "bf16x6":
        return BF16_MFMA_PEAK_TFLOPS / 6
    t = nt_flops / (BF16_MFMA_PEAK_TFLOPS / 3) + tn_flops / (BF16_MFMA_PEAK_TFLOPS / 6)
    return (nt_flops + tn_flops) / t


def cpu_baseline(budget_s=20.0):
    """The oracle (CPU restatement of the reference step) on this host's cores."""
    from oracle import nerf_oracle as orc
    from tests.helpers import synthetic_rays
    threads = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():      # the box's CPU share
        threads = min(threads, int(os.environ["OMP_NUM_THREADS"]))
    threads = max(1, threads)
    torch.set_num_threads(threads)
    torch.manual_seed(42)
    net = orc.OracleNerf(hidden_dim=HIDDEN)
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    b = synthetic_rays(R=RAYS, S=SAMPLES, seed=3)
    img = torch.rand(1, 3, H, W)
    depth_img = 1.0 + 7.0 * torch.rand(1, 1, H, W)
    ray_idx = torch.randperm(H * W)[:RAYS]

    def step():
        orc.train_step_render(net, opt, img, depth_img, b["K"], b["c2w"], b["scale"], ray_idx,
                              b["noise"], {"num_points": SAMPLES})

    step()                                                  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        step()
        n += 1
        el = time.perf_counter() - t0
        if el > budget_s or n >= 20:
            break
    return {"value": RAYS * n / el, "unit": "rays/s", "cores": threads, "kind": "port",
            "sample": f"oracle train step (torch CPU fp32), {RAYS} rays x {SAMPLES} samples, D={HIDDEN}, "
                      f"{n} timed steps after 1 warm-up ({el:.1f} s)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--gemm-precision", choices=list(PRECISION), default="f16x3",
                    help="GEMM arithmetic: f32 emulated by a row-scaled 2-word fp16 split (f16x3, default), by a "
                         "3-word bf16 split (bf16x6), or the exact-f32 MFMA (f32); all f32-accurate")
    ap.add_argument("--no-alt", dest="alt", action="store_false",
                    help="skip timing the other GEMM arithmetics (reported as alt_gemm)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    from model import _hip
    _hip.load_library()

    cfg = make_cfg()
    data, c2w = synthetic_scene(dev)

    def measure(precision, with_hooks=True):
        """W warm-up + K timed train steps with the GEMMs in `precision` (0 exact-f32 MFMA,
        1 split-bf16, 2 fp16 pair); returns (max-over-ranks seconds, last loss dict, GEMM hook stats)."""
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
            t0 = time.perf_counter()
            for i in range(args.steps):
                ld = one(it0 + i)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            t1 = time.perf_counter()
            stats = _hip.prof_read() if hooks else None
            _hip.prof_enable(False)
            el = t1 - t0
            if world > 1:
                t = torch.tensor([el], device=dev, dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                el = t.item()
            return el, ld, stats

        for i in range(args.warmup):
            one(i)
        el, ld, _ = timed(args.warmup, False)
        el_h, _, stats = timed(args.warmup + args.steps, True) if with_hooks else (None, None, None)
        return el, ld, stats, net, el_h

    main_prec = PRECISION[args.gemm_precision]
    elapsed, ld, (gemm_ms, gemm_launches, _, gemm_union_ms), net, elapsed_hooks = measure(main_prec)
    alt = None
    if args.alt:
        # the other GEMM arithmetics on the same workload, reported beside the headline
        alt = []
        for name, prec in PRECISION.items():
            if prec == main_prec:
                continue
            el2, ld2, _, _, _ = measure(prec, with_hooks=False)
            alt.append({"gemm_arithmetic": name, "value": world * RAYS / (el2 / args.steps),
                        "ms_per_step": 1e3 * el2 / args.steps, "final_loss": ld2["loss"].detach().item()})
        _hip.gemm_set_precision(main_prec)
    loss = ld["loss"].detach().item()
    psnr = -10.0 * math.log10(max(ld["l2_mean"].detach().item(), 1e-10))
    if not math.isfinite(loss):
        raise RuntimeError(f"non-finite loss {loss}")

    if rank == 0:
        ms = 1e3 * elapsed / args.steps
        nt_fl, tn_fl = algorithmic_gemm_flops(net, RAYS * SAMPLES, split=True)
        alg = (nt_fl + tn_fl) * args.steps
        achieved = alg / (gemm_ms * 1e-3) / 1e12 if gemm_ms > 0 else None
        # achieved: algorithmic FLOPs / summed per-launch durations (the contract's per-launch
        # average).  The dW GEMMs run on a side stream concurrently with the dX chain, which
        # stretches each launch; achieved_union divides by the union of the launch intervals.
        achieved_union = alg / (gemm_union_ms * 1e-3) / 1e12 if gemm_union_ms > 0 else None
        peak = gemm_peak(args.gemm_precision, nt_fl, tn_fl)
        kname = {"bf16x6": "k_gemm_nt_x6/k_gemm_tn_x6 (f32 as 3xbf16, 6 products on MFMA 32x32x16 bf16, field MLP)",
                 "f16x3": "k_gemm_nt_x6<H> (f32 as row-scaled 2xfp16, 3 products on MFMA 32x32x16 f16; fwd + dX) / "
                          "k_gemm_tn_x6 (bf16x6; dW), field MLP",
                 "f32": "k_gemm_nt/k_gemm_tn (FP32 MFMA 32x32x2, field MLP)"}[args.gemm_precision]
        traffic, traffic_note = None, None
        tpath = os.path.join(ROOT, "profiles", "r01", "gemm_traffic.json")
        # template arguments of the 256x256-tile forward launch per arithmetic (older summaries
        # predate the trailing fp16-pair flag)
        fwd_tags = {"bf16x6": ("<256, 256, 2, 2, 0, true>", "<256, 256, 2, 2, 0, true, false"),
                    "f16x3": ("<128, 256, 2, 2, 0, true, true, 2>",)}.get(args.gemm_precision, ())
        if fwd_tags and os.path.exists(tpath):
            # HBM bytes of one 256x256-tile forward launch (131072 x 256 x 256, mask out) from
            # the committed rocprofv3 PMC passes (FETCH_SIZE x2 + WRITE_SIZE); algorithmic:
            # x 134.2 MB + y 134.2 MB + ReLU bits 4.2 MB + weight image 0.4 MB = 273 MB
            t = json.load(open(tpath))
            fwd = [x for x in t["launches"] if any(tag in x["kernel"] for tag in fwd_tags)]
            if fwd:
                traffic = fwd[0]["bytes"]
                traffic_note = (f"{fwd[0]['kernel'].split('(')[0]} forward 131072x256x256, one launch, bytes from "
                                "profiles/r01/gemm_traffic.json (algorithmic 2.73e8)")
        roof = {"bound": "mfma", "kernel": kname,
                "achieved": achieved, "peak": peak, "unit": "TFLOP/s (f32-equivalent)",
                "frac": (achieved / peak) if achieved else None, "traffic": traffic, "traffic_note": traffic_note,
                "achieved_union": achieved_union,
                "frac_union": (achieved_union / peak) if achieved_union else None,
                "algorithmic_gflop_per_step": alg / args.steps / 1e9,
                "launches_per_step": gemm_launches / args.steps,
                "avg_launch_us": 1e3 * gemm_ms / max(1, gemm_launches),
                "gemm_ms_per_step": gemm_ms / args.steps,
                "timing": "second timed pass of the same K steps with hipEvent pairs around every GEMM launch "
                          "(ms_per_step of that pass: %.3f)" % (1e3 * elapsed_hooks / args.steps),
                "gemm_union_ms_per_step": gemm_union_ms / args.steps}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            log("timing the CPU baseline (oracle) ...")
            cpu = cpu_baseline(args.cpu_budget)
        out = {"metric": METRIC, "value": world * RAYS / (elapsed / args.steps), "unit": "rays/s",
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
               "gemm_arithmetic": args.gemm_precision,
               "data": "synthetic (V_KITTI-shaped scene, random-init NeRF D=256; no dataset offline)",
               "config": {"workload": "config 2: V_KITTI scene-1 shape 188x621, 1024 rays x 128 samples per GPU, "
                                      "poses fixed, full train_step (render fwd+bwd, rgb-l2+depth-l1, Adam)",
                          "global_batch": world * RAYS, "seq_len": SAMPLES, "hidden_dim": HIDDEN,
                          "parallelism": f"dp{world}"},
               "final_loss": loss, "train_psnr_last_step": psnr,
               "roofline": roof, "cpu_baseline": cpu, "alt_gemm": alt}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

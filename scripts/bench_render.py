"""Full-frame eval render throughput.

188x621 = 116 748 rays x 128 samples per frame, eval mode (no noise, z-depth), D=256
random-init field, the frame sharded in contiguous ray tiles over the ranks and
assembled by one RCCL all-gather (model/render_dist.py).  Prints one JSON line:
rays/s (whole job), frames/s, ms per frame.

    python scripts/bench_render.py [--frames K --warmup W]
    python scripts/bench_render.py --gpus N      (spawns N ranks, one per GPU)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

H, W, FOCAL, S, HIDDEN = 188, 621, 362.5, 128, 256


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--gemm-precision", choices=["f32", "bf16x6", "f16x3"], default="f16x3")
    ap.add_argument("--gpus", type=int, default=1)
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        from bench import spawn_ranks        # N ranks as a child torch.distributed.run
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:], script=os.path.abspath(__file__)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench_render: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    from model import _hip
    from model.official_nerf import OfficialStaticNerf
    from model.render_dist import render_image
    from model.rendering import Renderer
    from model.common import arange_pixels
    from model.synthetic import camera_K, make_cfg, rigid_c2w
    _hip.load_library()
    _hip.gemm_set_precision({"f32": 0, "bf16x6": 1, "f16x3": 2}[args.gemm_precision])
    cfg = make_cfg(hidden=HIDDEN, S=S)
    torch.manual_seed(42)
    net = OfficialStaticNerf(cfg).to(dev)
    rnd = Renderer(net, cfg["rendering"], device=dev)
    K = camera_K(H, W, FOCAL, FOCAL).to(dev)
    w2c = torch.inverse(rigid_c2w(0)).unsqueeze(0).to(dev)
    scale = torch.eye(4, device=dev).unsqueeze(0)
    pix = arange_pixels((H, W), 1, device=dev)[1]
    for _ in range(args.warmup):
        render_image(rnd, pix, K, w2c, scale)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.frames):
        rgb, depth = render_image(rnd, pix, K, w2c, scale)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    if not torch.isfinite(rgb).all():
        raise RuntimeError("non-finite render")
    if rank == 0:
        n = H * W
        print(json.dumps({"metric": "full-frame eval render rays/s (188x621, 128 samples/ray, D=256)",
                          "value": args.frames * n / el, "unit": "rays/s", "n_gpus": dist.get_world_size() if world > 1 else 1,
                          "frames": args.frames, "warmup": args.warmup, "ms_per_frame": 1e3 * el / args.frames,
                          "frames_per_s": args.frames / el, "higher_is_better": True, "scaling": "strong",
                          "dtype": "f32", "gemm_arithmetic": args.gemm_precision, "data": "synthetic",
                          "config": {"workload": "config 4: eval render of one 188x621 frame, contiguous ray "
                                                 "tiles per GPU + RCCL all-gather of rgb/depth",
                                     "rays_per_frame": n, "samples": S, "hidden_dim": HIDDEN,
                                     "parallelism": f"ray-tiles{world}"}}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

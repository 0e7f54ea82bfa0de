"""PSNR convergence parity (BASELINE.json north_star: "converge to the same PSNR ±0.1 dB").

For every (width, seed) the drop-in training step (Trainer.train_step: HIP render forward /
backward, fused loss, HipAdam) and the oracle (CPU restatement of training.py:70-100, run
by torch on the GPU as the checker: it is device-agnostic and gfx950 has no TF32, so its
fp32 GEMMs are true fp32) train the same initial field on the same synthetic V_KITTI-shaped
scene with identical ray draws and stratified noise every step.  The HIP side is trained
once per GEMM arithmetic (exact-f32 MFMA, bf16x6, f16x3).  Every --every steps all sides
render every pixel without noise and report PSNR (common.py:623-630); the run continues
to --steps (default 2000).  One JSON line per (width, seed) and a summary line.

    python scripts/convergence.py [--steps 2000 --seeds 0 1 2 --widths 64 256]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-nope-nerf_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

MODES = {"f32": 0, "bf16x6": 1, "f16x3": 2}
SHAPES = {64: (64, 256), 256: (128, 1024)}      # width -> (samples per ray, rays per step)
H, W, FX = 94, 310, 181.25                       # half the V_KITTI frame (188 x 621, fx 362.5)


def scene(seed, dev):
    """A smooth synthetic image + depth prior (U-shaped road-like ramp, 5 % holes)."""
    g = torch.Generator().manual_seed(1000 + seed)
    yy, xx = torch.meshgrid(torch.linspace(0, 1, H), torch.linspace(0, 1, W), indexing="ij")
    ph = torch.rand(3, generator=g) * 6.28
    img = torch.stack([0.5 + 0.35 * torch.sin(5 * xx + 2 * yy + ph[0]), 0.5 + 0.35 * torch.cos(4 * yy - 3 * xx + ph[1]),
                       0.35 + 0.3 * torch.sin(3 * xx * yy + ph[2])], 0).unsqueeze(0)
    depth = 1.5 + 5.0 * yy + 0.5 * torch.sin(4 * xx) + 0.05 * torch.rand(H, W, generator=g)
    holes = torch.rand(H, W, generator=g) < 0.05
    depth[holes] = 0.0
    return img.to(dev), depth.unsqueeze(0).to(dev), ~holes


def psnr(mse):
    return float(-10.0 * math.log10(max(mse, 1e-10)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--every", type=int, default=250)
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--widths", type=int, nargs="+", default=[64, 256])
    ap.add_argument("--modes", nargs="+", default=list(MODES))
    args = ap.parse_args()
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    import model as mdl
    from model import _hip
    from model.optim import HipAdam
    from oracle import nerf_oracle as orc
    from tests.helpers import camera_K, make_cfg, rigid_c2w
    _hip.load_library()
    dev = torch.device("cuda:0")
    K = camera_K(H, W, FX, FX).to(dev)
    scale = torch.eye(4, device=dev).unsqueeze(0)
    pix = orc.arange_pixels(H, W, device=dev)[1]
    summary = []
    for D in args.widths:
        S, R = SHAPES[D]
        for seed in args.seeds:
            t0 = time.time()
            img, depth, valid = scene(seed, dev)
            c2w = rigid_c2w(seed + 5, 0.2).to(dev)
            w2c = torch.inverse(c2w).unsqueeze(0)
            img_flat = img.view(1, 3, -1).permute(0, 2, 1)
            cfg = make_cfg(hidden=D, S=S)
            t = cfg["training"]
            t["n_training_points"] = R
            t["pc_weight"], t["rgb_s_weight"] = [0.0, 0.0], [0.0, 0.0]
            data = {"img": img, "img.idx": torch.tensor([0]), "img.depth": depth, "img.depth_mask": valid.unsqueeze(0),
                    "img.camera_mat": K, "img.scale_mat": scale, "img.pose_gt": c2w.unsqueeze(0)}
            torch.manual_seed(42 + seed)
            init = mdl.OfficialStaticNerf(cfg).state_dict()
            # oracle
            ref = orc.OracleNerf(hidden_dim=D).to(dev)
            ref.load_state_dict(init)
            opt_o = torch.optim.Adam(ref.parameters(), lr=1e-3)
            # HIP sides
            sides = {}
            for name in args.modes:
                net = mdl.OfficialStaticNerf(cfg)
                net.load_state_dict(init)
                rnd = mdl.Renderer(net, cfg["rendering"], device=dev)
                nn_model = mdl.get_model(rnd, cfg, device=dev)
                opt = HipAdam(nn_model.parameters(), lr=1e-3)
                pose = mdl.LearnPose(1, False, False, cfg, init_c2w=c2w.unsqueeze(0)).to(dev)
                sides[name] = (mdl.Trainer(nn_model, opt, t, device=dev, pose_param_net=pose), rnd)

            def eval_hip(name):
                _hip.gemm_set_precision(MODES[name])
                with torch.no_grad():
                    out = sides[name][1].nope_nerf(pix, depth.reshape(1, -1, 1), K, w2c, scale, add_noise=False,
                                                   dense_depth=True)
                return psnr(((out["rgb"] - img_flat) ** 2).mean().item())

            def eval_oracle():
                with torch.no_grad():
                    rgb = []
                    for r0 in range(0, H * W, 8192):
                        o = orc.render_nope_nerf(ref, pix[:, r0:r0 + 8192], depth.reshape(1, -1, 1)[:, r0:r0 + 8192],
                                                 K, w2c, scale, cfg["rendering"], noise=None)
                        rgb.append(o["rgb"])
                    rgb = torch.cat(rgb, 1)
                return psnr(((rgb - img_flat) ** 2).mean().item())

            curve = {"step": [], "oracle": [], **{m: [] for m in args.modes}}

            def record(step):
                curve["step"].append(step)
                curve["oracle"].append(eval_oracle())
                for m in args.modes:
                    curve[m].append(eval_hip(m))
                print(f"D={D} seed={seed} step {step}: oracle {curve['oracle'][-1]:.4f} dB  " +
                      "  ".join(f"{m} {curve[m][-1]:.4f}" for m in args.modes), file=sys.stderr, flush=True)

            record(0)
            g = torch.Generator().manual_seed(77 + seed)
            for step in range(1, args.steps + 1):
                ray_idx = torch.randperm(H * W, generator=g)[:R]
                while not valid.flatten()[ray_idx].any():          # training.py:280-283
                    ray_idx = torch.randperm(H * W, generator=g)[:R]
                noise = torch.rand(1, R, S, generator=g)
                ri, nz = ray_idx.to(dev), noise.to(dev)
                orc.train_step_render(ref, opt_o, img, depth.unsqueeze(1), K, c2w, scale, ri, nz, cfg["rendering"])
                for m in args.modes:
                    _hip.gemm_set_precision(MODES[m])
                    tr = sides[m][0]
                    tr.inject = (ri, nz)
                    tr.train_step(data, it=step, epoch=0, scheduling_start=0)
                if step % args.every == 0 or step == args.steps:
                    record(step)
            final = {m: curve[m][-1] for m in args.modes}
            last = curve["oracle"][-1]
            k = max(0, len(curve["step"]) - 3)                      # ~500 steps before the end
            line = {"width": D, "samples": S, "rays": R, "seed": seed, "steps": args.steps, "image": [H, W],
                    "psnr_oracle": last, "psnr_hip": final, "delta_db": {m: final[m] - last for m in args.modes},
                    "oracle_gain_last_500_steps_db": last - curve["oracle"][k],
                    "curve": curve, "seconds": time.time() - t0}
            print(json.dumps(line), flush=True)
            summary.append(line)
    worst = {m: max(abs(l["delta_db"][m]) for l in summary) for m in args.modes}
    print(json.dumps({"summary": True, "max_abs_delta_db": worst, "runs": len(summary),
                      "bar_db": 0.1, "pass": all(v <= 0.1 for v in worst.values())}), flush=True)


if __name__ == "__main__":
    main()

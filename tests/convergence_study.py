"""PSNR convergence parity (BASELINE.json north_star: "converge to the same PSNR ±0.1 dB").

For every (width, seed) the drop-in training step (Trainer.train_step: HIP render forward /
backward, fused loss, HipAdam) and the oracle (CPU restatement of training.py:70-100, run
by torch on the GPU as the checker: it is device-agnostic and gfx950 has no TF32, so its
fp32 GEMMs are true fp32) train the same initial field on the same synthetic V_KITTI-shaped
scene with identical ray draws and stratified noise every step.  The HIP side is trained
once per GEMM arithmetic (exact-f32 MFMA, bf16x6, f16x3).

Training is chaotic: after a few hundred Adam steps two fp32 runs that differ only in
rounding follow different trajectories, and a single snapshot PSNR swings by dB from one
step to the next.  So the study compares the PLATEAU: the PSNR of the mean full-frame MSE
over the evaluations in the last --window steps (every --every-late steps), per seed and
averaged over seeds.  As a control it trains a second oracle whose network runs in the
reference's own 64 000-sample chunks (rendering.py:102-111: exact arithmetic is unchanged,
the GEMM rounding is not) -- the reference-vs-reference spread is the floor any port can be
held to.  The scene has fine texture (a blurred noise layer over smooth gradients) so the
fields plateau below the noise-free 45-50 dB regime.  One JSON line per (width, seed) and a
summary line.

    python tests/convergence_study.py [--steps 2000 --seeds 0 1 2 --widths 64 256]

(Under tests/: it runs the oracle as the checker, which only tests may do.)
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
    """Smooth gradients + a blurred noise texture (correlation ~3 px), depth prior a road-like
    ramp with 5 % holes."""
    g = torch.Generator().manual_seed(1000 + seed)
    yy, xx = torch.meshgrid(torch.linspace(0, 1, H), torch.linspace(0, 1, W), indexing="ij")
    ph = torch.rand(3, generator=g) * 6.28
    img = torch.stack([0.5 + 0.3 * torch.sin(5 * xx + 2 * yy + ph[0]), 0.5 + 0.3 * torch.cos(4 * yy - 3 * xx + ph[1]),
                       0.35 + 0.25 * torch.sin(3 * xx * yy + ph[2])], 0).unsqueeze(0)
    tex = torch.nn.functional.avg_pool2d(torch.rand(1, 3, H, W, generator=g) - 0.5, 3, stride=1, padding=1,
                                         count_include_pad=False)
    img = (img + 0.5 * tex).clamp(0, 1)
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
    ap.add_argument("--window", type=int, default=500, help="plateau window (last steps)")
    ap.add_argument("--every-late", type=int, default=50, help="evaluation spacing inside the window")
    ap.add_argument("--chunk", type=int, default=64000,
                    help="control oracle's network chunk (the reference's n_max_network_queries); capped at half a "
                         "step's samples so the control always splits its GEMMs")
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--widths", type=int, nargs="+", default=[64, 256])
    ap.add_argument("--modes", nargs="+", default=list(MODES))
    ap.add_argument("--lr-milestones", type=float, nargs="*", default=[],
                    help="fractions of --steps at which every side's Adam learning rate is multiplied by --lr-gamma "
                         "(the same MultiStepLR on the oracle and the HIP sides; train.py:79-82 uses MultiStepLR too)")
    ap.add_argument("--lr-gamma", type=float, default=0.3)
    ap.add_argument("--no-control", dest="control", action="store_false",
                    help="skip the chunked-oracle control (halves the oracle time)")
    args = ap.parse_args()
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    import model as mdl
    from model import _hip
    from model.optim import HipAdam
    from oracle import nerf_oracle as orc
    from model.synthetic import camera_K, make_cfg, rigid_c2w
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
            ref_b = orc.OracleNerf(hidden_dim=D).to(dev)       # control: the reference's chunked network
            ref_b.load_state_dict(init)
            opt_b = torch.optim.Adam(ref_b.parameters(), lr=1e-3)
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

            def eval_oracle(net):
                with torch.no_grad():
                    rgb = []
                    for r0 in range(0, H * W, 8192):
                        o = orc.render_nope_nerf(net, pix[:, r0:r0 + 8192], depth.reshape(1, -1, 1)[:, r0:r0 + 8192],
                                                 K, w2c, scale, cfg["rendering"], noise=None)
                        rgb.append(o["rgb"])
                    rgb = torch.cat(rgb, 1)
                return psnr(((rgb - img_flat) ** 2).mean().item())

            sides_all = ["oracle"] + (["oracle_chunked"] if args.control else []) + list(args.modes)
            milestones = sorted(int(round(f * args.steps)) for f in args.lr_milestones)
            optims = [opt_o, opt_b] + [sides[m][0].optimizer for m in args.modes]
            curve = {"step": [], **{m: [] for m in sides_all}}

            def record(step):
                curve["step"].append(step)
                curve["oracle"].append(eval_oracle(ref))
                if args.control:
                    curve["oracle_chunked"].append(eval_oracle(ref_b))
                for m in args.modes:
                    curve[m].append(eval_hip(m))
                print(f"D={D} seed={seed} step {step}: " + "  ".join(f"{m} {curve[m][-1]:.4f}" for m in sides_all),
                      file=sys.stderr, flush=True)

            record(0)
            g = torch.Generator().manual_seed(77 + seed)
            for step in range(1, args.steps + 1):
                if step - 1 in milestones:                          # MultiStepLR on every side alike
                    for o in optims:
                        for grp in o.param_groups:
                            grp["lr"] *= args.lr_gamma
                ray_idx = torch.randperm(H * W, generator=g)[:R]
                while not valid.flatten()[ray_idx].any():          # training.py:280-283
                    ray_idx = torch.randperm(H * W, generator=g)[:R]
                noise = torch.rand(1, R, S, generator=g)
                ri, nz = ray_idx.to(dev), noise.to(dev)
                orc.train_step_render(ref, opt_o, img, depth.unsqueeze(1), K, c2w, scale, ri, nz, cfg["rendering"])
                if args.control:
                    orc.train_step_render(ref_b, opt_b, img, depth.unsqueeze(1), K, c2w, scale, ri, nz, cfg["rendering"],
                                          chunk=min(args.chunk, R * S // 2))
                for m in args.modes:
                    _hip.gemm_set_precision(MODES[m])
                    tr = sides[m][0]
                    tr.inject = (ri, nz)
                    tr.train_step(data, it=step, epoch=0, scheduling_start=0)
                late = step > args.steps - args.window
                if step % args.every == 0 or step == args.steps or (late and step % args.every_late == 0):
                    record(step)
            # plateau: PSNR of the mean MSE over the evaluations inside the window
            win = [i for i, st in enumerate(curve["step"]) if st >= args.steps - args.window]
            plateau = {m: -10.0 * math.log10(sum(10 ** (-curve[m][i] / 10) for i in win) / len(win)) for m in sides_all}
            early = [i for i, st in enumerate(curve["step"]) if args.steps - 2 * args.window <= st < args.steps - args.window]
            prev = (-10.0 * math.log10(sum(10 ** (-curve["oracle"][i] / 10) for i in early) / len(early))
                    if early else None)
            line = {"width": D, "samples": S, "rays": R, "seed": seed, "steps": args.steps, "image": [H, W],
                    "plateau_window_steps": args.window, "plateau_evals": len(win), "plateau_psnr": plateau,
                    "lr_milestones": milestones, "lr_gamma": args.lr_gamma,
                    "delta_db": {m: plateau[m] - plateau["oracle"] for m in sides_all if m != "oracle"},
                    "oracle_plateau_gain_over_previous_window_db": (plateau["oracle"] - prev) if prev else None,
                    "curve": curve, "seconds": time.time() - t0}
            print(json.dumps(line), flush=True)
            summary.append(line)
    keys = [m for m in summary[0]["delta_db"]]
    agg = {}
    for D in args.widths:
        runs = [l for l in summary if l["width"] == D]
        agg[D] = {}
        for m in keys + ["oracle"]:
            v = [l["plateau_psnr"][m] for l in runs]
            agg[D][m] = {"mean_plateau_psnr": sum(v) / len(v)}
        for m in keys:
            d = [l["delta_db"][m] for l in runs]
            mu = sum(d) / len(d)
            sd = (sum((x - mu) ** 2 for x in d) / max(1, len(d) - 1)) ** 0.5
            agg[D][m].update({"mean_delta_db": mu, "std_delta_db": sd, "max_abs_delta_db": max(abs(x) for x in d)})
    ok = all(abs(agg[D][m]["mean_delta_db"]) <= 0.1 for D in args.widths for m in args.modes)
    print(json.dumps({"summary": True, "per_width": agg, "seeds": args.seeds, "bar_db": 0.1,
                      "bar": "|mean over seeds of plateau PSNR(HIP) - plateau PSNR(oracle)| <= 0.1 dB",
                      "pass": ok}), flush=True)


if __name__ == "__main__":
    main()

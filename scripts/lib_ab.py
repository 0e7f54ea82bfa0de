"""A/B of whole libraries on the cfg2 training step: bench.py (eager, no alt / cpu / cfg3 /
render lines) in one child process per library and round, libraries interleaved over rounds;
prints each run's ms/step and the per-library median.  Diagnostic builds are made outside the
tree's sources and are not committed.

    python scripts/lib_ab.py [--rounds 2] my-nope-nerf_amd/lib/ab/x.so ...

A setting may also be the tree's library under environment knobs, "env:NERF_WGRAD_GROUPS=2[,K=V]"
(every run starts from the same seeds and weights, so the settings see the same data -- unlike an
in-process A/B whose trainers drift apart); --exec auto times the replayed graph too.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--exec", dest="exec_mode", default="eager", choices=["eager", "auto"])
    ap.add_argument("libs", nargs="*")
    args = ap.parse_args()
    libs = ["my-nope-nerf_amd/lib/libnerf_hip.so"] + args.libs
    res = {lib: [] for lib in libs}
    for r in range(args.rounds):
        for lib in libs:
            if lib.startswith("env:"):
                env = dict(os.environ, NERF_HIP_LIB=os.path.join(ROOT, libs[0]),
                           **dict(kv.split("=", 1) for kv in lib[4:].split(",")))
            else:
                env = dict(os.environ, NERF_HIP_LIB=os.path.join(ROOT, lib))
            out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(args.steps),
                                  "--warmup", "5", "--no-alt", "--no-cpu-baseline", "--no-cfg3",
                                  "--exec", args.exec_mode], env=env, capture_output=True, text=True, timeout=600)
            line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
            if not line:
                print(lib, "FAILED", out.stderr[-600:], flush=True)
                sys.exit(1)
            d = json.loads(line[-1])
            res[lib].append(d["ms_per_step"])
            rk = d.get("roofline", {}).get("per_kind", {})
            kinds = " ".join(f"{k} {v['avg_launch_us']:.1f}us" for k, v in rk.items())
            frame = (d.get("render_cfg4") or {}).get("ms_per_frame", float("nan"))
            gr = d.get("ms_per_step_graph")
            gtxt = f" (eager {d['ms_per_step_eager']:.4f}, graph {gr:.4f})" if gr else ""
            print(f"round {r} {lib}: {d['ms_per_step']:.4f} ms/step{gtxt}  frame {frame:.2f} ms  {kinds}", flush=True)
    for lib, v in res.items():
        print(f"median {lib}: {statistics.median(v):.4f} ms/step over {len(v)}", flush=True)


if __name__ == "__main__":
    main()

"""Diagnostic A/B of the weight-gradient kernel: the standalone 256 x 256 layer
(wgrad_bench.py) with each library given on the command line (NERF_HIP_LIB), one child
process per library.  Diagnostic builds are made outside the tree's sources and are not
committed.

    python scripts/wgrad_ab.py lib/ab/x.so lib/ab/y.so ...
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for lib in ["my-nope-nerf_amd/lib/libnerf_hip.so"] + sys.argv[1:]:
    env = dict(os.environ, NERF_HIP_LIB=os.path.join(ROOT, lib) if not os.path.isabs(lib) else lib)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "wgrad_bench.py"), "--shapes", "256x256",
                          "--no-check"], env=env, capture_output=True, text=True)
    lines = [ln for ln in out.stdout.splitlines() if "policy 8" in ln]
    print(lib, lines[0] if lines else out.stderr[-400:], flush=True)

"""Round-6 verdict item 8: does forking k_heads_reduce beside the input-gradient chain stretch
the chain?  Reads rocprofv3 kernel traces of the cfg2 bench (eager), one per NERF_HEADS_PLACE
setting, and prints per setting the in-step duration distribution (mean, p50, p95, max) of
k_mlp_chain_bwd and k_heads_reduce and the median step span (scripts/timeline.py's step split).

    python scripts/heads_ab.py place5=<trace.csv> place1=<trace.csv> [--skip 3] > summary.json
"""
from __future__ import annotations

import csv
import json
import statistics
import sys


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(round(q * (len(v) - 1))))]


def summary(path, skip):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [s for s, _, n in rows if "k_sample_rays" in n]
    steps = [[r for r in rows if starts[i] <= r[0] < starts[i + 1]] for i in range(len(starts) - 1)][skip:]
    out = {"steps": len(steps)}
    span = [(max(e for _, e, _ in st) - st[0][0]) / 1e3 for st in steps]
    out["step_span_us_median"] = statistics.median(span)
    for key in ("k_mlp_chain_bwd", "k_heads_reduce", "k_heads_bwd", "k_mlp_chain_train2"):
        d = [(e - s) / 1e3 for st in steps for s, e, n in st if key in n]
        if d:
            out[key] = {"n": len(d), "mean_us": statistics.mean(d), "p50_us": pct(d, 0.5), "p95_us": pct(d, 0.95),
                        "max_us": max(d), "min_us": min(d)}
    return out


def main():
    skip = 3
    args = [a for a in sys.argv[1:]]
    if "--skip" in args:
        i = args.index("--skip")
        skip = int(args[i + 1])
        del args[i:i + 2]
    res = {}
    for a in args:
        name, path = a.split("=", 1)
        res[name] = summary(path, skip)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

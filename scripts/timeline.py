"""Critical-path view of a rocprofv3 kernel trace (``--kernel-trace --output-format csv``):
per step, the busy union of all kernels, the idle gaps, and per kernel family the time
during which it was the ONLY kernel running (exposed) vs overlapped.

    python scripts/timeline.py <run_kernel_trace.csv> [--marker k_sample_rays] [--skip 3]

A step starts at each launch of the marker kernel (the ray sampler opens every
train_step); the first --skip steps are dropped (warm-up)."""
from __future__ import annotations

import argparse
import csv
import re
import statistics
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name)
    n = n.replace("void ", "").replace("nerf::", "")
    if "at::native" in n:
        m = re.search(r"at::native::(?:\(anonymous namespace\)::)?(\w+)", n)
        return "torch:" + (m.group(1) if m else n[:40])
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="k_sample_rays")
    ap.add_argument("--skip", type=int, default=3)
    ap.add_argument("--gaps", type=float, default=0.0, help="list idle gaps of at least this many us")
    args = ap.parse_args()
    rows = []
    with open(args.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    starts = [s for s, _, n in rows if args.marker in n]
    steps = []
    for i in range(len(starts) - 1):
        steps.append([r for r in rows if starts[i] <= r[0] < starts[i + 1]])
    steps = steps[args.skip:]
    if not steps:
        raise SystemExit("no complete steps found")
    span, busy, gaps = [], [], []
    excl = defaultdict(list)
    total = defaultdict(list)
    for st in steps:
        t0 = st[0][0]
        t1 = max(e for _, e, _ in st)
        span.append((t1 - t0) / 1e3)
        # sweep: exclusive time per kernel name when it runs alone
        ev = []
        for s, e, n in st:
            ev.append((s, 1, n))
            ev.append((e, -1, n))
        ev.sort(key=lambda x: (x[0], x[1]))
        active = defaultdict(int)
        last = t0
        b = 0
        ex = defaultdict(float)
        for t, d, n in ev:
            live = [k for k, v in active.items() if v > 0]
            if len(live) >= 1:
                b += t - last
            if len(live) == 1:
                ex[live[0]] += t - last
            active[n] += d
            last = t
        busy.append(b / 1e3)
        gaps.append((t1 - t0 - b) / 1e3)
        tot = defaultdict(float)
        for s, e, n in st:
            tot[n] += (e - s) / 1e3
        for n in set(list(tot) + list(ex)):
            excl[n].append(ex.get(n, 0.0) / 1e3)
            total[n].append(tot.get(n, 0.0))
    med = statistics.median
    print(f"steps analysed: {len(steps)}  span {med(span):.1f} us  busy {med(busy):.1f} us  idle gaps {med(gaps):.1f} us")
    print(f"{'kernel':60s} {'sum us':>9s} {'alone us':>9s}")
    for n in sorted(total, key=lambda k: -med(total[k])):
        print(f"{n:60s} {med(total[n]):9.1f} {med(excl[n]):9.1f}")
    if args.gaps:
        # idle intervals of the median step, keyed by (kernel that ended last, kernel that starts next)
        st = steps[len(steps) // 2]
        out = []
        end_max, prev = st[0][1], st[0][2]
        for s, e, n in st[1:]:
            if s > end_max:
                out.append(((s - end_max) / 1e3, prev, n, (end_max - st[0][0]) / 1e3))
            if e > end_max:
                end_max, prev = e, n
        print(f"\nidle gaps of one step (>= {args.gaps} us), in order: at_us  gap_us  after -> before")
        for g, a, b, at in out:
            if g >= args.gaps:
                print(f"{at:9.1f} {g:7.1f}  {a} -> {b}")


if __name__ == "__main__":
    main()

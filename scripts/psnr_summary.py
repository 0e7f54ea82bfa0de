"""Summary of tests/convergence_study.py runs (one JSON line per (width, seed) plus a summary
line per run) over several files: per-mode mean / std / max |delta| of the plateau PSNR against
the fp32 oracle over all seeds, and the +-0.1 dB bar on the mean.

    python scripts/psnr_summary.py profiles/r06/psnr_study_seeds012.jsonl profiles/r06/psnr_study_seeds345.jsonl
"""
import json
import statistics
import sys


def main():
    rows = []
    for path in sys.argv[1:]:
        for line in open(path):
            d = json.loads(line)
            if not d.get("summary"):
                rows.append(d)
    rows.sort(key=lambda d: (d["width"], d["seed"]))
    modes = sorted({m for d in rows for m in d["delta_db"]})
    out = {"source": sys.argv[1:], "seeds": [d["seed"] for d in rows], "widths": sorted({d["width"] for d in rows}),
           "bar": "|mean over seeds of plateau PSNR(HIP) - plateau PSNR(oracle)| <= 0.1 dB"}
    for m in modes:
        v = [d["delta_db"][m] for d in rows]
        out[m] = {"mean_delta_db": statistics.mean(v), "std_delta_db": statistics.pstdev(v),
                  "max_abs_delta_db": max(abs(x) for x in v), "per_seed": v}
    out["oracle_mean_plateau_psnr"] = statistics.mean(d["plateau_psnr"]["oracle"] for d in rows)
    out["pass"] = all(abs(out[m]["mean_delta_db"]) <= 0.1 for m in modes if m != "oracle_chunked")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

"""HBM bytes per fused eval-render launch (k_mlp_chain_fwd<true>, one 188x621 x 128-sample
frame) from two rocprofv3 PMC passes of scripts/bench_render.py (FETCH_SIZE x2 per the gfx950
correction in MI355X_MICROARCH.md's HBM section, WRITE_SIZE as is; KiB), against what the
unfused path moves per frame.

    python scripts/render_pmc_summary.py gpurun_out/r02bi/pmc_fetch gpurun_out/r02bi/pmc_write
"""
import collections
import csv
import json
import statistics
import sys

RAYS, S, D = 188 * 621, 128, 256


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        agg[r["Kernel_Name"].replace("void nerf::", "").split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    fetch, write = load(sys.argv[1]), load(sys.argv[2])
    k = "k_mlp_chain_fwd<true>"
    rd = 2 * statistics.median(fetch[k]["FETCH_SIZE"]) * 1024
    wr = statistics.median(write[k]["WRITE_SIZE"]) * 1024
    n = RAYS * S
    out_bytes = 8 * n + 16 * RAYS          # alpha + z per sample, rgb + depth per ray (the out-dict)
    # the per-layer path per frame: encodings written + read (2 x 64 floats x 2), ten layer outputs
    # written + read (9 x D + D/2 floats), raw4 written + read: a lower bound of its HBM bytes
    unfused = 4 * n * (2 * 2 * 64 + 2 * (9 * D + D // 2) + 2 * 4)
    print(json.dumps({
        "kernel": k, "launches_profiled": len(fetch[k]["FETCH_SIZE"]),
        "read_bytes_per_frame": rd, "write_bytes_per_frame": wr, "bytes_per_frame": rd + wr,
        "bytes_per_sample": (rd + wr) / n,
        "algorithmic_out_bytes_per_frame": out_bytes,
        "unfused_activation_bytes_per_frame_lower_bound": unfused,
        "source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of "
                  "`scripts/bench_render.py --frames 2 --warmup 1`; FETCH_SIZE x2 (gfx950 correction)"}, indent=1))


if __name__ == "__main__":
    main()

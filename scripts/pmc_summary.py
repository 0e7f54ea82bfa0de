"""Summarise rocprofv3 PMC passes of the GEMM launches into per-launch HBM bytes per GEMM
kind (MI355X_MICROARCH.md HBM section: FETCH_SIZE is in KiB and counts half of the bytes
of 16-B-per-lane streaming reads on gfx950 -> x2; WRITE_SIZE exact).  The passes are
separate runs of the same command (`bench.py --steps 3 --warmup 2 --no-alt
--no-cpu-baseline --exec eager` under `--kernel-include-regex 'k_gemm_(nt|tn)_x6'`); launches of one
kernel are summarised by their median.

    python scripts/pmc_summary.py gpurun_out/r02g/pmc_fetch gpurun_out/r02g/pmc_write \\
        [gpurun_out/r02g/pmc_sq] > profiles/r02/gemm_traffic.json
"""
import collections
import csv
import json
import statistics
import sys

M = 131072          # samples per cfg2 step (1024 rays x 128)
D = 256
# kernel template -> (GEMM kind of bench.py's roofline, algorithmic bytes per launch, note)
KINDS = {
    "k_gemm_nt_x6<128, 256, 2, 2, 0, true, true, 2, false>": (
        "fwd", 4 * M * D * 2 + 4 * D * D + M * D / 8, "x 134.2 MB + y 134.2 MB + W 0.26 MB + ReLU bits 4.2 MB "
        "(256-wide layers; the skip layer reads 320 columns)"),
    "k_gemm_nt_x6<128, 256, 2, 2, 1, true, true, 2, false>": (
        "dx", 4 * M * D * 2 + 4 * D * D + M * D / 8, "dy 134.2 MB + dx 134.2 MB + W^T 0.26 MB + ReLU bits 4.2 MB"),
    "k_gemm_tn_x6<256, 128, 4, 2, true, 1, 2>": (
        "dw", 4 * M * D * 2 + 4 * D * D, "dy 134.2 MB + x 134.2 MB + dW 0.26 MB; one launch is both XCD-paired "
        "256 x 128 column tiles, so dy is fetched by two blocks of one XCD; measured writes are the 128 split-K "
        "slabs (33.6 MB)"),
    "nerf::k_mlp_chain_train2": (
        "chain_fwd", 4 * M * 64 * 2 + 4 * M * 2 + 4 * M * D * 9 + 4 * M * 128 + 4 * M * 9 * 8 + 4 * M * 4 +
        4 * (M // 128) * D * 9 + 4 * M * 4,
        "reads enc_p + enc_d 67.1 MB + their row maxima 1.0 MB (weights stream from L2); writes the nine 256-wide "
        "outputs 1208 MB + hr 67.1 MB + ReLU words 37.7 MB + column maxima 9.4 MB + raw4 2.1 MB"),
    "k_gemm_tn_x6_seg<256, 128, 4, 2, 64, 4, 2, 2, 1>": (
        "dw", 4 * M * (D + D + 64) + 4 * D * (D + 64), "dy 134.2 MB + h3 134.2 MB + enc_p 33.6 MB + dW 0.33 MB "
        "(l4: two XCD-grouped 256 x 128 tiles over h3 and the 256 x 64 tile over enc_p, dy fetched once per XCD); "
        "measured writes are the 128 split-K slabs (41.9 MB)"),
    "k_gemm_tn_x6_seg<128, 256, 2, 4, 64, 4, 2, 1, 1>": (
        "dw_narrow", 4 * M * (128 + D + 64) + 4 * 128 * (D + 64), "dy 67.1 MB + f 134.2 MB + enc_d 33.6 MB + dW "
        "0.16 MB (colour layer: the 128 x 256 tile over f and the 128 x 64 tile over enc_d, dy fetched once per XCD); "
        "measured writes are the 256 split-K slabs (41.9 MB)"),
    "nerf::k_wgrad_pair": (
        "dw", 4 * M * D * 2 + 4 * D * D, "dy 134.2 MB + x 134.2 MB + dW 0.26 MB; the two XCD-paired 256 x 128 "
        "column tiles of a split read dy from HBM once; measured writes are the 128 split-K slabs (33.6 MB)"),
    "nerf::k_wgrad_pairs": (
        "dw", 8 * (4 * M * D * 2 + 4 * D * D), "eight 256 x 256 layers (l_f .. l1, l4 over its h3 segment) in one "
        "launch: per layer dy 134.2 MB + x 134.2 MB + dW 0.26 MB; measured writes are the 8 x 128 split-K slabs "
        "(268 MB)"),
    "nerf::k_wgrad_two": (
        "dw_narrow", 4 * M * (D + 64) * 2 + 2 * 4 * D * 64, "l4's enc_p segment and l0 in one launch: per layer dy "
        "134.2 MB + enc_p 33.6 MB + dW 0.07 MB; measured writes are the split-K slabs (8.4 + 16.8 MB)"),
    "k_wgrad_one<128, 256>": (
        "dw_narrow", 4 * M * (128 + D) + 4 * 128 * D, "dyr 67.1 MB + f 134.2 MB + dW 0.13 MB (colour layer, f "
        "segment); measured writes are the 256 split-K slabs (33.6 MB)"),
    "k_wgrad_one<128, 64>": (
        "dw_narrow", 4 * M * (128 + 64) + 4 * 128 * 64, "dyr 67.1 MB + enc_d 33.6 MB + dW 0.03 MB (colour layer, "
        "enc_d segment); measured writes are the 256 split-K slabs (8.4 MB)"),
    "k_wgrad_seg<256, 128, 2, 64>": (
        "dw", 4 * M * (D + D + 64) + 4 * D * (D + 64), "dy 134.2 MB + h3 134.2 MB + enc_p 33.6 MB + dW 0.33 MB "
        "(l4); measured writes are the 128 split-K slabs (41.9 MB)"),
    "k_wgrad_seg<128, 256, 1, 64>": (
        "dw_narrow", 4 * M * (128 + D + 64) + 4 * 128 * (D + 64), "dyr 67.1 MB + f 134.2 MB + enc_d 33.6 MB + dW "
        "0.16 MB (colour layer); measured writes are the 256 split-K slabs (41.9 MB)"),
    "k_wgrad_one<256, 64>": (
        "dw_narrow", 4 * M * (D + 64) + 4 * D * 64, "dy 134.2 MB + enc_p 33.6 MB + dW 0.07 MB (l0); measured writes "
        "are the 256 split-K slabs (16.8 MB)"),
    "nerf::k_mlp_chain_bwd": (
        "chain_bwd", M * (16 + 16 + 8 * 32) + 4 * M * 128 + 4 * M * D * 9 + 4 * M * 10 + 4 * (M // 128) * (128 + 9 * D),
        "reads graw4 2.1 MB + the ReLU words of ten layers 37.7 MB (weights stream from L2); writes dyr 67.1 MB + "
        "the nine 256-wide input gradients 1208 MB + row maxima 5.2 MB + column maxima 9.4 MB"),
    # TN schedule 3 (round 5): dy counted once per layer (a second segment adds its x only), as
    # gemm_f32.hip's prof_next for k_wgrad_jobs
    "k_wgrad_jobs<3>": (
        "dw", (4 * M * (D + 128) + 4 * 128 * D + 4 * 128) + (4 * M * 64 + 4 * 128 * 64) +
        4 * (4 * M * 2 * D + 4 * D * D + 4 * D),
        "the colour layer over [f | enc_d] (dyr 67.1 MB + f 134.2 MB + enc_d 33.6 MB) + l_f, l7, l6, l5 (dy + x "
        "268.4 MB each); measured writes are the split-K slabs (round 5: 41.9 + 4 x 33.6 MB; round 6, two block groups at half the splits: 21 + 4 x 16.8 MB)"),
    "k_wgrad_jobs<6>": (
        "dw", (4 * M * 2 * D + 4 * D * D + 4 * D) + (4 * M * 64 + 4 * D * 64) + 3 * (4 * M * 2 * D + 4 * D * D + 4 * D) +
        (4 * M * (64 + D) + 4 * D * 64 + 4 * D),
        "l4 over [h3 | enc_p] (dy + h3 268.4 MB + enc_p 33.6 MB) + l3, l2, l1 (268.4 MB each) + l0 (dy 134.2 MB + "
        "enc_p 33.6 MB); measured writes are the split-K slabs (round 5: 41.9 + 3 x 33.6 + 16.8 MB; round 6, block groups: 21 + 3 x 16.8 + 8.4 MB)"),
    "k_gemm_tn_x6<256, 256, 2, 2, true, 1>": (
        "dw", 4 * M * D * 2 + 4 * D * D, "dy 134.2 MB + x 134.2 MB + dW 0.26 MB; measured writes are the 256 "
        "split-K slabs (67 MB)"),
}


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        agg[r["Kernel_Name"].replace("void nerf::", "").split("(")[0]][r["Counter_Name"]].append(
            float(r["Counter_Value"]))
    return agg


def main():
    fetch, write = load(sys.argv[1]), load(sys.argv[2])
    sq = load(sys.argv[3]) if len(sys.argv) > 3 else {}
    out = []
    for k in sorted(fetch):
        rd = 2 * statistics.median(fetch[k]["FETCH_SIZE"]) * 1024
        wr = statistics.median(write[k]["WRITE_SIZE"]) * 1024
        e = {"kernel": k, "launches_profiled": len(fetch[k]["FETCH_SIZE"]), "read_bytes": rd, "write_bytes": wr,
             "bytes": rd + wr}
        if k in KINDS:
            kind, alg, note = KINDS[k]
            e.update({"kind": kind, "algorithmic_bytes": alg, "traffic_over_algorithmic": (rd + wr) / alg,
                      "note": f"in-step launches, median over the profiled steps; algorithmic: {note}"})
        if k in sq:
            s = {c: statistics.median(v) for c, v in sq[k].items()}
            waves = s.get("SQ_WAVES", 0) or 1
            # SQ_WAVE_CYCLES / _WAIT_INST_ANY / _ACTIVE_INST_ANY count quad-cycles (guide)
            e["per_wave_cycles"] = {"lifetime": 4 * s.get("SQ_WAVE_CYCLES", 0) / waves,
                                    "waiting_on_dependencies": 4 * s.get("SQ_WAIT_INST_ANY", 0) / waves,
                                    "issuing": 4 * s.get("SQ_ACTIVE_INST_ANY", 0) / waves,
                                    "mfma_busy": s.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / waves}
        out.append(e)
    # per GEMM kind (bench.py roofline.per_kind): mean HBM bytes over every launch of the kind's
    # kernels -- the same launch set bench.py averages its algorithmic bytes over, so the two
    # divide (a kind such as dw mixes launches of different sizes: l_f..l5, l4, l3..l1)
    kinds = collections.defaultdict(lambda: {"read": 0.0, "write": 0.0, "launches": 0})
    for k in sorted(fetch):
        if k not in KINDS:
            continue
        kd = kinds[KINDS[k][0]]
        kd["read"] += 2 * sum(fetch[k]["FETCH_SIZE"]) * 1024
        kd["write"] += sum(write[k]["WRITE_SIZE"]) * 1024
        kd["launches"] += len(fetch[k]["FETCH_SIZE"])
    per_kind = {k: {"bytes_per_launch": (v["read"] + v["write"]) / v["launches"],
                    "read_bytes_per_launch": v["read"] / v["launches"],
                    "write_bytes_per_launch": v["write"] / v["launches"], "launches_profiled": v["launches"]}
                for k, v in kinds.items()}
    print(json.dumps({"source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / --pmc WRITE_SIZE / SQ counters "
                                "(separate passes) of `bench.py --steps 3 --warmup 2 --no-alt --no-cpu-baseline`, "
                                "--kernel-include-regex 'k_gemm_(nt|tn)_x6|k_wgrad|k_mlp_chain'; FETCH_SIZE x2 (gfx950 correction)",
                      "launches": out, "kinds": per_kind}, indent=1))


if __name__ == "__main__":
    main()

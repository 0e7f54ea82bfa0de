"""Per-wave SQ counters of the two training chains (k_mlp_chain_train2, k_mlp_chain_bwd) from two
rocprofv3 PMC passes of the cfg2 bench step (scripts/gpu/check.sh pmc:ch1 / pmc:ch2):

    python scripts/chain_sq_summary.py gpurun_out/r05d/pmc_ch1 gpurun_out/r05d/pmc_ch2 > profiles/r05/chain_sq.json

SQ_INSTS_VALU counts the MFMA instructions too (the static instruction counts of the fully
unrolled kernels, scripts/isa/isa_mix.py, reproduce it), so both ratios are given: all VALU
per MFMA (the verdict's VALU/MFMA) and the non-MFMA VALU per MFMA.  SQ_WAVE_CYCLES,
SQ_WAIT_* and SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md); SQ_VALU_MFMA_BUSY_CYCLES
counts cycles (16 per v_mfma_f32_16x16x32_f16)."""
import collections
import csv
import json
import sys


def per_wave(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        k = r["Kernel_Name"].split("(")[0].replace("nerf::", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return {k: {c: v / agg[k]["SQ_WAVES"] for c, v in cs.items() if c != "SQ_WAVES"} | {
        "waves_per_dispatch": agg[k]["SQ_WAVES"] / len(disp[k]), "dispatches": len(disp[k])} for k, cs in agg.items()}


def main():
    a, b = per_wave(sys.argv[1]), per_wave(sys.argv[2])
    out = {"source": f"{sys.argv[1]} + {sys.argv[2]} (rocprofv3 --pmc, bench.py --steps 3 --warmup 2 --exec eager)",
           "kernels": {}}
    for k in sorted(set(a) & set(b)):
        c = {**a[k], **b[k]}
        mfma = c["SQ_INSTS_MFMA"]
        life = 4 * c["SQ_WAVE_CYCLES"]
        out["kernels"][k] = {
            "per_wave": {n: round(v, 1) for n, v in sorted(c.items())},
            "valu_per_mfma": c["SQ_INSTS_VALU"] / mfma,
            "non_mfma_valu_per_mfma": (c["SQ_INSTS_VALU"] - mfma) / mfma,
            "wave_cycles": life,
            "wait_any_frac": 4 * c["SQ_WAIT_ANY"] / life,
            "wait_inst_any_frac": 4 * c["SQ_WAIT_INST_ANY"] / life,
            "wait_inst_lds_frac": 4 * c["SQ_WAIT_INST_LDS"] / life,
            # two waves share a SIMD: its MFMA pipe is busy 2 x (per-wave busy cycles) of a wave's life
            "simd_mfma_busy_frac": 2 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / life,
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

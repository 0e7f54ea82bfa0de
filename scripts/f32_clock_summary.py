"""Per-kernel effective clock and MFMA busy of the exact-f32 GEMMs from a rocprofv3 PMC
pass of scripts/f32_clock.py (--pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES
SQ_WAVE_CYCLES SQ_WAVES --kernel-trace).

    effective clock = GRBM_GUI_ACTIVE / 8 (XCDs) / dispatch duration   (MI355X_MICROARCH.md, DVFS)
    MFMA issue floor = (M x 256 x 256 / (32 x 32 x 2)) v_mfma_f32_32x32x2_f32 x 64 cycles over
                       1024 SIMDs, at that clock
    SQ_VALU_MFMA_BUSY_CYCLES per SIMD-cycle of the dispatch (its unit is calibrated here by the
    ratio to the floor)

    python scripts/f32_clock_summary.py <pmc dir> [rows]
"""
import collections
import csv
import glob
import json
import statistics
import sys


def main():
    d = sys.argv[1]
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 4 * 131072
    ctr = collections.defaultdict(lambda: collections.defaultdict(dict))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("void nerf::", "").split("(")[0]
            disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
            ctr[name][disp][r["Counter_Name"]] = float(r["Counter_Value"])
    dur = {}
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
            dur[disp] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    n_mfma = rows * 256 * 256 / (32 * 32 * 2)
    out = {}
    for name, per in ctr.items():
        clocks, busy, dts = [], [], []
        for disp, c in per.items():
            if disp not in dur or "GRBM_GUI_ACTIVE" not in c:
                continue
            dt = dur[disp]
            clk = c["GRBM_GUI_ACTIVE"] / 8 / dt
            clocks.append(clk)
            dts.append(dt)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                busy.append(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * clk * dt))
        if not clocks:
            continue
        clk, dt = statistics.median(clocks), statistics.median(dts)
        floor = n_mfma * 64 / 1024 / clk
        out[name] = {"dispatches": len(clocks), "duration_us": dt * 1e6, "effective_clock_ghz": clk / 1e9,
                     "mfma_issue_floor_us_at_that_clock": floor * 1e6,
                     "mfma_floor_fraction": floor / dt if "gemm" in name else None,
                     "sq_valu_mfma_busy_per_simd_cycle": statistics.median(busy) if busy else None,
                     "tflops": 2.0 * rows * 256 * 256 / dt / 1e12 if "gemm" in name else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

"""Merge several rocprofv3 PMC passes (``--pmc``, one directory each) into one per-kernel table:
SQ_* counters per wave (divided by SQ_WAVES of the same pass), every other block's counters per
dispatch.  SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* / SQ_INST_CYCLES_* count quad-cycles,
SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES / SQ_LDS_* cycles (MI355X_MICROARCH.md).

    python scripts/pmc_merge.py gpurun_out/r06f/pmc_vm gpurun_out/r06f/pmc_lds ... > summary.json
"""
import collections
import csv
import glob
import json
import sys


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    path = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("nerf::", "").replace("void ", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    out = {}
    for k, cs in agg.items():
        nd = len(disp[k])
        w = cs.get("SQ_WAVES", 0.0)
        row = {"dispatches": nd}
        for c, v in cs.items():
            if c == "SQ_WAVES":
                row["waves_per_dispatch"] = v / nd
            elif c.startswith("SQ_") and w:
                row[c + "/wave"] = v / w
            else:
                row[c + "/dispatch"] = v / nd
        out[k] = row
    return out


def main():
    res = collections.defaultdict(dict)
    for d in sys.argv[1:]:
        for k, row in load(d).items():
            res[k].update(row)
    print(json.dumps({"sources": sys.argv[1:], "kernels": res}, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()

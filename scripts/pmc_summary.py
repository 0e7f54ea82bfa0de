"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes of `gemm_bench.py --quick --x6` into
per-launch HBM bytes (MI355X_MICROARCH.md HBM section: FETCH_SIZE is in KiB and counts
half of the bytes of 16-B-per-lane streaming reads on gfx950 -> x2; WRITE_SIZE exact).

    python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write > profiles/r01/gemm_traffic.json
"""
import csv
import json
import sys


def load(d, counter):
    agg = {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if r["Counter_Name"] != counter:
            continue
        key = (int(r["Dispatch_Id"]), r["Kernel_Name"])
        agg[key] = agg.get(key, 0.0) + float(r["Counter_Value"])
    return agg


def main():
    fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    # the two passes run the same launch sequence: pair them by order
    fk, wk = sorted(fetch), sorted(write)
    out = []
    for (fd, fn), (wd, wn) in zip(fk, wk):
        if "gemm" not in fn:
            continue
        assert fn == wn, (fn, wn)
        rd = 2 * fetch[(fd, fn)] * 1024
        wr = write[(wd, wn)] * 1024
        out.append({"kernel": fn.split("(")[0], "read_bytes": rd, "write_bytes": wr, "bytes": rd + wr})
    print(json.dumps({"source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) "
                                "of scripts/gemm_bench.py --quick --x6; FETCH_SIZE x2 (gfx950 correction)",
                      "launches": out}, indent=1))


if __name__ == "__main__":
    main()

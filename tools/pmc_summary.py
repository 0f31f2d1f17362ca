"""Summarise rocprofv3 output for profiles/: per-kernel dispatch statistics and per-dispatch PMC
means (FETCH_SIZE / WRITE_SIZE corrected as MI355X_MICROARCH.md §HBM prescribes: both in KB,
FETCH_SIZE doubled on gfx950 for 16-B coalesced reads).

    python tools/pmc_summary.py <rocprof dir> [<rocprof dir> ...] > summary.json
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("mha_hd64::(anonymous namespace)::", "")


def main():
    kernels = defaultdict(list)
    counters = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    kernels[row["Kernel_Name"]].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    counters[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {"kernel_trace": {}, "pmc": {}}
    for k, v in sorted(kernels.items(), key=lambda kv: -sum(kv[1])):
        out["kernel_trace"][short(k)] = {"calls": len(v), "avg_ns": round(statistics.mean(v), 1),
                                         "median_ns": statistics.median(v), "min_ns": min(v)}
    for k, cs in counters.items():
        e = {c: {"mean": round(statistics.mean(v), 2), "n": len(v)} for c, v in sorted(cs.items())}
        if "FETCH_SIZE" in cs:
            e["hbm_read_bytes_per_dispatch"] = round(statistics.mean(cs["FETCH_SIZE"]) * 1024 * 2)
        if "WRITE_SIZE" in cs:
            e["hbm_write_bytes_per_dispatch"] = round(statistics.mean(cs["WRITE_SIZE"]) * 1024)
        out["pmc"][short(k)] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

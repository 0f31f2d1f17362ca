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
    # drop the return type and the namespaces that carry parentheses, then the argument list
    name = name.removeprefix("void ").replace("(anonymous namespace)::", "").replace("mha_hd64::", "")
    return name.split("(")[0]


def main():
    kernels = defaultdict(list)
    intervals = defaultdict(list)
    counters = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            with open(path) as f:
                rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
            for i, row in enumerate(rows):
                t0, t1 = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
                kernels[row["Kernel_Name"]].append(t1 - t0)
                # dispatch-to-dispatch interval inside back-to-back runs of one kernel (graph
                # replays): the quantity bench.py's event timing of K launches measures
                if i and rows[i - 1]["Kernel_Name"] == row["Kernel_Name"]:
                    gap = t0 - int(rows[i - 1]["Start_Timestamp"])
                    if gap < 3 * (t1 - t0) + 5000:
                        intervals[row["Kernel_Name"]].append(gap)
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    counters[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {"kernel_trace": {}, "pmc": {}}
    for k, v in sorted(kernels.items(), key=lambda kv: -sum(kv[1])):
        e = {"calls": len(v), "avg_ns": round(statistics.mean(v), 1), "median_ns": statistics.median(v),
             "min_ns": min(v)}
        iv = intervals.get(k)
        if iv:
            e["back_to_back_launches"] = len(iv)
            e["dispatch_interval_avg_ns"] = round(statistics.mean(iv), 1)
            e["dispatch_interval_median_ns"] = statistics.median(iv)
        out["kernel_trace"][short(k)] = e
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

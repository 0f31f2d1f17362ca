"""Summarise tools/gpu/matcher_pmc.sh output: per kernel of one fp16 matcher forward, dispatches
per forward, median duration (kernel trace), HBM bytes read / written per dispatch (FETCH_SIZE x 2
and WRITE_SIZE in KB: the gfx950 correction of MI355X_MICROARCH.md) and the bandwidth that implies
against the ~8 TB/s HBM peak; totals per forward.

    python tools/matcher_traffic.py <dir> <P> <n>
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402

HBM_PEAK = 8.0e12


def main():
    d, P, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    # the graph replays only: dispatches from the third pair-inputs dispatch on (the first two are the
    # eager warm-up forwards; model set-up copies and casts come before them)
    rows_kt = []
    for path in glob.glob(os.path.join(d, "kt", "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            rows_kt += list(csv.DictReader(f))
    rows_kt.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows_kt) if "pair_inputs" in r["Kernel_Name"]]
    window = rows_kt[starts[2]:] if len(starts) > 2 else rows_kt
    forwards = max(1, len(starts) - 2)
    dur = defaultdict(list)
    for row in window:
        dur[short(row["Kernel_Name"])].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    ctr = defaultdict(lambda: defaultdict(list))
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        for path in glob.glob(os.path.join(d, "pmc_" + c, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    if row["Counter_Name"] == c:
                        ctr[short(row["Kernel_Name"])][c].append(float(row["Counter_Value"]))
    per_fwd_ref = forwards
    rows, tot_t, tot_r, tot_w = [], 0.0, 0.0, 0.0
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        calls = round(len(v) / per_fwd_ref, 2) if per_fwd_ref else None
        med = statistics.median(v) * 1e-9
        c = ctr.get(k, {})
        rd = statistics.median(c["FETCH_SIZE"]) * 2048 if c.get("FETCH_SIZE") else None
        wr = statistics.median(c["WRITE_SIZE"]) * 1024 if c.get("WRITE_SIZE") else None
        e = {"kernel": k, "per_forward": calls, "median_us": round(med * 1e6, 2)}
        if calls is not None and calls < 0.5:  # once per run, after the replays (the tool's own checks)
            e["outside_forward"] = True
            rows.append(e)
            continue
        if rd is not None and wr is not None:
            e.update({"hbm_read_MB": round(rd / 1e6, 3), "hbm_write_MB": round(wr / 1e6, 3),
                      "hbm_GBps": round((rd + wr) / med / 1e9, 1), "hbm_frac": round((rd + wr) / med / HBM_PEAK, 3)})
            if calls:
                tot_r += rd * calls
                tot_w += wr * calls
        if calls:
            tot_t += med * calls
        rows.append(e)
    print(json.dumps({"P": P, "n": n, "forwards_traced": forwards, "kernels": rows,
                      "per_forward": {"kernel_ms": round(tot_t * 1e3, 4), "hbm_read_MB": round(tot_r / 1e6, 2),
                                      "hbm_write_MB": round(tot_w / 1e6, 2),
                                      "avg_hbm_frac": round((tot_r + tot_w) / max(tot_t, 1e-12) / HBM_PEAK, 3)},
                      "how": "FETCH_SIZE x 2 + WRITE_SIZE (KB) per dispatch, medians; counter collection starts "
                             "each dispatch with a cold L2 (profiles/r02/l2_retention.txt), so these are upper "
                             "bounds on a graph replay's HBM traffic"}, indent=1))


if __name__ == "__main__":
    main()

"""Summarise a tools/pmc_passes.sh output directory for the main attention kernel.

    python tools/summarize_pmc.py gpurun_out/prof_<tag>_<workload> [kernel-substring]
Prints per-dispatch means of every counter, the derived ratios used in DESIGN.md, and the
HBM bytes per launch with the gfx950 FETCH_SIZE correction (x2, MI355X_MICROARCH.md §HBM)."""
import collections
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "fwd_kernel"
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "pmc_*", "*counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            if pat in row["Kernel_Name"]:
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in vals.items()}
    for k in sorted(m):
        print(f"{k:30s} {m[k]:.6g}  (n={len(vals[k])})")
    kt = {}
    for f in glob.glob(os.path.join(d, "kt", "*kernel_stats.csv")):
        for row in csv.DictReader(open(f)):
            if pat in row["Name"]:
                kt = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]), "min_ns": float(row["MinNs"])}
    out = {"kernel_trace": kt}
    if "SQ_WAVE_CYCLES" in m:
        wc = m["SQ_WAVE_CYCLES"]
        out["wait_any_frac"] = m.get("SQ_WAIT_ANY", 0) / wc
        out["wait_inst_any_frac"] = m.get("SQ_WAIT_INST_ANY", 0) / wc
        out["active_inst_any_frac"] = m.get("SQ_ACTIVE_INST_ANY", 0) / wc
    if "SQ_WAVES" in m:
        w = m["SQ_WAVES"]
        out["valu_insts_per_wave"] = m.get("SQ_INSTS_VALU", 0) / w
        out["mfma_insts_per_wave"] = m.get("SQ_INSTS_MFMA", 0) / w
        out["lds_insts_per_wave"] = m.get("SQ_INSTS_LDS", 0) / w
        out["salu_insts_per_wave"] = m.get("SQ_INSTS_SALU", 0) / w
    if "FETCH_SIZE" in m:
        out["hbm_read_bytes"] = m["FETCH_SIZE"] * 1024 * 2   # gfx950: FETCH_SIZE reads half of wide streams
    if "WRITE_SIZE" in m:
        out["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m and kt:
        # MFMA busy summed over all SIMDs vs (SIMDs x kernel cycles at the observed clock)
        out["mfma_busy_per_simd_cycles"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

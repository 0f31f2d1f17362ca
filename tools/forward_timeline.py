"""Timeline of the last graph-replayed forward in a rocprofv3 kernel trace of
tools/matcher_profile.py: each kernel's duration and the idle gap before it (dispatch-to-dispatch
seams inside the graph), summed by kernel family.

    python tools/forward_timeline.py <dir>/m_kernel_trace.csv [kernels per forward]

Without a count, one forward is cut at the assignment head's combine pass (its last kernel, once per forward)."""
import csv
import sys
import re
from collections import defaultdict


E3_NAMES = {"0": "", "1": " +split2", "2": " +qkv", "3": " +head"}


def family(name):
    n = name.removeprefix("void ").replace("(anonymous namespace)::", "").replace("mha_hd64::", "")
    for k in ("mha_hd64_stream_kernel", "mha_hd64_direct16_kernel", "mha_hd64_direct_kernel", "mha_hd64_fwd_kernel",
              "linear_tile_kernel", "linear_kernel", "linear_ln_kernel", "ffn_rows16_kernel", "ffn_rows_kernel",
              "assign_lse_kernel", "assign_close_kernel", "assign_combine_kernel", "ln_gelu", "lse16", "combine16",
              "pair_inputs", "Cijk"):
        if k in n:
            if k.startswith("linear") and k != "linear_ln_kernel":
                return n.split("(")[0]
            if k.startswith("ffn_rows"):  # the phase-3 kind: the E3 template argument (demangled or not)
                if k == "ffn_rows16_kernel":  # <D, E3, NB3(, SP)>
                    m = re.search(r"ffn_rows16_kernel<\d+, (\d+),", n) or re.search(r"ffn_rows16_kernelILi\d+ELi(\d+)E", n)
                else:  # <MB, D, E3, NB3>
                    m = re.search(r"ffn_rows_kernel<\d+, \d+, (\d+),", n) or re.search(r"ffn_rows_kernelILi\d+ELi\d+ELi(\d+)E", n)
                return k + (E3_NAMES.get(m.group(1), "") if m else "")
            return k
    return "FW " + n.split("(")[0][:60]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    per = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    if per:
        last = rows[-per:]
    else:  # one forward = the kernels after the second-to-last forward's last kernel (its combine pass)
        marks = [i for i, n in enumerate(names) if "assign_combine" in n or "combine16" in n]
        last = rows[marks[-2] + 1:marks[-1] + 1] if len(marks) >= 2 else rows
        per = len(last)
    t0 = int(last[0]["Start_Timestamp"])
    t1 = int(last[-1]["End_Timestamp"])
    busy = defaultdict(float)
    gaps = defaultdict(float)
    count = defaultdict(int)
    prev_end = None
    for r in last:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        f = family(r["Kernel_Name"])
        busy[f] += (e - s) / 1e3
        count[f] += 1
        if prev_end is not None:
            gaps[f] += max(0, s - prev_end) / 1e3
        prev_end = e
    print(f"kernels per forward {per}; forward {(t1 - t0) / 1e3:.1f} us; kernel time {sum(busy.values()):.1f} us; "
          f"gaps {sum(gaps.values()):.1f} us")
    for f in sorted(busy, key=lambda k: -busy[k]):
        print(f"{busy[f]:8.1f} us busy {gaps[f]:7.1f} us gap before  {count[f]:3d} x  {f}")


if __name__ == "__main__":
    main()

"""Per-forward kernel breakdown of a rocprofv3 kernel trace of tools/matcher_profile.py:

    python tools/trace_forward.py <dir>/m_kernel_stats.csv [attention launches per forward = 18]

Forwards = attention-kernel calls / 18 (two grouped launches per layer, 9 layers); prints us per
forward per kernel, our kernels vs framework (torch / hipBLASLt / runtime copy) launches."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
per = int(sys.argv[2]) if len(sys.argv) > 2 else 18
att = [r for r in rows if "mha_hd64_" in r["Name"] and "kernel" in r["Name"]]
nf = sum(int(r["Calls"]) for r in att) / per
ours = ("mha_hd64", "linear_", "lse", "combine", "pair_inputs", "ln_gelu", "merge", "split", "qkv_rotary")
tot = fw_t = fw_n = 0.0
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    us, calls = float(r["TotalDurationNs"]) / 1e3 / nf, int(r["Calls"]) / nf
    own = any(k in r["Name"] for k in ours)
    tot += us
    if not own:
        fw_t += us
        fw_n += calls
    print(f"{us:9.1f} us/fwd  {calls:6.1f} calls/fwd  avg {float(r['AverageNs']) / 1e3:8.2f} us  {'   ' if own else 'FW '}{r['Name'][:100]}")
print(f"forwards {nf:.1f}; total {tot:.1f} us per forward; framework launches {fw_n:.1f} per forward, {fw_t:.1f} us")

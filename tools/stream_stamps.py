"""Diagnostic: where a step of the persistent streaming kernel spends its cycles, from a
-DMHA_STREAM_STAMPS build (tools/build_stream_variant.sh stamps -DMHA_STREAM_STAMPS).
    [STREAM_WAVES=8] python tools/stream_stamps.py <lib.so> [batch] [nq] [nkv]
Per wave: s_memtime cycles per step by segment (refill issue, decision/seam, phase A issue,
phase B issue, DMA wait, barrier), medians and p90 over waves, steps per wave, the in-kernel clock
(s_memtime / s_memrealtime) and the share of a wave's life spent in steps."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

from lightglue_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
lib = _lib.load()
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
W = int(os.environ.get("STREAM_WAVES", "4"))  # forced plan 23 with kv_waves 4 / 8
nq = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
nkv = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
dev = torch.device("cuda:0")
q = torch.randn(B, 4, nq, 64, device=dev).half()
k = torch.randn(B, 4, nkv, 64, device=dev).half()
v = torch.randn(B, 4, nkv, 64, device=dev).half()
o = torch.empty_like(q)
ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
st = torch.zeros(512 * 8 * 48, dtype=torch.int64, device=dev)
lib.mha_hd64_set_stamp_buffer(st.data_ptr())
s = torch.cuda.current_stream().cuda_stream
for _ in range(20):
    assert lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, 4, nq, nkv, 0, 0, 23,
                                      W, 0, ws.data_ptr(), ws.numel(), s, 3) == 0
torch.cuda.synchronize()
items = B * 4 * -(-nq // (32 * W))
grid = min(items, 512 if W == 4 else 256)
t = st[: grid * W * 48].view(grid * W, 48).cpu().numpy().astype(np.float64)
# layout (csrc/mha_hd64_stream.hip, MHA_STREAM_STAMPS): 0 the first item's tile 0 (kernel
# prologue), 1 first steps, 2 middle loop, 3 tail + last steps + epilogues, 6 middle steps, 14
# items, 8..11 entry / exit clocks, 12 end of the kernel prologue's loads
items = np.maximum(t[:, 14], 1)
nmid = np.maximum(t[:, 6], 1)
out = {"batch": B, "nq": nq, "nkv": nkv, "grid": grid, "waves": W, "items_per_wave_med": float(np.median(t[:, 14])),
       "middle_steps_per_wave_med": float(np.median(t[:, 6]))}
out["first_tile0_cyc_med"] = round(float(np.median(t[:, 0])), 1)
out["first_step_cyc_med"] = round(float(np.median(t[:, 1] / items)), 1)
out["middle_step_cyc_med"] = round(float(np.median(t[:, 2] / nmid)), 1)
out["tail_last_epilogue_cyc_med"] = round(float(np.median(t[:, 3] / items)), 1)
life = t[:, 10] - t[:, 8]
real = (t[:, 11] - t[:, 9]) / 100.0  # us at 100 MHz
out["wave_life_cyc_med"] = float(np.median(life))
pro = t[:, 12] - t[:, 8]
out["kernel_prologue_cyc_med"] = float(np.median(pro))
acc = pro + t[:, 0] + t[:, 1] + t[:, 2] + t[:, 3]
out["accounted_frac_med"] = round(float(np.median(acc / np.maximum(life, 1))), 3)
out["middle_frac_med"] = round(float(np.median(t[:, 2] / np.maximum(life, 1))), 3)
out["clock_ghz_med"] = round(float(np.median(life / np.maximum(real, 1e-9) / 1e3)), 3)
out["kernel_span_us"] = round(float((t[:, 11].max() - t[:, 9].min()) / 100.0), 2)
# launch timeline on the global 100 MHz clock: when waves start and end relative to the first start
t0 = t[:, 9].min()
ent = (t[:, 9] - t0) / 100.0
ext = (t[:, 11] - t0) / 100.0
out["entry_us_p50_p90_max"] = [round(float(np.percentile(ent, q)), 2) for q in (50, 90, 100)]
out["exit_us_min_p10_p50_max"] = [round(float(np.percentile(ext, q)), 2) for q in (0, 10, 50, 100)]
out["wave_life_us_min_p50_max"] = [round(float(np.percentile(real, q)), 2) for q in (0, 50, 100)]
# by XCD (blockIdx % 8 under round-robin placement) and by half of the grid
wg = np.arange(grid * W) // W
clk = life / np.maximum(real, 1e-9) / 1e3
out["life_us_by_xcd"] = [round(float(np.median(real[wg % 8 == x])), 2) for x in range(8)]
out["clock_ghz_by_xcd"] = [round(float(np.median(clk[wg % 8 == x])), 3) for x in range(8)]
out["life_us_by_half"] = [round(float(np.median(real[wg < grid // 2])), 2), round(float(np.median(real[wg >= grid // 2])), 2)]
out["middle_cyc_by_xcd"] = [round(float(np.median((t[:, 2] / nmid)[wg % 8 == x])), 1) for x in range(8)]
# chained segments (cycles per item, per middle step)
names = ["item_advance", "next_q_issue", "first_A", "first_B", "first_epi_wait", "first_barrier", "mid_A", "mid_B",
         "mid_wait", "mid_barrier", "tail_A", "tail_B", "tail_wait", "tail_barrier", "to_last", "read_q", "last_A",
         "last_B", "last_wait", "last_barrier"]
seg = {}
for k, nm in enumerate(names):
    col = t[:, 16 + k]
    den = nmid if nm.startswith("mid") else items
    seg[nm] = round(float(np.median(col / den)), 1)
out["segments"] = seg
print(json.dumps(out))

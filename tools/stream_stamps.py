"""Diagnostic: where a step of the persistent streaming kernel spends its cycles, from a
-DMHA_STREAM_STAMPS build (tools/build_stream_variant.sh stamps -DMHA_STREAM_STAMPS).
    python tools/stream_stamps.py <lib.so> [batch] [nq] [nkv]
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
nq = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
nkv = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
dev = torch.device("cuda:0")
q = torch.randn(B, 4, nq, 64, device=dev).half()
k = torch.randn(B, 4, nkv, 64, device=dev).half()
v = torch.randn(B, 4, nkv, 64, device=dev).half()
o = torch.empty_like(q)
ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
st = torch.zeros(512 * 8 * 16, dtype=torch.int64, device=dev)
lib.mha_hd64_set_stamp_buffer(st.data_ptr())
s = torch.cuda.current_stream().cuda_stream
for _ in range(20):
    assert lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, 4, nq, nkv, 0, 0, 23,
                                      0, 0, ws.data_ptr(), ws.numel(), s, 3) == 0
torch.cuda.synchronize()
W = int(os.environ.get("MHA_HD64_STREAM_WAVES", "8"))
items = B * 4 * -(-nq // (32 * W))
grid = min(items, 512 if W == 4 else 256)
t = st[: grid * W * 16].view(grid * W, 16).cpu().numpy().astype(np.float64)
steps = t[:, 6]
per = t[:, :6] / np.maximum(steps, 1)[:, None]
names = ["refill_issue", "decision", "phaseA", "phaseB", "dma_wait", "barrier"]
out = {"batch": B, "nq": nq, "nkv": nkv, "grid": grid, "steps_per_wave_med": float(np.median(steps))}
for i, n in enumerate(names):
    out[n] = {"med": round(float(np.median(per[:, i])), 1), "p90": round(float(np.percentile(per[:, i], 90)), 1)}
out["step_total_med"] = round(float(np.median(per.sum(1))), 1)
life = t[:, 10] - t[:, 8]
real = (t[:, 11] - t[:, 9]) / 100.0  # us at 100 MHz
out["wave_life_cyc_med"] = float(np.median(life))
out["in_steps_frac_med"] = round(float(np.median(t[:, :6].sum(1) / np.maximum(life, 1))), 3)
out["clock_ghz_med"] = round(float(np.median(life / np.maximum(real, 1e-9) / 1e3)), 3)
out["prologue_cyc_med"] = float(np.median(t[:, 12] - t[:, 8]))
out["epilogues_cyc_med"] = float(np.median(t[:, 13]))
out["entry_spread_cyc"] = float(t[:, 8].max() - t[:, 8].min())
out["exit_spread_cyc"] = float(t[:, 10].max() - t[:, 10].min())
out["kernel_span_us"] = round(float((t[:, 11].max() - t[:, 9].min()) / 100.0), 2)
print(json.dumps(out))

"""Diagnostic: per-step phase cycles of the steady loop from a -DMHA_STEPSTAMPS build.
    python tools/stepstamps.py <lib.so> batch nq nkv q_waves kv_waves splits
Phases per full step (wave averages): A = refill issue -> last QK MFMA issued (phase A),
B = -> after PV / row max / LDS refill (phase B), C = barrier wait."""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

from lightglue_amd import _lib, synth  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
lib = _lib.load()
B, nq, nkv, qw, kw, sp = (int(x) for x in sys.argv[2:8])
dev = torch.device("cuda:0")
qn, kn, vn = synth.qkv(3, nq, nkv, batch=B)
q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in (qn, kn, vn))
o = torch.empty_like(q)
ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
st = torch.zeros((1 << 16) + (1 << 18), dtype=torch.int64, device=dev)
lib.mha_hd64_set_stamp_buffer(st.data_ptr())
s = torch.cuda.current_stream().cuda_stream
for _ in range(30):
    lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, 4, nq, nkv, 0, 0, qw, kw, sp,
                               ws.data_ptr(), ws.numel(), s, 1)
torch.cuda.synchronize()
rbw = 2 if qw >= 10 else 1
qw_ = qw - 10 if qw >= 10 else qw
nwg = (-(-nq // (32 * qw_ * rbw))) * B * 4 * sp
nw = qw_ * kw
t = st[(1 << 16):(1 << 16) + nwg * 8 * 4].view(nwg, 8, 4)[:, :nw, :].cpu().numpy().astype("int64")
cnt = t[:, :, 3] - 1  # first accumulation carries zero deltas
res = {"shape": [B, nq, nkv, qw, kw, sp], "steps_per_wave": int(statistics.median(cnt.ravel()))}
for i, name in enumerate("ABC"):
    per = t[:, :, i] / cnt.clip(min=1)
    res[f"{name}_cyc_med"] = round(float(statistics.median(per.ravel())), 1)
    res[f"{name}_cyc_max"] = round(float(per.max()), 1)
for w in range(nw):
    res[f"wave{w}"] = [round(float(statistics.median((t[:, w, i] / cnt[:, w].clip(min=1)).ravel())), 1) for i in range(3)]
print(json.dumps(res), flush=True)

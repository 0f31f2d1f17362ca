"""Diagnostic: per-workgroup phase timestamps from a -DMHA_STAMPS build.
    python tools/stamps.py <lib.so> batch nq nkv q_waves kv_waves splits [phase_mask]
Slots: 0 entry, 1 after prologue (Q + 2 K/V stages in LDS), 2 after the KV loop,
3 after the in-workgroup merge, 5 (in-launch combine) after the partial stores drained and the
ticket was drawn, 4 at the end (the last arriver's merged output stored). phase_mask 3 = the
production launch (in-launch combine when splitting), 1 = main kernel only."""
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
MASK = int(sys.argv[8]) if len(sys.argv) > 8 else 1
dev = torch.device("cuda:0")
qn, kn, vn = synth.qkv(3, nq, nkv, batch=B)
q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in (qn, kn, vn))
o = torch.empty_like(q)
ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
st = torch.zeros(1 << 20, dtype=torch.int64, device=dev)
lib.mha_hd64_set_stamp_buffer(st.data_ptr())
s = torch.cuda.current_stream().cuda_stream
for _ in range(20):  # warm (inputs resident, clocks up)
    lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, 4, nq, nkv, 0, 0, qw, kw, sp,
                               ws.data_ptr(), ws.numel(), s, MASK)
torch.cuda.synchronize()
nwg = (-(-nq // (32 * qw))) * B * 4 * sp
t = st[: nwg * 8].view(nwg, 8).cpu().numpy().astype("int64")
t0 = t[:, 0].min()
rel = (t[:, :6] - t0)
d = {"shape": [B, nq, nkv, qw, kw, sp], "wgs": nwg,
     "kernel_span_cyc": int(t[:, 4].max() - t0),
     "start_spread_cyc": int(t[:, 0].max() - t0)}
for i, name in enumerate(["prologue", "loop", "merge", "store"]):
    seg = t[:, i + 1] - t[:, i]
    d[name + "_med_cyc"] = int(statistics.median(seg))
    d[name + "_max_cyc"] = int(seg.max())
if MASK == 3 and sp > 1:  # in-launch combine: publish (stores drained + ticket), then last arrivers
    pub = t[:, 5] - t[:, 3]
    d["publish_med_cyc"] = int(statistics.median(pub))
    d["publish_max_cyc"] = int(pub.max())
    tail = t[:, 4] - t[:, 5]
    last = tail > statistics.median(tail) * 4 + 100
    d["last_arrivers"] = int(last.sum())
    if last.any():
        d["reduce_med_cyc_last"] = int(statistics.median(tail[last]))
        d["reduce_max_cyc_last"] = int(tail[last].max())
    d["end_of_last_arriver_med_cyc"] = int(statistics.median(rel[last, 4])) if last.any() else None
    d["slot5_minus_slot3"] = "stores + vmcnt(0) + barrier + ticket + barrier"
print(json.dumps(d))

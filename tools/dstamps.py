"""Diagnostic: phase timestamps of the single-pass kernel from a -DMHA_STAMPS build
(tools/build_direct_variant.sh stamps -DMHA_STAMPS).
    python tools/dstamps.py <lib.so> nq nkv [plan code: 21 (32-row kernel, default) | 22 (16-row)]
Slots (wave 0 of every workgroup, s_memtime cycles): 0 entry, 1 Q + K(0) landed, 2 scores and
probabilities of every tile done, 3 V(0) landed, 4 PV done, 5 after the epilogue barrier,
6 output stores acknowledged. Prints medians / maxima of each segment and of the start spread."""
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
nq, nkv = int(sys.argv[2]), int(sys.argv[3])
code = int(sys.argv[4]) if len(sys.argv) > 4 else 21
rows = 16 if code == 22 else 32
dev = torch.device("cuda:0")
qn, kn, vn = synth.qkv(3, nq, nkv)
q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in (qn, kn, vn))
o = torch.empty_like(q)
ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
st = torch.zeros(1 << 16, dtype=torch.int64, device=dev)
lib.mha_hd64_set_stamp_buffer(st.data_ptr())
s = torch.cuda.current_stream().cuda_stream
res = []
for rep in range(30):  # back-to-back launches (clocks up); keep the last
    lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), 1, 4, nq, nkv, 0, 0, code, 0, 0,
                               ws.data_ptr(), ws.numel(), s, 3)
torch.cuda.synchronize()
nwg = -(-nq // rows) * 4
t = st[: nwg * 8].view(nwg, 8).cpu().numpy().astype("int64")
t0 = t[:, 0].min()
d = {"nq": nq, "nkv": nkv, "wgs": nwg, "start_spread_cyc": int(t[:, 0].max() - t0),
     "span_cyc": int(t[:, 6].max() - t0)}
names = ["qk0_landed", "scores", "v0_landed", "pv", "epi_barrier", "merge_store"]
for i, n in enumerate(names):
    seg = t[:, i + 1] - t[:, i]
    d[n + "_med"] = int(statistics.median(seg))
    d[n + "_max"] = int(seg.max())
d["end_med_from_t0"] = int(statistics.median(t[:, 6] - t0))
if nkv > 1024 and code == 21:  # two-pass form: slot 7 = second pass starts (first pass's PVs done)
    d["pass1_start_med_from_t0"] = int(statistics.median(t[:, 7] - t0))
    d["pass1_med"] = int(statistics.median(t[:, 4] - t[:, 7]))
    d["v0_to_pass1_med"] = int(statistics.median(t[:, 7] - t[:, 3]))
print(json.dumps(d))

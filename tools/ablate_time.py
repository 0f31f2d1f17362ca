"""Diagnostic: time one library build (ablation variant) on fixed shapes.
    python tools/ablate_time.py <lib.so>"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from lightglue_amd import _lib, synth  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
lib = _lib.load()
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
res = {"lib": os.path.basename(sys.argv[1])}
for (qw, kw, batch, nkv) in ((4, 2, 32, 2048), (4, 1, 32, 2048), (4, 2, 32, 128)):
    nq = 1024
    qn, kn, vn = synth.qkv(3, nq, nkv, batch=batch)
    q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in (qn, kn, vn))
    o = torch.empty_like(q)

    def run():
        return lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), batch, 4, nq,
                                          nkv, 0, 0, qw, kw, 1, ws.data_ptr(), ws.numel(), stream.cuda_stream, 1)
    assert run() == 0
    t = statistics.median(bench.event_durations_ms(torch, run, 30, stream)[5:])
    res[f"{qw}x{kw}_B{batch}_kv{nkv}_us"] = round(t * 1e3, 2)
print(json.dumps(res), flush=True)

"""Diagnostic: per-launch time of a forced ring-kernel shape on batched 1024-row calls at two key
lengths (slope = steady-state cost per 64-key tile, intercept = fixed cost), for whichever
library MHA_HD64_LIB points at (ablation builds from tools/ablate_build.sh). One JSON line.
    MHA_HD64_LIB=... python tools/ablate_batched.py q_waves kv_waves tag"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from lightglue_amd import _lib, synth  # noqa: E402

lib = _lib.load()
qw, kw, tag = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
res = {"tag": tag, "shape": [qw, kw]}
for batch in (8, 16):
    for nkv in (1024, 2048):
        qn, kn, vn = synth.qkv(3, 1024, nkv, batch=batch)
        q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in (qn, kn, vn))
        o = torch.empty_like(q)

        def run():
            return lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), batch, 4, 1024,
                                              nkv, 0, 0, qw, kw, 1, ws.data_ptr(), ws.numel(), stream.cuda_stream, 1)
        assert run() == 0, _lib.last_error()
        res[f"b{batch}_k{nkv}"] = round(bench.graph_per_launch_ms(torch, run, stream, k=100, reps=3) * 1e3, 2)
print(json.dumps(res), flush=True)

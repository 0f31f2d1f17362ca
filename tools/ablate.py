"""Diagnostic: main-kernel time vs key length / batch for one workgroup shape (slope = cost per
key tile, intercept = fixed prologue/epilogue cost). Prints one JSON line per point.
    python tools/ablate.py q_waves kv_waves [splits]"""
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
qw, kw = int(sys.argv[1]), int(sys.argv[2])
sp = int(sys.argv[3]) if len(sys.argv) > 3 else 1
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
ws = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
for batch, nq in ((8, 1024), (16, 1024), (32, 1024)):
    for nkv in (128, 512, 1024, 2048, 4096):
        qn, kn, vn = synth.qkv(3, nq, nkv, batch=batch)
        q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in (qn, kn, vn))
        o = torch.empty_like(q)

        def run():
            return lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), batch, 4, nq,
                                              nkv, 0, 0, qw, kw, sp, ws.data_ptr(), ws.numel(), stream.cuda_stream, 1)
        assert run() == 0, _lib.last_error()
        t = statistics.median(bench.event_durations_ms(torch, run, 40, stream)[5:])
        fl = bench.call_flops(batch, 4, nq, nkv)
        print(json.dumps({"batch": batch, "nq": nq, "nkv": nkv, "us": round(t * 1e3, 2),
                          "tflops": round(fl / (t * 1e-3) / 1e12, 1)}), flush=True)
# event overhead reference: an empty-ish launch
t0 = statistics.median(bench.event_durations_ms(torch, lambda: torch.cuda._sleep(1), 40, stream)[5:])
print(json.dumps({"event_overhead_us": round(t0 * 1e3, 2)}))

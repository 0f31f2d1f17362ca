"""Saturated-launch sweep: per-launch graph-replay time of batched B x 4 x Nq x Nkv fp16 launches
under forced plans (ring (4,2), ring (4,1), 0 = planner).
One JSON line per case.
    python tools/tput_sweep.py [BxN[xNKV] ...]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from lightglue_amd import _lib, synth  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
cases = [tuple(int(x) for x in c.split("x")) for c in sys.argv[1:]] or [(8, 1024), (16, 1024), (32, 1024), (2, 2048),
                                                                      (4, 2048), (4, 512), (16, 512)]
for case in cases:
    b, nq = case[0], case[1]
    nkv = case[2] if len(case) > 2 else nq
    qn, kn, vn = synth.qkv(3, nq, nkv, batch=b)
    q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in (qn, kn, vn))
    o = torch.empty_like(q)
    fl = bench.call_flops(b, 4, nq, nkv)
    row = {"case": f"{b}x4x{nq}x{nkv}"}
    # warm the clocks first (DVFS: the first plan timed after an idle gap otherwise reads slow),
    # then every plan, the planner's again last
    warm = lambda: lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), b, 4, nq,  # noqa
                                              nkv, 0, 0, 0, 0, 0, ws.data_ptr(), ws.numel(), stream.cuda_stream, 3)
    bench.graph_per_launch_ms(torch, warm, stream, k=400, reps=5)
    shapes = [("planner_first", 0, 0), ("ring42", 4, 2), ("ring41", 4, 1)]
    # EXTRA_SHAPES="q-k,...": forced (q_waves, kv_waves) codes, e.g. 12-2 = (2,2) with 64-row waves
    shapes += [(f"ring{x}", int(x.split("-")[0]), int(x.split("-")[1]))
               for x in os.environ.get("EXTRA_SHAPES", "").split(",") if x]
    for name, qw, kw in shapes + [("planner", 0, 0)]:
        def run():
            return lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), b, 4, nq, nkv,
                                              0, 0, qw, kw, 1 if qw else 0, ws.data_ptr(), ws.numel(),
                                              stream.cuda_stream, 3)
        if run() != 0:
            row[name] = None
            continue
        us = bench.graph_per_launch_ms(torch, run, stream, k=100, reps=3) * 1e3
        row[name] = {"us": round(us, 2), "frac": round(fl / (us * 1e-6) / 1e12 / bench.PEAK_F16_TFLOPS, 4)}
    print(json.dumps(row), flush=True)

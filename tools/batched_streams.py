"""Saturated throughput with launch overlap: S streams, each replaying a graph of L back-to-back
batched launches (B calls of 1x4xNxN fp16 per launch, the planner's plan), all streams at once.
Whole-GPU calls/s and fraction of the 2.5 PFLOP/s fp16 peak. One JSON line per (B, S).
    python tools/batched_streams.py [N]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import lightglue_amd  # noqa: E402
from lightglue_amd import synth  # noqa: E402

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
L = 20
for B in (8, 16, 32):
    for S in (1, 2, 3):
        streams = [torch.cuda.Stream(dev) for _ in range(S)]
        graphs = []
        for i, st in enumerate(streams):
            q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in synth.qkv(50 + i, n, n, batch=B))
            o = torch.empty_like(q)
            with torch.cuda.stream(st):
                lightglue_amd.mha_hd64_batched(q, k, v, out=o)
                st.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=st):
                    for _ in range(L):
                        lightglue_amd.mha_hd64_batched(q, k, v, out=o)
            graphs.append((g, st, q, k, v, o))
        for g, st, *_ in graphs:
            with torch.cuda.stream(st):
                g.replay()
        torch.cuda.synchronize()
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            for g, st, *_ in graphs:
                with torch.cuda.stream(st):
                    g.replay()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        calls = S * L * B
        fl = calls * bench.call_flops(1, 4, n, n)
        print(json.dumps({"B": B, "streams": S, "launches_per_stream": L, "calls_per_s": round(calls / best, 1),
                          "tflops": round(fl / best / 1e12, 1),
                          "frac": round(fl / best / 1e12 / bench.PEAK_F16_TFLOPS, 4)}), flush=True)
        del graphs

"""Where the fixed per-replay cost of a short K-step timed region comes from: K calls timed by one
event pair, submitted (a) as a graph replay, (b) eagerly, both behind a sleep kernel; and event
pairs with nothing between them."""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import lightglue_amd  # noqa: E402
from lightglue_amd import synth  # noqa: E402

dev = torch.device("cuda:0")
q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in synth.qkv(1, 1024, 1024))
o = torch.empty_like(q)
st = torch.cuda.Stream(dev)
with torch.cuda.stream(st):
    for _ in range(20):
        lightglue_amd.mha_hd64(q, k, v, out=o)
st.synchronize()


def run(K, R, mode):
    g = None
    if mode == "graph":
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for _ in range(K):
                lightglue_amd.mha_hd64(q, k, v, out=o)
        g.replay()
        st.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(R)]
    with torch.cuda.stream(st):
        torch.cuda._sleep(int(3e8))
        for a, b in ev:
            a.record(st)
            if mode == "graph":
                g.replay()
            elif mode == "eager":
                for _ in range(K):
                    lightglue_amd.mha_hd64(q, k, v, out=o)
            b.record(st)
    st.synchronize()
    t = [a.elapsed_time(b) * 1e3 for a, b in ev]
    return statistics.median(t)


for mode in ("none", "eager", "graph"):
    for K in (1, 20, 200):
        if mode == "none" and K > 1:
            continue
        us = run(K, 50, mode)
        print(f"{mode:6s} K={K:4d}: median {us:9.2f} us per event pair, {us / K:7.3f} us per call", flush=True)


def run_block(K, R):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        for _ in range(K):
            lightglue_amd.mha_hd64(q, k, v, out=o)
    g.replay()
    st.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        torch.cuda._sleep(int(3e8))
        a.record(st)
        for _ in range(R):
            g.replay()
        b.record(st)
    st.synchronize()
    return a.elapsed_time(b) * 1e3 / R


for K in (1, 20, 200):
    us = run_block(K, 100)
    print(f"block  K={K:4d}: {us:9.2f} us per replay (100 replays in one event pair), {us / K:7.3f} us per call",
          flush=True)

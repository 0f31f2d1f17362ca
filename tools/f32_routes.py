"""Float path (fp32 Q/K/V -> fp32 O) routes per shape, timed in graphs of back-to-back launches:
'grouped' = mha_hd64_grouped with the typed workspace (the planner's convert launch + fp16
single-pass kernel where those apply, or the in-kernel rounding of the 16-row one-pass forms);
'batched' = mha_hd64_batched with the fp16-sized workspace (no room for converted copies: the
ring kernel rounding fp32 on load, unless the 16-row one-pass form takes it in-kernel).
    python tools/f32_routes.py BxNQ-NKV ..."""
import hashlib
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

import lightglue_amd  # noqa: E402
from lightglue_amd import synth  # noqa: E402


def per_launch_us(fn, stream, k=200, reps=5):
    with torch.cuda.stream(stream):
        fn()
    stream.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        for _ in range(k):
            fn()
    g.replay()
    stream.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            e0.record(stream)
            g.replay()
            e1.record(stream)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / k)
    return statistics.median(ts)


def main():
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    for s in sys.argv[1:]:
        b, _, rest = s.rpartition("x")
        b = int(b or 1)
        nq, nkv = (int(x) for x in rest.split("-"))
        q, k, v = (torch.from_numpy(x).to(dev).float().contiguous() for x in synth.qkv(100, nq, nkv, batch=b))
        ref = torch.softmax((q @ k.transpose(-1, -2)) * 0.125, -1) @ v
        o1, o2 = torch.empty_like(q), torch.empty_like(q)
        row = {"batch": b, "nq": nq, "nkv": nkv}
        for name, fn, o in (("grouped", lambda: lightglue_amd.mha_hd64_grouped([(q, k, v)], outs=[o1]), o1),
                            ("batched", lambda: lightglue_amd.mha_hd64_batched(q, k, v, out=o2), o2)):
            us = per_launch_us(fn, stream)
            torch.cuda.synchronize()
            row[name] = {"us": round(us, 3), "max_abs": float((o - ref).abs().max()),
                         "digest": hashlib.sha256(o.cpu().numpy().tobytes()).hexdigest()[:12]}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

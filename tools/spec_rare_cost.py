"""Diagnostic: what the streaming kernel's speculative max costs when its rare path runs. B calls of
1x4x1024^2 per launch (forced plan 23, both forms), three inputs: random (no item overflows), one
spike (every head's query rows 5 and 645 meet a key row scaled by `gain`: 1 or 2 of a head's items
recomputed), all items (a spike key for one query row of every 128-row block: every item
recomputed); each library in the list timed by graph replay, interleaved, median us per launch.

    python tools/spec_rare_cost.py lib_a.so[,lib_b.so] [B=32] [gain=6]
"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tools"), os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

from stream_check import STREAM, forced, load  # noqa: E402


def main():
    libs = [load(p) for p in sys.argv[1].split(",")]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    gain = float(sys.argv[3]) if len(sys.argv) > 3 else 6.0
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream()
    ws = torch.empty(5242880, dtype=torch.uint8, device=dev)
    g = torch.Generator(device="cpu").manual_seed(5)
    q = torch.randn(B, 4, 1024, 64, generator=g)
    k = torch.randn(B, 4, 1024, 64, generator=g)
    v = torch.randn(B, 4, 1024, 64, generator=g)
    cases = {"random": k.clone(), "one_spike": k.clone(), "all_items": k.clone()}
    cases["one_spike"][:, :, 900] = q[:, :, 5] * gain
    cases["one_spike"][:, :, 300] = q[:, :, 645] * gain
    for i in range(8):
        cases["all_items"][:, :, 700 + 37 * i] = q[:, :, 128 * i + 9] * gain
    qd, vd = q.half().to(dev), v.half().to(dev)
    K = 20
    graphs, outs = {}, {}
    for li, lib in enumerate(libs):
        for w in (4, 8):
            for name, kk in cases.items():
                kd = kk.half().to(dev)
                o = torch.empty_like(qd)
                with torch.cuda.stream(stream):
                    forced(lib, qd, kd, vd, o, STREAM, ws, stream, w)
                    gr = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gr, stream=stream):
                        for _ in range(K):
                            forced(lib, qd, kd, vd, o, STREAM, ws, stream, w)
                graphs[(li, w, name)] = gr
                outs[(li, w, name)] = (kd, o)
    torch.cuda.synchronize()
    times = {key: [] for key in graphs}
    for _ in range(5):
        for key, gr in graphs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(stream):
                e0.record(stream)
                gr.replay()
                e1.record(stream)
            e1.synchronize()
            times[key].append(e0.elapsed_time(e1) * 1e3 / K)
    for (li, w, name), ts in times.items():
        kd, o = outs[(li, w, name)]
        ref = torch.softmax((qd[:2].float() @ kd[:2].float().transpose(-1, -2)) * 0.125, -1) @ vd[:2].float()
        err = float((o[:2].float() - ref).abs().max())
        print(json.dumps({"lib": li, "waves": w, "input": name, "calls": B, "us_per_launch": round(statistics.median(ts), 3),
                          "max_abs_vs_fp32_first2": err}), flush=True)


if __name__ == "__main__":
    main()

"""Diagnostic: whole fp16 matcher forwards at P pairs of 1024 keypoints with the projections' tile
form forced (lg_linear_set_wide(mode) for each mode listed) against the default (by size, -1);
graph replay, interleaved, median ms per forward.

    python tools/form_fwd_ab.py [P list, default 4,8,16,32] [modes, default 1]
"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

from lightglue_amd import _lib  # noqa: E402
from lightglue_amd import matcher as mt  # noqa: E402


def main():
    Ps = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [4, 8, 16, 32]
    modes = [-1] + ([int(c) for c in sys.argv[2]] if len(sys.argv) > 2 else [1])
    lib = _lib.load()
    dev, dt, n = torch.device("cuda:0"), torch.float16, 1024
    st = torch.cuda.Stream(dev)
    model = mt.LightGlueMatcher(n_layers=9).eval()
    model.load_state_dict(mt.seeded_state_dict(7, 9), strict=True)
    model = model.to(dev, dt)
    with torch.no_grad():
        for P in Ps:
            ps = [mt.synthetic_pair(80 + i, n, n) for i in range(P)]
            pair = tuple(torch.cat([p[j] for p in ps], 0).to(dev, dt) for j in range(4))
            graphs, outs = {}, {}
            for mode in modes:
                prev = lib.lg_linear_set_wide(mode)
                with torch.cuda.stream(st):
                    for _ in range(2):
                        outs[mode] = model(*pair)
                    st.synchronize()
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=st):
                        model(*pair)
                graphs[mode] = g
                lib.lg_linear_set_wide(prev)
            torch.cuda.synchronize()
            times = {m: [] for m in modes}
            for _ in range(21):
                for m, g in graphs.items():
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    with torch.cuda.stream(st):
                        e0.record(st)
                        g.replay()
                        e1.record(st)
                    e1.synchronize()
                    times[m].append(e0.elapsed_time(e1))
            same = all(torch.equal(a, b) for m in modes for a, b in zip(outs[-1], outs[m]))
            print(json.dumps({"P": P, "n": n, "ms": {("default" if m < 0 else f"form{m}"): round(statistics.median(t), 4) for m, t in times.items()},
                              "pairs_per_s": {("default" if m < 0 else f"form{m}"): round(P * 1e3 / statistics.median(t), 1) for m, t in times.items()},
                              "outputs_bitwise_equal": same}), flush=True)


if __name__ == "__main__":
    main()

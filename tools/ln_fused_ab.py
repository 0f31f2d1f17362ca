"""Diagnostic: lg_linear_cat_ln_gelu as one launch (linear_ln_kernel, lg_linear_set_ln_fused(1)) vs
two (lg_linear_cat + lg_layernorm_gelu), by size: the op alone at P pairs of n keypoints (graph of
back-to-back calls, interleaved), then whole fp16 matcher forwards at P = 1 (graph replay).

    python tools/ln_fused_ab.py [n=1024] [forward cases PxN,PxN... (default 1x512,1x1024,1x2048)]
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


def graph_us(fn, st, k=20, rounds=7):
    with torch.cuda.stream(st):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for _ in range(k):
                fn()
    return g


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    lib = _lib.load()
    dev, dt, h = torch.device("cuda:0"), torch.float16, 4
    st = torch.cuda.Stream(dev)
    K = 20
    for P in (1, 2, 4, 8, 16, 32):
        M = P * 2 * n
        x = torch.randn(1, M, 256, device=dev, dtype=dt) * 0.5
        c0 = torch.randn(P, h, n, 64, device=dev, dtype=dt)
        c1 = torch.randn(P, h, n, 64, device=dev, dtype=dt)
        w, b = torch.randn(512, 512, device=dev, dtype=dt) * 0.05, torch.randn(512, device=dev, dtype=dt)
        ln = torch.nn.LayerNorm(512).to(dev, dt)
        graphs, outs = {}, {}
        for mode in (0, 2):
            prev = lib.lg_linear_set_ln_fused(mode)
            graphs[mode] = graph_us(lambda: mt._Hip.linear_cat_ln_gelu(x, c0, c1, w, b, ln), st, K)
            outs[mode] = mt._Hip.linear_cat_ln_gelu(x, c0, c1, w, b, ln)
            lib.lg_linear_set_ln_fused(prev)
        torch.cuda.synchronize()
        times = {m: [] for m in graphs}
        for _ in range(7):
            for m, g in graphs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(st):
                    e0.record(st)
                    g.replay()
                    e1.record(st)
                e1.synchronize()
                times[m].append(e0.elapsed_time(e1) * 1e3 / K)
        d = float((outs[0].float() - outs[2].float()).abs().max())
        print(json.dumps({"op": "linear_cat_ln_gelu", "P": P, "n": n, "M": M,
                          "two_launch_us": round(statistics.median(times[0]), 2),
                          "one_launch_us": round(statistics.median(times[2]), 2), "max_diff": d}), flush=True)

    model = mt.LightGlueMatcher(n_layers=9).eval()
    model.load_state_dict(mt.seeded_state_dict(7, 9), strict=True)
    model = model.to(dev, dt)
    cases = [(1, 512), (1, 1024), (1, 2048)] if len(sys.argv) < 3 else [tuple(map(int, c.split("x"))) for c in sys.argv[2].split(",")]
    for P, nn in cases:
        ps = [mt.synthetic_pair(80 + i, nn, nn) for i in range(P)]
        pair = tuple(torch.cat([p[j] for p in ps], 0).to(dev, dt) for j in range(4))
        res = {}
        for mode in (0, 2, 0, 2):
            prev = lib.lg_linear_set_ln_fused(mode)
            with torch.no_grad(), torch.cuda.stream(st):
                for _ in range(2):
                    model(*pair)
                st.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=st):
                    model(*pair)
            lib.lg_linear_set_ln_fused(prev)
            g.replay()
            st.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            with torch.cuda.stream(st):
                for _ in range(20):
                    g.replay()
            e1.record(st)
            st.synchronize()
            res.setdefault(mode, []).append(round(e0.elapsed_time(e1) / 20, 4))
        print(json.dumps({"forward": f"P={P}", "n": nn, "ms_two_launch": res[0], "ms_one_launch": res[2],
                          "pairs_per_s_two": round(P * 1e3 / min(res[0]), 1), "pairs_per_s_one": round(P * 1e3 / min(res[2]), 1)}), flush=True)


if __name__ == "__main__":
    main()

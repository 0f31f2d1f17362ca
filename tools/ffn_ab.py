"""A/B timing of lg_linear_cat_ffn's forms (lg_linear_set_ffn_fused: 0 its two calls, 1 the one-launch
form by size, 2 ffn_rows_kernel (32 / 64 rows), 3 ffn_rows16_kernel) — the op alone at P pairs of
n keypoints (a graph of back-to-back calls per form, replays interleaved), then whole fp16 matcher
forwards (graph replay, interleaved), with the max |difference| of each form's outputs from the first.

    python tools/ffn_ab.py [--modes 0,2] [--ops 1x512,1x1024,1x2048,4x1024] [--forwards 1x512,1x1024]
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

from lightglue_amd import _lib  # noqa: E402
from lightglue_amd import matcher as mt  # noqa: E402


def replay_ms(graphs, st, reps, rounds=7):
    times = {k: [] for k in graphs}
    for _ in range(rounds):
        for k, g in graphs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(st):
                e0.record(st)
                g.replay()
                e1.record(st)
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / reps)
    return {k: statistics.median(v) for k, v in times.items()}


def sizes(s):
    return [tuple(int(v) for v in t.split("x")) for t in s.split(",") if t]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="0,1")
    ap.add_argument("--ops", default="1x512,1x1024,1x2048,2x1024,4x1024,8x1024")
    ap.add_argument("--forwards", default="1x512,1x1024,1x2048,4x1024")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--chains", default=None, help="A/B of the chained forward's fused projections (LG_CHAIN values, "
                    "comma-separated, e.g. 'sqh,sh,'): forwards only, against the first")
    a = ap.parse_args()
    modes = [int(m) for m in a.modes.split(",")]
    lib = _lib.load()
    dev, dt, h = torch.device("cuda:0"), torch.float16, 4
    st = torch.cuda.Stream(dev)
    K = a.reps
    with torch.no_grad():
        for P, n in sizes(a.ops):
            M = P * 2 * n
            gen = torch.Generator().manual_seed(P * 7 + n)
            rnd = lambda *s: torch.randn(*s, generator=gen).to(dev, dt)  # noqa: E731
            x = rnd(1, M, 256) * 0.5
            c0, c1 = rnd(P, h, n, 64), rnd(P, h, n, 64)
            w, b = rnd(512, 512) * 0.05, rnd(512) * 0.1
            w2, b2 = rnd(256, 512) * 0.05, rnd(256) * 0.1
            ln = torch.nn.LayerNorm(512).to(dev, dt)
            wp = mt.ffn_pack(w, w2)
            graphs, outs = {}, {}
            for mode in modes:
                prev = lib.lg_linear_set_ffn_fused(mode)
                with torch.cuda.stream(st):
                    outs[mode] = mt._Hip.ffn(x, c0, c1, w, b, ln, w2, b2, wp)
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=st):
                        for _ in range(K):
                            mt._Hip.ffn(x, c0, c1, w, b, ln, w2, b2, wp)
                graphs[mode] = g
                lib.lg_linear_set_ffn_fused(prev)
            torch.cuda.synchronize()
            t = replay_ms(graphs, st, K)
            o0 = outs[modes[0]].float()
            print(json.dumps({"op": "ffn", "P": P, "n": n, "M": M, "us": {str(m): round(t[m] * 1e3, 2) for m in modes},
                              "max_abs_vs_first": {str(m): float((outs[m].float() - o0).abs().max()) for m in modes}}),
                  flush=True)
            del graphs

        model = mt.LightGlueMatcher(n_layers=9).eval()
        if a.chains is not None:
            return chain_ab(a, model, dev, dt, st)
        model.load_state_dict(mt.seeded_state_dict(7, 9), strict=True)
        model = model.to(dev, dt)
        for P, n in sizes(a.forwards):
            ps = [mt.synthetic_pair(80 + i, n, n) for i in range(P)]
            pair = tuple(torch.cat([p[j] for p in ps], 0).to(dev, dt) for j in range(4))
            graphs, res = {}, {}
            for mode in modes:
                prev = lib.lg_linear_set_ffn_fused(mode)
                with torch.cuda.stream(st):
                    for _ in range(2):
                        res[mode] = model(*pair)
                    st.synchronize()
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=st):
                        model(*pair)
                graphs[mode] = g
                lib.lg_linear_set_ffn_fused(prev)
            torch.cuda.synchronize()
            t = replay_ms(graphs, st, 1, rounds=21)
            r0 = res[modes[0]]
            print(json.dumps({"forward": f"P={P}", "n": n, "ms": {str(m): round(t[m], 4) for m in modes},
                              "pairs_per_s": {str(m): round(P * 1e3 / t[m], 1) for m in modes},
                              "desc_max_abs_vs_first": {str(m): float((res[m][0].float() - r0[0].float()).abs().max()) for m in modes},
                              "scores_max_abs_vs_first": {str(m): float((res[m][2] - r0[2]).abs().max()) for m in modes}}),
                  flush=True)
            del graphs


def chain_ab(a, model, dev, dt, st):
    model.load_state_dict(mt.seeded_state_dict(7, 9), strict=True)
    model = model.to(dev, dt)
    chains = a.chains.split(",")
    for P, n in sizes(a.forwards):
        ps = [mt.synthetic_pair(80 + i, n, n) for i in range(P)]
        pair = tuple(torch.cat([p[j] for p in ps], 0).to(dev, dt) for j in range(4))
        graphs, res = {}, {}
        for c in chains:
            model.chain_kinds = c
            with torch.cuda.stream(st):
                for _ in range(2):
                    res[c] = model(*pair)
                st.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=st):
                    model(*pair)
            graphs[c] = g
        model.chain_kinds = None
        torch.cuda.synchronize()
        t = replay_ms(graphs, st, 1, rounds=21)
        r0 = res[chains[0]]
        print(json.dumps({"forward": f"P={P}", "n": n, "ms": {c: round(t[c], 4) for c in chains},
                          "same_as_first": {c: all(torch.equal(u, w) for u, w in zip(res[c], r0)) for c in chains}}),
              flush=True)
        del graphs


if __name__ == "__main__":
    main()

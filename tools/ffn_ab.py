"""Diagnostic: the whole FFN in one launch (lg_linear_cat_ffn's ffn_kernel, lg_linear_set_ffn_fused(1))
against its two calls (lg_linear_cat_ln_gelu + lg_linear(res = x), lg_linear_set_ffn_fused(0)): the op
alone at P pairs of 1024 keypoints (graph of back-to-back calls, interleaved), then whole fp16 matcher
forwards at P = 8 / 16 / 32 (graph replay, interleaved).

    python tools/ffn_ab.py [lib_a.so,lib_b.so,...   (the op alone through each library: ablation builds)]
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


def op_libs(paths):
    """The op alone at P = 16 / 32 through each library (ablation builds), interleaved."""
    import ctypes
    libs = []
    for path in paths:
        lib = ctypes.CDLL(os.path.abspath(path))
        for name, (args, res) in list(_lib.SIGNATURES.items()) + list(_lib.HOOKS.items()):
            if hasattr(lib, name):
                getattr(lib, name).argtypes, getattr(lib, name).restype = args, res
        libs.append(lib)
    dev, dt, h, n = torch.device("cuda:0"), torch.float16, 4, 1024
    st = torch.cuda.Stream(dev)
    K = 20
    for P in (16, 32):
        M = P * 2 * n
        x = torch.randn(1, M, 256, device=dev, dtype=dt) * 0.5
        c0 = torch.randn(P, h, n, 64, device=dev, dtype=dt)
        c1 = torch.randn(P, h, n, 64, device=dev, dtype=dt)
        w, b = torch.randn(512, 512, device=dev, dtype=dt) * 0.05, torch.randn(512, device=dev, dtype=dt)
        w2, b2 = torch.randn(256, 512, device=dev, dtype=dt) * 0.05, torch.randn(256, device=dev, dtype=dt)
        g_, be = torch.ones(512, device=dev, dtype=dt), torch.zeros(512, device=dev, dtype=dt)
        hb = torch.empty(1, M, 512, device=dev, dtype=dt)
        out = torch.empty(1, M, 256, device=dev, dtype=dt)
        graphs = {}
        for i, lib in enumerate(libs):
            call = lambda lib=lib: lib.lg_linear_cat_ffn(x.data_ptr(), c0.data_ptr(), c1.data_ptr(), h, n, n, P, w.data_ptr(),  # noqa: E731
                                                         b.data_ptr(), g_.data_ptr(), be.data_ptr(), 1e-5, w2.data_ptr(),
                                                         b2.data_ptr(), hb.data_ptr(), out.data_ptr(), st.cuda_stream)
            with torch.cuda.stream(st):
                assert call() == 0
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=st):
                    for _ in range(K):
                        call()
            graphs[os.path.basename(paths[i])] = g
        torch.cuda.synchronize()
        t = replay_ms(graphs, st, K)
        print(json.dumps({"op": "ffn", "P": P, "us": {k: round(v * 1e3, 2) for k, v in t.items()}}), flush=True)


def main():
    if len(sys.argv) > 1:
        return op_libs(sys.argv[1].split(","))
    lib = _lib.load()
    dev, dt, h, n = torch.device("cuda:0"), torch.float16, 4, 1024
    st = torch.cuda.Stream(dev)
    K = 20
    with torch.no_grad():
        for P in (16, 32):
            M = P * 2 * n
            x = torch.randn(1, M, 256, device=dev, dtype=dt) * 0.5
            c0 = torch.randn(P, h, n, 64, device=dev, dtype=dt)
            c1 = torch.randn(P, h, n, 64, device=dev, dtype=dt)
            w, b = torch.randn(512, 512, device=dev, dtype=dt) * 0.05, torch.randn(512, device=dev, dtype=dt)
            w2, b2 = torch.randn(256, 512, device=dev, dtype=dt) * 0.05, torch.randn(256, device=dev, dtype=dt)
            ln = torch.nn.LayerNorm(512).to(dev, dt)
            graphs, outs = {}, {}
            for mode in (0, 1):
                prev = lib.lg_linear_set_ffn_fused(mode)
                with torch.cuda.stream(st):
                    outs[mode] = mt._Hip.ffn(x, c0, c1, w, b, ln, w2, b2)
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=st):
                        for _ in range(K):
                            mt._Hip.ffn(x, c0, c1, w, b, ln, w2, b2)
                graphs[mode] = g
                lib.lg_linear_set_ffn_fused(prev)
            torch.cuda.synchronize()
            t = replay_ms(graphs, st, K)
            print(json.dumps({"op": "ffn", "P": P, "M": M, "two_calls_us": round(t[0] * 1e3, 2), "one_launch_us": round(t[1] * 1e3, 2),
                              "bitwise_equal": bool(torch.equal(outs[0], outs[1]))}), flush=True)

        model = mt.LightGlueMatcher(n_layers=9).eval()
        model.load_state_dict(mt.seeded_state_dict(7, 9), strict=True)
        model = model.to(dev, dt)
        for P in (8, 16, 32):
            ps = [mt.synthetic_pair(80 + i, n, n) for i in range(P)]
            pair = tuple(torch.cat([p[j] for p in ps], 0).to(dev, dt) for j in range(4))
            graphs, res = {}, {}
            for mode in (0, 1):
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
            same = all(torch.equal(a, b) for a, b in zip(res[0], res[1]) if torch.is_tensor(a))
            print(json.dumps({"forward": f"P={P}", "n": n, "ms_two_calls": round(t[0], 4), "ms_one_launch": round(t[1], 4),
                              "pairs_per_s_two": round(P * 1e3 / t[0], 1), "pairs_per_s_one": round(P * 1e3 / t[1], 1),
                              "outputs_bitwise_equal": same}), flush=True)


if __name__ == "__main__":
    main()

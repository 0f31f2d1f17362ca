"""Diagnostic: lg_linear_cat_ln_gelu (the FFN's Linear -> LayerNorm -> GELU) through several library
builds (A/B forms), the op alone at P pairs of 1024 keypoints, graph replay interleaved.

    python tools/ln_lib_ab.py lib_a.so,lib_b.so [P list, default 16,32]
"""
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

from lightglue_amd import _lib  # noqa: E402


def main():
    paths = sys.argv[1].split(",")
    Ps = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [16, 32]
    libs = []
    for path in paths:
        lib = ctypes.CDLL(os.path.abspath(path))
        for name, (args, res) in list(_lib.SIGNATURES.items()) + list(_lib.HOOKS.items()):
            if hasattr(lib, name):
                getattr(lib, name).argtypes, getattr(lib, name).restype = args, res
        libs.append(lib)
    dev, dt, h, n, K = torch.device("cuda:0"), torch.float16, 4, 1024, 20
    st = torch.cuda.Stream(dev)
    for P in Ps:
        M = P * 2 * n
        x = torch.randn(1, M, 256, device=dev, dtype=dt) * 0.5
        c0 = torch.randn(P, h, n, 64, device=dev, dtype=dt)
        c1 = torch.randn(P, h, n, 64, device=dev, dtype=dt)
        w, b = torch.randn(512, 512, device=dev, dtype=dt) * 0.05, torch.randn(512, device=dev, dtype=dt)
        g_, be = 1 + 0.1 * torch.randn(512, device=dev, dtype=dt), 0.1 * torch.randn(512, device=dev, dtype=dt)
        outs = [torch.empty(1, M, 512, device=dev, dtype=dt) for _ in libs]
        graphs = {}
        for i, lib in enumerate(libs):
            call = lambda lib=lib, o=outs[i]: lib.lg_linear_cat_ln_gelu(x.data_ptr(), c0.data_ptr(), c1.data_ptr(), h, n, n, P,  # noqa: E731
                                                                         w.data_ptr(), b.data_ptr(), g_.data_ptr(), be.data_ptr(),
                                                                         1e-5, o.data_ptr(), st.cuda_stream)
            with torch.cuda.stream(st):
                assert call() == 0
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=st):
                    for _ in range(K):
                        call()
            graphs[os.path.basename(paths[i])] = g
        torch.cuda.synchronize()
        times = {k: [] for k in graphs}
        for _ in range(7):
            for k, g in graphs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(st):
                    e0.record(st)
                    g.replay()
                    e1.record(st)
                e1.synchronize()
                times[k].append(e0.elapsed_time(e1) * 1e3 / K)
        d = max(float((o.float() - outs[0].float()).abs().max()) for o in outs)
        print(json.dumps({"op": "cat_ln_gelu", "P": P, "M": M, "us": {k: round(statistics.median(v), 2) for k, v in times.items()},
                          "max_diff_vs_first": d}), flush=True)


if __name__ == "__main__":
    main()

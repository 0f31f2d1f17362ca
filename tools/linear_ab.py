"""Diagnostic: the matcher projections (include/lightglue_glue.h lg_linear*) in their 64 x 64 and
256 x 128-tile, 256 x 256-tile, 128 x 256-tile and 128 x 128-tile 4-wave forms (lg_linear_set_wide
0 / 1 / 2 / 3 / 4-5) at P image pairs of n keypoints per image, graph
replay of back-to-back launches, interleaved; TFLOP/s of each.

    python tools/linear_ab.py [P] [n] [op substring] [modes, e.g. 012] [b]

With a fifth argument "b": yardsticks in the same run -- torch.nn.functional.linear (hipBLASLt,
fp16, plain [M, N] output + bias) on the op's M / K / N, and a device copy of the op's algorithmic
bytes (its HBM roofline at the copy rate); yardsticks only, never a product path. "cat_ln_gelu" is
lg_linear_cat_ln_gelu (its form by size; the mode list only switches the projection forms)."""
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
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    only = sys.argv[3] if len(sys.argv) > 3 else ""  # op-name substring (counter runs)
    modes = tuple(int(c) for c in sys.argv[4]) if len(sys.argv) > 4 and sys.argv[4] else (0, 1, 2)
    yard = len(sys.argv) > 5 and sys.argv[5] == "b"
    lib = _lib.load()
    dev, dt, h = torch.device("cuda:0"), torch.float16, 4
    M = P * 2 * n
    sp = (n, n, P)
    x = torch.randn(1, M, 256, device=dev, dtype=dt) * 0.5
    hx = torch.randn(1, M, 512, device=dev, dtype=dt) * 0.5
    cos = torch.randn(1, M, 64, device=dev, dtype=dt)
    sin = torch.randn(1, M, 64, device=dev, dtype=dt)
    c0, c1 = torch.randn(P, h, n, 64, device=dev, dtype=dt), torch.randn(P, h, n, 64, device=dev, dtype=dt)
    w768, b768 = torch.randn(768, 256, device=dev, dtype=dt) * 0.05, torch.randn(768, device=dev, dtype=dt)
    w2, b2 = torch.randn(512, 256, device=dev, dtype=dt) * 0.05, torch.randn(512, device=dev, dtype=dt)
    w3, b3 = torch.randn(512, 512, device=dev, dtype=dt) * 0.05, torch.randn(512, device=dev, dtype=dt)
    w4, b4 = torch.randn(256, 512, device=dev, dtype=dt) * 0.05, torch.randn(256, device=dev, dtype=dt)
    ln = torch.nn.LayerNorm(512).to(dev, dt)
    ops = {
        "qkv_rotary k256 n768": (lambda: mt._Hip.linear_qkv_rotary(x, w768, b768, cos, sin, h, sp), 256 * 768),
        "split2 k256 n512": (lambda: mt._Hip.linear_split2(x, w2, b2, h, sp), 256 * 512),
        "cat k512 n512": (lambda: mt._Hip.linear_cat(x, c0, c1, w3, b3), 512 * 512),
        "linear+res k512 n256": (lambda: mt._Hip.linear(hx, w4, b4, x), 512 * 256),
        "cat_ln_gelu k512 n512": (lambda: mt._Hip.linear_cat_ln_gelu(x, c0, c1, w3, b3, ln), 512 * 512),
    }
    # algorithmic bytes per op: A + W + bias + outputs (+ cos/sin, + residual)
    nbytes = {
        "qkv_rotary k256 n768": 2 * (M * 256 + 768 * 256 + 768 + M * 768 + 2 * M * 64),
        "split2 k256 n512": 2 * (M * 256 + 512 * 256 + 512 + M * 512),
        "cat k512 n512": 2 * (M * 512 + 512 * 512 + 512 + M * 512),
        "linear+res k512 n256": 2 * (M * 512 + 256 * 512 + 256 + 2 * M * 256),
        "cat_ln_gelu k512 n512": 2 * (M * 512 + 512 * 512 + 3 * 512 + M * 512),
    }
    blas = {}
    if yard:
        xa, xb = x.view(M, 256), hx.view(M, 512)
        blas = {
            "qkv_rotary k256 n768": lambda: torch.nn.functional.linear(xa, w768, b768),
            "split2 k256 n512": lambda: torch.nn.functional.linear(xa, w2, b2),
            "cat k512 n512": lambda: torch.nn.functional.linear(xb, w3, b3),
            "linear+res k512 n256": lambda: torch.nn.functional.linear(xb, w4, b4),
            "cat_ln_gelu k512 n512": lambda: torch.nn.functional.linear(xb, w3, b3),
        }
        pool = torch.empty(2 * max(nbytes.values()) // 2 + 16, dtype=torch.uint8, device=dev)
    st = torch.cuda.Stream(dev)
    K = 20
    graphs = {}
    ops = {k: v for k, v in ops.items() if only in k}
    for name, (fn, _) in ops.items():
        for wide in modes:
            lib.lg_linear_set_wide(wide)
            with torch.cuda.stream(st):
                fn()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=st):
                    for _ in range(K):
                        fn()
            graphs[(name, wide)] = g
        if yard:
            half = nbytes[name] // 2 // 16 * 16
            src_, dst_ = pool[:half], pool[half:2 * half]
            for key, fn_ in (("blas", blas[name]), ("copy", lambda: dst_.copy_(src_))):
                with torch.cuda.stream(st):
                    fn_()
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=st):
                        for _ in range(K):
                            fn_()
                graphs[(name, key)] = g
    lib.lg_linear_set_wide(-1)
    torch.cuda.synchronize()
    times = {k: [] for k in graphs}
    for _ in range(5):
        for k, g in graphs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(st):
                e0.record(st)
                g.replay()
                e1.record(st)
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) * 1e3 / K)
    for name, (_, kn) in ops.items():
        row = {"op": name, "M": M}
        for wide in modes:
            us = statistics.median(times[(name, wide)])
            # (files before round 5's forms 4 / 5 labelled forms 1 / 2 / 3 "wide" / "square" / "square5")
            row[("narrow", "wide", "square", "square5", "t128x128_4w", "t128x128_4w_bk32")[wide]] = {
                "us": round(us, 2), "tflops": round(2.0 * M * kn / us / 1e6, 1)}
        row["alg_MB"] = round(nbytes[name] / 1e6, 2)
        if yard:
            us = statistics.median(times[(name, "blas")])
            row["hipblaslt_F_linear"] = {"us": round(us, 2), "tflops": round(2.0 * M * kn / us / 1e6, 1)}
            us = statistics.median(times[(name, "copy")])
            row["copy_alg_bytes"] = {"us": round(us, 2), "TB_s": round(nbytes[name] / us / 1e6, 2)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

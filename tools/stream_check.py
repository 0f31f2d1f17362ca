"""Diagnostic: the persistent streaming kernel (forced plan code 23) against a torch fp32
reference and against the planner's other plans, then per-launch times by graph replay.

    python tools/stream_check.py [--quick] [--lib path/to/libmha_hd64.so]

Parity: max-abs of the stream kernel's fp16 / fp32 outputs vs softmax(q kᵀ / 8) v in fp32 (torch,
on the GPU, from the same fp16 inputs) over ragged and batched shapes. Timing: K launches of the
batched call (B calls of 1x4x1024x1024 stacked in the batch dimension) captured in one graph,
stream kernel vs the planner's default plan, interleaved rounds, median; frac = FLOPs / time /
2.5 PFLOP/s. One JSON object per line on stdout."""
import argparse
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

from lightglue_amd import _lib  # noqa: E402

STREAM = 23


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    for name, (args, res) in list(_lib.SIGNATURES.items()) + list(_lib.HOOKS.items()):
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
    return lib


def forced(lib, q, k, v, o, code, ws, stream, kvw=0):
    b, h, nq, _ = q.shape
    nkv = k.shape[2]
    st = lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), b, h, nq, nkv,
                                    int(q.dtype == torch.float32), int(o.dtype == torch.float32), code, kvw, 0,
                                    ws.data_ptr(), ws.numel(), stream.cuda_stream, 3)
    if st != 0:
        raise RuntimeError(lib.mha_hd64_last_error().decode())


def reference(q, k, v):
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * 0.125
    return torch.matmul(torch.softmax(s, dim=-1), v.float())


def parity(lib, dev, quick):
    shapes = [(1, 100, 77), (1, 128, 64), (1, 33, 65), (1, 1, 1), (1, 129, 1), (2, 300, 1000), (3, 1000, 777),
              (1, 64, 2048), (5, 257, 63), (1, 1024, 1024), (8, 1024, 1024), (16, 1024, 1024), (2, 2048, 2048),
              (40, 128, 128), (1, 1000, 3)]
    if quick:
        shapes = shapes[:6] + [(16, 1024, 1024)]
    stream = torch.cuda.current_stream()
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    g = torch.Generator(device="cpu").manual_seed(7)
    for b, nq, nkv in shapes:
        q = (torch.randn(b, 4, nq, 64, generator=g) * 1.0).half().to(dev)
        k = (torch.randn(b, 4, nkv, 64, generator=g) * 1.0).half().to(dev)
        v = torch.randn(b, 4, nkv, 64, generator=g).half().to(dev)
        ref = reference(q, k, v)
        row = {"shape": [b, 4, nq, nkv]}
        for od in (torch.float16, torch.float32):
            res = {}
            for name, code, kvw in (("stream4", STREAM, 4), ("stream8", STREAM, 8), ("planner", 0, 0)):
                o = torch.full(q.shape, float("nan"), dtype=od, device=dev)
                forced(lib, q, k, v, o, code, ws, stream, kvw)
                torch.cuda.synchronize()
                res[name] = {"max_abs_vs_fp32": float((o.float() - ref).abs().max()), "nan": bool(torch.isnan(o).any())}
            row["f16out" if od == torch.float16 else "f32out"] = res
        print(json.dumps(row), flush=True)


def timing(lib, dev, quick):
    stream = torch.cuda.Stream()
    ws = torch.empty(5242880, dtype=torch.uint8, device=dev)
    batches = (8, 12, 16, 24, 32, 64) if not quick else (16, 32)
    for B in batches:
        q = torch.randn(B, 4, 1024, 64, device=dev).half()
        k = torch.randn(B, 4, 1024, 64, device=dev).half()
        v = torch.randn(B, 4, 1024, 64, device=dev).half()
        o = torch.empty_like(q)
        K = max(20, 400 // B)
        graphs = {}
        for name, code, kvw in (("stream4", STREAM, 4), ("stream8", STREAM, 8), ("ring", 4, 1), ("planner", 0, 0)):
            with torch.cuda.stream(stream):
                forced(lib, q, k, v, o, code, ws, stream, kvw)  # warm, plan
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr, stream=stream):
                    for _ in range(K):
                        forced(lib, q, k, v, o, code, ws, stream, kvw)
            graphs[name] = gr
        torch.cuda.synchronize()
        times = {n: [] for n in graphs}
        for _ in range(7):
            for n, gr in graphs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(stream):  # replay() runs on the current stream
                    e0.record(stream)
                    gr.replay()
                    e1.record(stream)
                e1.synchronize()
                times[n].append(e0.elapsed_time(e1) * 1e3 / K)
        flops = 4.0 * B * 4 * 1024 * 1024 * 64
        out = {"calls_per_launch": B, "launches_per_graph": K}
        for n, ts in times.items():
            us = statistics.median(ts)
            out[n] = {"us_per_launch": round(us, 3), "frac": round(flops / (us * 1e-6) / 2.5e15, 4)}
        print(json.dumps(out), flush=True)


def slope(libs, dev, waves=(4, 8)):
    """Per-step cost without item seams: one item per workgroup (B = 16 calls of nq = 1024: 256
    items of 256 rows / 512 of 128 rows = one residency round), nkv = 1024 .. 8192; the slope of
    launch time over 64-key steps is the steady step, the intercept the launch's fixed cost. Also
    B = 32 and 64 at nkv = 1024 (2 and 4 items per workgroup). Libraries and forms interleaved."""
    stream = torch.cuda.Stream()
    ws = torch.empty(5242880, dtype=torch.uint8, device=dev)
    K = 20
    nkvs = (1024, 2048, 4096, 8192)
    cfgs = [(16, n) for n in nkvs] + [(32, 1024), (64, 1024)]
    data = {}
    for B, n in cfgs:
        data[(B, n)] = (torch.randn(B, 4, 1024, 64, device=dev).half(), torch.randn(B, 4, n, 64, device=dev).half(),
                        torch.randn(B, 4, n, 64, device=dev).half(), torch.empty(B, 4, 1024, 64, device=dev).half())
    graphs = {}
    for li, lib in enumerate(libs):
        for w in waves:
            for B, n in cfgs:
                q, k, v, o = data[(B, n)]
                with torch.cuda.stream(stream):
                    forced(lib, q, k, v, o, STREAM, ws, stream, w)
                    gr = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gr, stream=stream):
                        for _ in range(K):
                            forced(lib, q, k, v, o, STREAM, ws, stream, w)
                graphs[(li, w, B, n)] = gr
    torch.cuda.synchronize()
    times = {key: [] for key in graphs}
    for _ in range(7):
        for key, gr in graphs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(stream):
                e0.record(stream)
                gr.replay()
                e1.record(stream)
            e1.synchronize()
            times[key].append(e0.elapsed_time(e1) * 1e3 / K)
    for li in range(len(libs)):
        for w in waves:
            us = [statistics.median(times[(li, w, 16, n)]) for n in nkvs]
            steps = [n // 64 for n in nkvs]
            mx, my = statistics.mean(steps), statistics.mean(us)
            b = sum((x - mx) * (y - my) for x, y in zip(steps, us)) / sum((x - mx) ** 2 for x in steps)
            extra = {f"b{B}_us": round(statistics.median(times[(li, w, B, 1024)]), 3) for B in (32, 64)}
            extra.update({f"b{B}_frac": round(4.0 * B * 4 * 1024 * 1024 * 64 / (extra[f"b{B}_us"] * 1e-6) / 2.5e15, 4)
                          for B in (32, 64)})
            print(json.dumps({"lib": li, "waves": w, "b16_us": [round(u, 3) for u in us], "nkv": list(nkvs),
                              "us_per_step": round(b, 4), "intercept_us": round(my - b * mx, 3),
                              "b16_frac": round(4.0 * 16 * 4 * 1024 * 1024 * 64 / (us[0] * 1e-6) / 2.5e15, 4),
                              **extra}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--lib", default=_lib.LIB_PATH)
    ap.add_argument("--no-timing", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--slope", default=None, help="comma-separated libraries: per-step slope of each (A/B)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    if args.slope:
        slope([load(p) for p in args.slope.split(",")], dev)
        return
    lib = load(args.lib)
    if not args.no_parity:
        parity(lib, dev, args.quick)
    if not args.no_timing:
        timing(lib, dev, args.quick)


if __name__ == "__main__":
    main()

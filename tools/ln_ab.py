"""Diagnostic: lg_layernorm_gelu (fp16, dim 512: the matcher FFN's LayerNorm + GELU) from several
builds of the library in one process (each loaded with its own ctypes handle), graph replay of
back-to-back launches, interleaved; plus a device copy of the same bytes (the op's HBM yardstick).
Each build's output is compared with the first's (max |diff|, differing elements).

    python tools/ln_ab.py <lib.so>[,<lib.so>...] [rows=32768]
"""
import ctypes
import json
import statistics
import sys

import torch


def main():
    libs = sys.argv[1].split(",")
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    x = torch.randn(rows, 512, device=dev, dtype=torch.float16) * 2
    g = (1 + 0.2 * torch.randn(512, device=dev)).half()
    b = (0.2 * torch.randn(512, device=dev)).half()
    st = torch.cuda.Stream(dev)
    K = 20
    graphs, outs = {}, {}
    for i, path in enumerate(libs):
        lib = ctypes.CDLL(path)
        fn = lib.lg_layernorm_gelu
        fn.restype = ctypes.c_int32
        fn.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                       ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p]
        y = torch.empty_like(x)
        call = (lambda fn=fn, y=y: fn(1, x.data_ptr(), g.data_ptr(), b.data_ptr(), rows, 512, 1e-5, y.data_ptr(),
                                       ctypes.c_void_p(st.cuda_stream)))
        with torch.cuda.stream(st):
            assert call() == 0, path
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=st):
                for _ in range(K):
                    call()
        graphs[i], outs[i] = gr, y
    src = torch.empty(rows * 512 * 2, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    with torch.cuda.stream(st):
        dst.copy_(src)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=st):
            for _ in range(K):
                dst.copy_(src)
    graphs["copy"] = gr
    torch.cuda.synchronize()
    times = {k: [] for k in graphs}
    for _ in range(7):
        for k, gr in graphs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(st):
                e0.record(st)
                gr.replay()
                e1.record(st)
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) * 1e3 / K)
    nbytes = 2 * rows * 512 * 2
    for i, path in enumerate(libs):
        us = statistics.median(times[i])
        d = (outs[i].float() - outs[0].float()).abs()
        print(json.dumps({"lib": path, "rows": rows, "us": round(us, 2), "TB_s": round(nbytes / us / 1e6, 2),
                          "max_diff_vs_first": float(d.max()), "n_diff_vs_first": int((d > 0).sum())}), flush=True)
    us = statistics.median(times["copy"])
    print(json.dumps({"copy_same_bytes_us": round(us, 2), "TB_s": round(nbytes / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()

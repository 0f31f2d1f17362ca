"""Diagnostic: the single-pass kernel (forced plan 21) against the C oracle on assorted shapes, and
per-launch graph-replay times of the single 1x4xNxN call under the single-pass kernel vs the ring
kernel's (1,8) in-launch-combine plan. Prints one JSON line.

    python tools/direct_check.py [--time-only]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lightglue_amd import _lib, synth  # noqa: E402
from oracle import oracle  # noqa: E402

K = 200


def forced(lib, q, k, v, o, nq, nkv, qw, kw, sp, ws, batch=1):
    st = lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), batch, 4, nq, nkv,
                                    int(q.dtype == torch.float32), int(o.dtype == torch.float32), qw, kw, sp,
                                    ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream, 3)
    assert st == 0, _lib.last_error()


def per_launch_us(fn):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(K):
                fn()
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            g.replay()
            b.record(s)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3 / K)
    return sorted(ts)[len(ts) // 2]


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
    res = {}
    if "--time-only" not in sys.argv:
        errs = {}
        for nq, nkv in [(1, 1), (33, 65), (100, 77), (256, 256), (1000, 777), (1024, 1024), (64, 1024), (513, 513),
                        (2048, 1000), (300, 129), (97, 600)]:
            qn, kn, vn = synth.qkv(77 + nq + 3 * nkv, nq, nkv)
            q16, k16, v16 = (synth.round_f16(x) for x in (qn, kn, vn))
            ref = oracle.attention_c(q16, k16, v16)
            q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in (q16, k16, v16))
            for of in (0, 1):
                o = torch.full(q.shape, float("nan"), dtype=torch.float32 if of else torch.float16, device=dev)
                for code in (21, 22):
                    o.fill_(float("nan"))
                    forced(lib, q, k, v, o, nq, nkv, code, 0, 0, ws)
                    torch.cuda.synchronize()
                    got = o.float().cpu().numpy()
                    errs[f"{code}_{nq}x{nkv}_{'f32' if of else 'f16'}"] = (float(np.abs(got - ref).max())
                                                                          if np.isfinite(got).all() else "nonfinite")
        # peaky logits (rescale branch)
        qn, kn, vn = synth.qkv(4242, 256, 1024, q_std=3.0)
        q16, k16, v16 = (synth.round_f16(x) for x in (qn, kn, vn))
        ref = oracle.attention_c(q16, k16, v16)
        q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in (q16, k16, v16))
        o = torch.empty_like(q)
        for code in (21, 22):
            forced(lib, q, k, v, o, 256, 1024, code, 0, 0, ws)
            torch.cuda.synchronize()
            errs[f"{code}_peaky256x1024"] = float(np.abs(o.float().cpu().numpy() - ref).max())
        res["max_abs_err"] = errs
    for n in (512, 1024):
        qn, kn, vn = synth.qkv(5, n, n)
        q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in (qn, kn, vn))
        o = torch.empty_like(q)
        t_direct = per_launch_us(lambda: forced(lib, q, k, v, o, n, n, 21, 0, 0, ws))
        t_ring = per_launch_us(lambda: forced(lib, q, k, v, o, n, n, 1, 8, 0, ws))
        t_direct2 = per_launch_us(lambda: forced(lib, q, k, v, o, n, n, 21, 0, 0, ws))
        t16 = per_launch_us(lambda: forced(lib, q, k, v, o, n, n, 22, 0, 0, ws))
        res[f"us_{n}"] = {"direct": round(min(t_direct, t_direct2), 3), "direct16": round(t16, 3),
                          "ring_1x8": round(t_ring, 3)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()

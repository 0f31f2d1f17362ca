"""Measurement: the MHAHeadDim64 plugin's per-call time over the sizes the reference accepts
(Nq, Nkv <= 2048; lightglue_attention_plugin.cpp:312-359), for its two type paths (Half -> Half,
Float -> Float) and the fp16-in / fp32-out launcher (configs[2]). Each call is timed the headline's
way (bench.timed_replays: K direct enqueues with bindings prepared once, queued behind a sleep
kernel, HIP events around the K; median of the repetitions), with its algorithmic TFLOP/s and
fraction of the 2.5 PF fp16 dense peak, the planner's plan, and the max-abs error against a torch
fp32 reference of the same call. One JSON line per case.

    python tools/plugin_size_sweep.py [K=100]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import ctypes  # noqa: E402

import torch  # noqa: E402

import bench  # noqa: E402
from lightglue_amd import _lib, mha_hd64_batched, plugin, synth  # noqa: E402

SIZES = [(64, 64), (128, 128), (256, 256), (384, 384), (512, 512), (768, 768), (1024, 1024), (1536, 1536),
         (2048, 2048), (1000, 1000), (333, 777), (512, 1024), (1024, 512), (1024, 2048), (2048, 1024), (97, 2048)]


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    dev = torch.device("cuda:0")
    lib = _lib.load()
    st = torch.cuda.Stream(dev)
    nop = lambda: None  # noqa: E731  (one process: no barrier, the max over ranks is the value)
    for nq, nkv in SIZES:
        qn, kn, vn = synth.qkv(31, nq, nkv)
        q32, k32, v32 = (torch.from_numpy(x).to(dev).contiguous() for x in (qn, kn, vn))
        ref = torch.softmax((q32.double() / 8) @ k32.double().transpose(-1, -2), -1) @ v32.double()
        plan = (ctypes.c_int32 * 4)()
        lib.mha_hd64_plan(1, 4, nq, nkv, 5242880, plan)
        for path in ("half", "float", "half_in_float_out"):
            dt = torch.float32 if path == "float" else torch.float16
            q, k, v = (t.to(dt).contiguous() for t in (q32, k32, v32))
            out = torch.empty(q.shape, dtype=torch.float16 if path == "half" else torch.float32, device=dev)
            with torch.cuda.stream(st):
                if path == "half_in_float_out":
                    step = lambda: mha_hd64_batched(q, k, v, out_dtype=torch.float32, out=out)  # noqa: E731
                else:
                    step = plugin.bound_enqueue(q, k, v, out)
                for _ in range(5):
                    step()
            st.synchronize()
            err = float((out.double() - ref).abs().max())

            def run():
                for _ in range(steps):
                    step()

            t, host = bench.timed_replays(torch, run, st, nop, lambda x: x, 10)
            us = t * 1e6 / steps
            fl = bench.call_flops(1, 4, nq, nkv)
            print(json.dumps({"nq": nq, "nkv": nkv, "path": path, "us_per_call": round(us, 3),
                              "calls_per_s": round(1e6 / us, 1), "tflops": round(fl / us * 1e-6, 2),
                              "frac": round(fl / us * 1e-6 / 2500.0, 4), "max_abs_vs_fp64": err,
                              "plan": list(plan)[:3], "host_us_per_call": round(host * 1e6 / steps, 2)}), flush=True)


if __name__ == "__main__":
    main()

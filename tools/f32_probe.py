"""Float-boundary (fp32 Q/K/V -> fp32 O) per-call time for one library build (MHA_HD64_LIB selects it;
MHA_HD64_F32_INKERNEL=0 the convert launch + fp16 kernel): 2000 back-to-back calls in a graph, plus
an output digest so builds can be compared bit for bit. Usage: python tools/f32_probe.py [nq-nkv ...]"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def main():
    import torch

    import lightglue_amd
    from lightglue_amd import synth

    # "nq-nkv" or "BxNQ-NKV" (B calls stacked in the batch dimension of one launch)
    def parse(s):
        b, _, rest = s.rpartition("x")
        nq, nkv = (int(x) for x in rest.split("-"))
        return int(b or 1), nq, nkv

    shapes = [parse(s) for s in sys.argv[1:]] or [(1, 1024, 1024), (1, 512, 512)]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    barrier, reduce_max = bench.make_collectives(torch, None)
    for b, nq, nkv in shapes:
        q, k, v = (torch.from_numpy(x).to(dev).float().contiguous() for x in synth.qkv(100, nq, nkv, batch=b))
        call = lightglue_amd.mha_hd64 if b == 1 else lightglue_amd.mha_hd64_batched
        out = torch.empty_like(q)
        with torch.cuda.stream(stream):
            for _ in range(50):
                call(q, k, v, out=out)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for _ in range(2000):
                call(q, k, v, out=out)
        g.replay()
        stream.synchronize()
        t, _ = bench.timed_replays(torch, g.replay, stream, barrier, reduce_max, 5)
        ref = torch.softmax((q.half().float() @ k.half().float().transpose(-1, -2)) * 0.125, -1) @ v.half().float()
        print(json.dumps({"lib": os.environ.get("MHA_HD64_LIB", "default"),
                          "inkernel": os.environ.get("MHA_HD64_F32_INKERNEL", "1"),
                          "convert": os.environ.get("MHA_HD64_F32_CONVERT", "1"), "batch": b, "nq": nq, "nkv": nkv,
                          "us_per_launch": round(t / 2000 * 1e6, 3),
                          "max_abs_vs_fp32_of_fp16_inputs": float((out - ref).abs().max()),
                          "digest": hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()

"""Warm vs cold inputs for one library build (A/B of load-schedule changes; MHA_HD64_LIB selects it).

warm: 2000 calls on one Q/K/V in a graph (the headline's L2-resident inputs);
cold: bench.cold_inputs (each call on its own copy from a 640 MiB pool: inputs from HBM).
Prints one JSON line per shape, then the end-to-end matcher's ms per pair (50 replays). Usage: python tools/cold_probe.py [--no-matcher] [nq-nkv ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def main():
    import torch

    import lightglue_amd
    from lightglue_amd import synth

    args = [a for a in sys.argv[1:] if a != "--no-matcher"]
    shapes = [tuple(int(x) for x in s.split("-")) for s in args] or [(1024, 1024), (512, 512), (2048, 2048)]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    barrier, reduce_max = bench.make_collectives(torch, None)
    for nq, nkv in shapes:
        q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in synth.qkv(100, nq, nkv))
        out = torch.empty_like(q)
        with torch.cuda.stream(stream):
            for _ in range(50):
                lightglue_amd.mha_hd64(q, k, v, out=out)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for _ in range(2000):
                lightglue_amd.mha_hd64(q, k, v, out=out)
        g.replay()
        stream.synchronize()
        t, _ = bench.timed_replays(torch, g.replay, stream, barrier, reduce_max, 5)
        del g
        cold = bench.cold_inputs(torch, lightglue_amd, stream, q, k, v, barrier, reduce_max, 1)
        ref = out.float()
        print(json.dumps({"lib": os.environ.get("MHA_HD64_LIB", "default"), "nq": nq, "nkv": nkv,
                          "warm_us": round(t / 2000 * 1e6, 3), "cold_us": cold["us_per_call"],
                          "cold_identical": cold["outputs_identical_to_each_other"],
                          "out_sum": round(float(ref.sum()), 3)}), flush=True)
    # the matcher end to end: Q/K/V written by the producing kernels just before each call
    if "--no-matcher" in sys.argv:
        return
    m = bench.matcher_e2e(torch, dev, stream, 0, sizes=(512, 1024, 2048), reps=50)
    print(json.dumps({"lib": os.environ.get("MHA_HD64_LIB", "default"),
                      "matcher_ms": {n: r["ms"] for n, r in m.items()}}), flush=True)


if __name__ == "__main__":
    main()

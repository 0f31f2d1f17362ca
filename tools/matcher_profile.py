"""Diagnostic: the end-to-end fp16 matcher with P image pairs per forward (bench.py
matcher_batched_pairs' form), replayed from a graph, for a kernel trace:

    rocprofv3 --kernel-trace --stats -d <dir> -- python tools/matcher_profile.py [P] [n] [reps] [fp16|fp32]

Prints ms per forward and pairs/s (HIP events)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

from lightglue_amd import matcher  # noqa: E402


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    dt = torch.float32 if len(sys.argv) > 4 and sys.argv[4] == "fp32" else torch.float16
    dev = torch.device("cuda:0")
    model = matcher.LightGlueMatcher(n_layers=9).eval()
    model.load_state_dict(matcher.seeded_state_dict(7, 9), strict=True)
    model = model.to(dev, dt)
    ps = [matcher.synthetic_pair(80 + i, n, n) for i in range(P)]
    batch = tuple(torch.cat([p[j] for p in ps], 0).to(dev, dt) for j in range(4))
    st = torch.cuda.Stream(dev)
    with torch.no_grad(), torch.cuda.stream(st):
        for _ in range(2):
            model(*batch)
        st.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            out = model(*batch)
    g.replay()
    st.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    with torch.cuda.stream(st):
        for _ in range(reps):
            g.replay()
    e1.record(st)
    st.synchronize()
    ms = e0.elapsed_time(e1) / reps
    assert bool(torch.isfinite(out[2]).all())
    print(f"P={P} n={n}: {ms:.4f} ms per forward, {P * 1e3 / ms:.1f} pairs/s", flush=True)


if __name__ == "__main__":
    main()

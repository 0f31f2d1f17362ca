"""Diagnostic: what a matcher forward costs per graph replay beyond its kernels. For P pairs of n
keypoints (seeded fp16 model, as bench.py's matcher_batched_pairs): (a) bench.py's way — one captured
forward, `reps` replays back to back between two events; (b) `reps` forwards captured into ONE graph,
one replay; (c) (a) with the replays issued behind a long sleep kernel, so that the host has queued
them all before the GPU reaches the first. ms per forward each, medians of several rounds.

    python tools/forward_replay_overhead.py [n=1024] [P,...=1,16] [reps=10]
"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402


def main():
    from lightglue_amd import matcher

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    Ps = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,16").split(",")]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    model = matcher.LightGlueMatcher(n_layers=9).eval()
    model.load_state_dict(matcher.seeded_state_dict(7, 9), strict=True)
    model = model.to(dev, torch.float16)
    for P in Ps:
        ps = [matcher.synthetic_pair(80 + i, n, n) for i in range(P)]
        batch = tuple(torch.cat([p[j] for p in ps], 0).to(dev, torch.float16) for j in range(4))
        with torch.no_grad(), torch.cuda.stream(st):
            for _ in range(2):
                model(*batch)
            st.synchronize()
            g1 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1, stream=st):
                model(*batch)
            gk = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gk, stream=st):
                for _ in range(reps):
                    model(*batch)
        res = {"a_replays": [], "b_one_graph": [], "c_behind_sleep": []}
        for _ in range(5):
            for key in res:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                with torch.cuda.stream(st):
                    if key == "c_behind_sleep":
                        torch.cuda._sleep(50_000_000)
                    e0.record(st)
                    if key == "b_one_graph":
                        gk.replay()
                    else:
                        for _ in range(reps):
                            g1.replay()
                    e1.record(st)
                e1.synchronize()
                res[key].append(e0.elapsed_time(e1) / reps)
        print(json.dumps({"P": P, "n": n, "reps": reps, **{k: round(statistics.median(v), 4) for k, v in res.items()}}),
              flush=True)


if __name__ == "__main__":
    main()

"""Diagnostic: bench.py's matcher_batched_pairs at P pairs, with 1 and with 2 captured streams, and the
same forward through tools/forward_replay_overhead.py's harness, on one box: does the bench's own
setup change the single-stream ms per forward?

    python tools/bench_pairs_probe.py [P=16]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    for streams in (1, 2, 1):
        r = bench.matcher_batched_pairs(torch, dev, st, 0, n=1024, pairs=(P,), streams=streams)
        print(json.dumps({"P": P, "streams_captured": streams, "ms_per_forward": r[str(P)]["ms_per_forward"]}), flush=True)


if __name__ == "__main__":
    main()

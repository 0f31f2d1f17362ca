"""Diagnostic: one saved head (an .npz of q, k, v fp16 [1, 1, n, 64], e.g.
tests/golden/stream_spec_overflow_head.npz) through the streaming kernel (forced plan 23, kv_waves
4 and 8, fp16 and fp32 output) of each library given, against an fp64 reference: max error and the
non-finite rows.

    python tools/stream_head.py file.npz lib_a.so[,lib_b.so]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tools"), os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

from stream_check import STREAM, forced, load  # noqa: E402


def main():
    d = np.load(sys.argv[1])
    q, k, v = (d[n] for n in "qkv")
    s = np.einsum("bhqd,bhkd->bhqk", q.astype(np.float64), k.astype(np.float64)) * 0.125
    p = np.exp(s - s.max(-1, keepdims=True))
    ref = (p / p.sum(-1, keepdims=True)) @ v.astype(np.float64)
    dev = torch.device("cuda:0")
    ws = torch.empty(5242880, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    qd, kd, vd = (torch.from_numpy(x).to(dev) for x in (q, k, v))
    for path in sys.argv[2].split(","):
        lib = load(path)
        for w in (4, 8):
            for odt in (torch.float16, torch.float32):
                o = torch.full(qd.shape, float("nan"), dtype=odt, device=dev)
                forced(lib, qd, kd, vd, o, STREAM, ws, stream, w)
                torch.cuda.synchronize()
                got = o.float().cpu().numpy().astype(np.float64)
                bad = ~np.isfinite(got).all(-1)
                err = np.abs(np.nan_to_num(got, nan=1e9) - ref).max()
                print(json.dumps({"lib": os.path.basename(path), "waves": w, "out": str(odt).split(".")[-1],
                                  "max_err": float(err), "bad_rows": np.nonzero(bad.reshape(-1))[0].tolist()}))


if __name__ == "__main__":
    main()

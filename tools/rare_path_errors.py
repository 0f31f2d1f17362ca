"""Diagnostic: where the streaming kernel's errors sit on the every-item-recomputed input of
tests/test_gpu_stream.py (one gain-8 spike key per 128-row block), per library (lazy / spec builds)
and kv_waves, fp32 output, against the fp64 C oracle: max error, its row, that row's max logit
minus its tile-0 max (log2 units; > 16 = the speculative form's overflow), and the error over the
rows whose max moved by less than 16.

    python tools/rare_path_errors.py lib_a.so[,lib_b.so] [nkv=200]
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
    from lightglue_amd import synth
    from oracle import oracle as oracle_mod

    oracle_mod.build()
    libs = sys.argv[1].split(",")
    nkv = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    batch, nq = 40, 512
    qn, kn, vn = synth.qkv(4242 + nkv, nq, nkv, batch=batch)
    for blk in range(nq // 128):
        kn = synth.spike(qn, kn, 128 * blk + 9 + 11 * blk, 64 + 37 * blk, 8.0)
    q16, k16, v16 = (synth.round_f16(x) for x in (qn, kn, vn))
    bsel = [0, 23, batch - 1]
    ref = oracle_mod.attention_c(q16[bsel], k16[bsel], v16[bsel])
    s = np.einsum("bhqd,bhkd->bhqk", q16[bsel].astype(np.float64), k16[bsel].astype(np.float64)) * 0.125 / np.log(2)
    move = s.max(-1) - s[..., :64].max(-1)
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream()
    ws = torch.empty(5242880, dtype=torch.uint8, device=dev)
    q, k, v = (torch.from_numpy(x).half().to(dev) for x in (q16, k16, v16))
    for path in libs:
        lib = load(path)
        for w in (4, 8):
            o = torch.full(q.shape, float("nan"), dtype=torch.float32, device=dev)
            with torch.cuda.stream(stream):
                forced(lib, q, k, v, o, STREAM, ws, stream, w)
            torch.cuda.synchronize()
            got = o.cpu().numpy()[bsel].astype(np.float64)
            err = np.abs(got - ref).max(-1)
            i = np.unravel_index(int(err.argmax()), err.shape)
            print(json.dumps({"lib": os.path.basename(path), "waves": w, "nkv": nkv, "max_err": float(err.max()),
                              "at": [int(x) for x in i], "move_log2_at": float(move[i]),
                              "rows_over16": int((move > 16).sum()), "max_err_rows_under16": float(err[move <= 16].max()),
                              "max_err_rows_over16": float(err[move > 16].max()) if (move > 16).any() else None,
                              "p99_err": float(np.quantile(err, 0.99))}))


if __name__ == "__main__":
    main()

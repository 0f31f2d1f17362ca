"""Diagnostic: the first attention launch of the seeded fp16 matcher (P pairs stacked, n = 1024) whose
output holds a non-finite value: which layer / call, whether its inputs are finite, which rows are
bad, those rows' score move past tile 0's max (log2 units; > 16 overflows the speculative max's
fp16 P), and whether the same call launched alone through the streaming kernel (forced plan 23,
both kv_waves, non-grouped) reproduces it, also for the failing head alone (whose q, k, v it saves
under gpurun_out/nan_probe/ as .npy). Prints JSON lines.

    python tools/matcher_nan_probe.py [P=8] [n=1024]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tools"), os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from stream_check import STREAM, forced, load  # noqa: E402


OUT = os.path.join(REPO, "gpurun_out", "nan_probe")


def main():
    from lightglue_amd import _lib, matcher

    P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    dev = torch.device("cuda:0")
    model = matcher.LightGlueMatcher(n_layers=9).eval()
    model.load_state_dict(matcher.seeded_state_dict(7, 9), strict=True)
    model = model.to(dev, torch.float16)
    ps = [matcher.synthetic_pair(80 + i, n, n) for i in range(P)]
    batch = tuple(torch.cat([p[j] for p in ps], 0).to(dev, torch.float16) for j in range(4))
    lib = load(_lib.LIB_PATH)
    ws = torch.empty(5242880, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    orig = model.attention
    state = {"launch": 0, "done": False}

    def probe(calls):
        outs = orig(calls)
        torch.cuda.synchronize()
        li = state["launch"]
        state["launch"] += 1
        if state["done"]:
            return outs
        for ci, ((q, k, v), o) in enumerate(zip(calls, outs)):
            if bool(torch.isfinite(o).all()):
                continue
            state["done"] = True
            bad = ~torch.isfinite(o).all(-1)  # [B, H, nq]
            s = torch.einsum("bhqd,bhkd->bhqk", q.float(), k.float()) * (0.125 / 0.6931471805599453)
            move = s.amax(-1) - s[..., :64].amax(-1)
            ref = torch.softmax(s * 0.6931471805599453, -1) @ v.float()
            rec = {"launch": li, "call": ci, "shape": list(q.shape), "nkv": k.shape[2],
                   "inputs_finite": [bool(torch.isfinite(t).all()) for t in (q, k, v)],
                   "bad_rows": int(bad.sum()), "bad_first": bad.nonzero()[:6].tolist(),
                   "move_bad_rows_max": float(move[bad].max()) if bad.any() else None,
                   "rows_move_over16": int((move > 16).sum()), "move_max": float(move.max()),
                   "abs_score_max": float(s.abs().max()),
                   "err_good_rows": float((o.float() - ref).abs().amax(-1)[~bad].max())}
            for w in (4, 8):
                o2 = torch.empty_like(q)
                forced(lib, q.contiguous(), k.contiguous(), v.contiguous(), o2, STREAM, ws, stream, w)
                torch.cuda.synchronize()
                rec[f"alone_w{w}_bad_rows"] = int((~torch.isfinite(o2).all(-1)).sum())
                rec[f"alone_w{w}_err"] = float((o2.float() - ref).abs().nan_to_num(1e9).max())
            b0, h0 = (int(x) for x in bad.nonzero()[0, :2])
            qh, kh, vh = (t[b0:b0 + 1, h0:h0 + 1].contiguous() for t in (q, k, v))
            os.makedirs(OUT, exist_ok=True)
            for name, t in (("q", qh), ("k", kh), ("v", vh)):
                np.save(os.path.join(OUT, f"nan_{name}.npy"), t.cpu().numpy())
            for w in (4, 8):  # the failing head alone
                o2 = torch.empty_like(qh)
                forced(lib, qh, kh, vh, o2, STREAM, ws, stream, w)
                torch.cuda.synchronize()
                rec[f"head_alone_w{w}_bad_rows"] = (~torch.isfinite(o2).all(-1)).nonzero()[:, 2].tolist()
            print(json.dumps(rec), flush=True)
        return outs

    model.attention = probe
    with torch.no_grad():
        out = model(*batch)
    torch.cuda.synchronize()
    print(json.dumps({"P": P, "n": n, "launches": state["launch"], "found": state["done"],
                      "outputs_finite": [bool(torch.isfinite(t).all()) for t in out]}))


if __name__ == "__main__":
    main()

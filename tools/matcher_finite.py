"""Diagnostic: is every output of the seeded fp16 matcher finite, per P (pairs stacked in one
forward, n = 1024, as bench.py's matcher_batched_pairs), with the library in MHA_HD64_LIB (or the
shipped one)? Prints per P: finite flags of descriptors / scores and the max |score| of finite ones,
and the largest |difference| from a per-pair forward (P = 1 each).

    [MHA_HD64_LIB=...] python tools/matcher_finite.py [n=1024] [P,...=1,4,8,16,32]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402


def main():
    from lightglue_amd import matcher

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    Ps = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,4,8,16,32").split(",")]
    dev = torch.device("cuda:0")
    model = matcher.LightGlueMatcher(n_layers=9).eval()
    model.load_state_dict(matcher.seeded_state_dict(7, 9), strict=True)
    model = model.to(dev, torch.float16)
    for P in Ps:
        ps = [matcher.synthetic_pair(80 + i, n, n) for i in range(P)]
        batch = tuple(torch.cat([p[j] for p in ps], 0).to(dev, torch.float16) for j in range(4))
        with torch.no_grad():
            out = model(*batch)
            torch.cuda.synchronize()
            fin = [bool(torch.isfinite(o).all()) if torch.is_tensor(o) and o.is_floating_point() else None for o in out]
            bad = {}
            for i, o in enumerate(out):
                if torch.is_tensor(o) and o.is_floating_point() and not bool(torch.isfinite(o).all()):
                    nf = ~torch.isfinite(o)
                    idx = nf.nonzero()[:4].tolist()
                    bad[i] = {"count": int(nf.sum()), "first": idx}
            single = []
            for i in range(min(P, 3)):
                o1 = model(*(t[i:i + 1] for t in batch))
                single.append(float((o1[2].float() - out[2][i:i + 1].float()).abs().nan_to_num(1e9).max()))
        print(json.dumps({"P": P, "n": n, "finite": fin, "bad": bad, "scores_vs_single": single,
                          "lib": os.environ.get("MHA_HD64_LIB", "shipped")}))


if __name__ == "__main__":
    main()

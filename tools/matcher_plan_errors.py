"""Diagnostic: where the fp16 matcher's matched-entry log-score
error comes from, single pair vs P pairs per forward.

For the 1024 x 1024, 9-layer sweep fixture (tests/golden/sweep_l9_1024x1024.npz: outputs of the
reference LightGlue), the fp16 model's errors against the reference (descriptors, log-scores, the
log-score on the reference's mutual nearest neighbours = tests/test_matcher.py's err_m) for:
  single   one pair per forward with the planner's default plans, and with other attention plans
           (concurrency hint 2 / 3: 32-row kernels; stream mode 0 / 1);
  batched  the fixture pair inside P = 4 / 8 pairs per forward (slot 0 and slot P/2), stream
           mode 0 (the LDS-ring kernel) and 1 (the streaming kernel, the planner's default);
  ulp      one pair per forward, each attention output perturbed by +-1 fp16 ulp on a seeded random
           10 % of its elements (8 seeds): how far an attention-rounding difference alone moves
           err_m after 9 layers.
One JSON line per run.

    python tools/matcher_plan_errors.py [float16|float32]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lightglue_amd  # noqa: E402
import test_matcher as tm  # noqa: E402
from lightglue_amd import _lib, matcher  # noqa: E402

NAME = "sweep_l9_1024x1024"


def errs(g, d0, d1, sc):
    rows = g["rows"]
    ed = max(float((d0[0, rows] - torch.from_numpy(g["desc0_rows"])).abs().max()),
             float((d1[0, rows] - torch.from_numpy(g["desc1_rows"])).abs().max()))
    es = max(float((sc[0, rows] - torch.from_numpy(g["scores_rows"])).abs().max()),
             float((sc[0, :, 0] - torch.from_numpy(g["scores_col0"])).abs().max()))
    mi, mj = g["matches_all"][:, 0], g["matches_all"][:, 1]
    dm = (sc[0, mi, mj].double() - torch.from_numpy(np.log(g["mscores_all"].astype(np.float64)))).abs()
    return {"desc": round(ed, 5), "scores": round(es, 4), "matched": round(float(dm.max()), 4),
            "matched_p99": round(float(np.quantile(dm.numpy(), 0.99)), 4),
            "matched_mean": round(float(dm.mean()), 5)}


def main():
    dtype = sys.argv[1] if len(sys.argv) > 1 else "float16"
    dt = getattr(torch, dtype)
    dev = torch.device("cuda:0")
    lib = _lib.load()
    g = np.load(os.path.join(tm.GOLD, f"{NAME}.npz"))
    meta = tm.SWEEP[NAME]
    model, pair = tm._sweep_model(NAME)
    model = model.to(dev, dt)

    base = {}

    def run(m, inputs, slot=0):
        with torch.no_grad():
            d0, d1, sc = m(*(t.to(dev, dt) for t in inputs))
            torch.cuda.synchronize()
        outs = tuple(t[slot:slot + 1].float().cpu() for t in (d0, d1, sc))
        e = errs(g, *outs)
        if base:  # against the default single-pair forward, every element (test_matcher's batched-vs-single check)
            e["vs_single_desc"] = round(max(float((outs[0] - base["d0"]).abs().max()), float((outs[1] - base["d1"]).abs().max())), 5)
            e["vs_single_scores"] = round(float((outs[2] - base["sc"]).abs().max()), 4)
        else:
            base.update(d0=outs[0], d1=outs[1], sc=outs[2])
        return e

    def out(kind, **kw):
        print(json.dumps({"dtype": dtype, "kind": kind, **kw}), flush=True)

    prev_mode = lightglue_amd.set_stream_mode(1)
    out("single", plan="default", **run(model, pair))
    for hint in (2, 3):
        lib.mha_hd64_set_concurrency_hint(hint)
        out("single", plan=f"concurrency hint {hint}", **run(model, pair))
    lib.mha_hd64_set_concurrency_hint(1)
    for P in (4, 8):
        ps = [matcher.synthetic_pair(meta["seed"] + 100 + i, meta["m"], meta["n"], overlap=meta["overlap"])
              for i in range(P)]
        for slot in (0, P // 2):
            qs = list(ps)
            qs[slot] = pair
            batch = tuple(torch.cat([p[j] for p in qs], 0) for j in range(4))
            for mode in (0, 1):
                lightglue_amd.set_stream_mode(mode)
                out("batched", P=P, slot=slot, stream_mode=mode, **run(model, batch, slot))
    lightglue_amd.set_stream_mode(1)

    base_attn = model.attention

    def perturbed(seed):
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed)

        def attn(calls):
            outs = base_attn(calls)
            res = []
            for o in outs:
                if o.dtype == torch.float16:
                    bits = o.view(torch.int16)
                    sel = torch.rand(o.shape, generator=gen, device=dev) < 0.1
                    step = torch.where(torch.rand(o.shape, generator=gen, device=dev) < 0.5, 1, -1).to(torch.int16)
                    o = torch.where(sel & (bits & 0x7FFF != 0), bits + step, bits).view(torch.float16)
                else:  # fp32 model: a relative 2^-11 nudge (an fp16 ulp)
                    sel = torch.rand(o.shape, generator=gen, device=dev) < 0.1
                    o = torch.where(sel, o * (1 + 2.0 ** -11 * torch.sign(torch.rand(o.shape, generator=gen, device=dev) - 0.5)), o)
                res.append(o)
            return res
        return attn

    ms, vs, vd = [], [], []
    for seed in range(8):
        model.attention = perturbed(seed)
        e = run(model, pair)
        ms.append(e["matched"])
        vs.append(e["vs_single_scores"])
        vd.append(e["vs_single_desc"])
        out("ulp", seed=seed, **e)
    model.attention = base_attn
    out("ulp_summary", matched_min=min(ms), matched_max=max(ms), matched_median=float(np.median(ms)),
        vs_single_scores_max=max(vs), vs_single_desc_max=max(vd))
    lightglue_amd.set_stream_mode(prev_mode)


if __name__ == "__main__":
    main()

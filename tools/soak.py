"""Soak test: sustained load on the shipped path for a fixed wall time, checking that every output
stays bitwise equal to the first one computed. Rotates through (a) 1000 headline plugin enqueues
(1x4x1024^2 fp16, bindings prepared once), (b) the batched launcher at 8 calls (streaming or
single-pass kernel by the planner), (c) the fp16 matcher forward at P = 1 and P = 16 pairs (graph
replays), (d) two streams of headline calls with separate workspaces; with "full" also (e) the
plugin's Float path, (f) grouped launches of four ragged calls, (g) four streams under the
concurrency hint 4, (h) the fp32 matcher at P = 1. A progress line every ~30 s, one JSON line at the
end; exit status 1 on any mismatch.

    python tools/soak.py [seconds=480] [basic|full]
"""
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

from lightglue_amd import matcher, mha_hd64_batched, mha_hd64_grouped, plugin, set_concurrency_hint, synth  # noqa: E402


def digest(*ts):
    h = hashlib.sha256()
    for t in ts:
        h.update(t.detach().contiguous().view(torch.uint8).cpu().numpy().tobytes())
    return h.hexdigest()[:16]


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 480.0
    full = len(sys.argv) > 2 and sys.argv[2] == "full"
    dev = torch.device("cuda:0")
    st, st2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in synth.qkv(21, 1024, 1024))
    out, out2 = torch.empty_like(q), torch.empty_like(q)
    with torch.cuda.stream(st):
        call = plugin.bound_enqueue(q, k, v, out)
    with torch.cuda.stream(st2):
        call2 = plugin.bound_enqueue(q, k, v, out2)
    qb, kb, vb = (torch.from_numpy(x).to(dev).half().contiguous() for x in synth.qkv(22, 1024, 1024, batch=8))
    ob = torch.empty_like(qb)
    model = matcher.LightGlueMatcher(n_layers=9).eval()
    model.load_state_dict(matcher.seeded_state_dict(7, 9), strict=True)
    model = model.to(dev, torch.float16)
    graphs = {}

    def capture(key, mdl, P, dt):
        ps = [matcher.synthetic_pair(80 + i, 1024, 1024) for i in range(P)]
        batch = tuple(torch.cat([p[j] for p in ps], 0).to(dev, dt) for j in range(4))
        with torch.no_grad(), torch.cuda.stream(st):
            for _ in range(2):
                mdl(*batch)
            st.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                res = mdl(*batch)
        graphs[key] = (g, batch, res, P)

    capture("P1", model, 1, torch.float16)
    capture("P16", model, 16, torch.float16)
    if full:
        model32 = matcher.LightGlueMatcher(n_layers=9).eval()
        model32.load_state_dict(matcher.seeded_state_dict(7, 9), strict=True)
        capture("fp32_P1", model32.to(dev, torch.float32), 1, torch.float32)
        q32, k32, v32 = (t.float().contiguous() for t in (q, k, v))
        o32 = torch.empty_like(q32)
        with torch.cuda.stream(st):
            call32 = plugin.bound_enqueue(q32, k32, v32, o32)
        ragged = [(600, 1000), (1000, 600), (333, 777), (1024, 1024)]
        gcalls = [tuple(torch.from_numpy(x).to(dev).half().contiguous() for x in synth.qkv(30 + i, a, b))
                  for i, (a, b) in enumerate(ragged)]
        gouts = [torch.empty_like(c[0]) for c in gcalls]
        hst = [torch.cuda.Stream(dev) for _ in range(4)]
        hq = [tuple(torch.from_numpy(x).to(dev).half().contiguous() for x in synth.qkv(40 + i, 1024, 1024)) for i in range(4)]
        ho = [torch.empty_like(t[0]) for t in hq]

    def work(name):
        if name == "headline":
            with torch.cuda.stream(st):
                for _ in range(1000):
                    call()
            st.synchronize()
            return digest(out), 1000
        if name == "batched8":
            with torch.cuda.stream(st):
                for _ in range(200):
                    mha_hd64_batched(qb, kb, vb, out=ob)
            st.synchronize()
            return digest(ob), 200 * 8
        if name == "two_streams":
            for s, c in ((st, call), (st2, call2)):
                with torch.cuda.stream(s):
                    for _ in range(500):
                        c()
            st.synchronize()
            st2.synchronize()
            return digest(out, out2), 1000
        if name == "float_path":
            with torch.cuda.stream(st):
                for _ in range(500):
                    call32()
            st.synchronize()
            return digest(o32), 500
        if name == "grouped_ragged":
            with torch.cuda.stream(st):
                for _ in range(200):
                    mha_hd64_grouped(gcalls, outs=gouts)
            st.synchronize()
            return digest(*gouts), 200 * len(gcalls)
        if name == "hint4":
            prev = set_concurrency_hint(4)
            try:
                for i, s_ in enumerate(hst):
                    with torch.cuda.stream(s_):
                        for _ in range(250):
                            plugin.mha_hd64(*hq[i], out=ho[i])
                for s_ in hst:
                    s_.synchronize()
            finally:
                set_concurrency_hint(prev)
            return digest(*ho), 1000
        g, _, res, P = graphs[name]
        for _ in range(20):
            g.replay()
        st.synchronize()
        ts = list(res.values()) if isinstance(res, dict) else list(res)
        return digest(*[t for t in ts if torch.is_tensor(t)]), 20 * P

    names = ["headline", "batched8", "two_streams", "P1", "P16"] + (
        ["float_path", "grouped_ragged", "hint4", "fp32_P1"] if full else [])
    first, counts, bad = {}, {n: 0 for n in names}, []
    t0 = last = time.time()
    rounds = 0
    while time.time() - t0 < seconds:
        for nme in names:
            d, units = work(nme)
            if nme not in first:
                first[nme] = d
            elif d != first[nme]:
                bad.append({"work": nme, "round": rounds, "digest": d, "first": first[nme]})
            counts[nme] += units
        rounds += 1
        if time.time() - last > 30:
            last = time.time()
            print(json.dumps({"elapsed_s": round(last - t0, 1), "rounds": rounds, "mismatches": len(bad)}), flush=True)
    print(json.dumps({"soak_s": round(time.time() - t0, 1), "rounds": rounds, "units": counts,
                      "units_meaning": "attention calls (headline, batched8, two_streams, float_path, grouped_ragged, "
                                       "hint4) / image pairs (P1, P16, fp32_P1)",
                      "digests": first, "mismatches": bad, "ok": not bad}), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

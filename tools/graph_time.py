"""Diagnostic: per-launch time of library variants, measured by hipGraph replay (no event overhead).

    python tools/graph_time.py lib1.so [lib2.so ...]

For each library (the shipped one or lib/exp/ ablation / experiment builds) and each case, K
launches are captured back to back into one graph (stream-ordered, as bench.py does) and the
graph is replayed; time per launch = replay time / K. Cases: the single 1x4x1024x1024 call
(main kernel only, and main + combine) with the planned shape, and a batched launch. Also
reports a 1-element torch kernel in the same harness (the floor of a dependent launch).
Variants are interleaved (A/B/A/B) and the median of several rounds is printed as JSON."""
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

from lightglue_amd import _lib, synth  # noqa: E402

K = 200
ROUNDS = 7


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    for name, (args, res) in list(_lib.SIGNATURES.items()) + list(_lib.HOOKS.items()):
        if not hasattr(lib, name):  # an older library build
            continue
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    return lib


def graph_of(fn, stream):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        fn()  # warm
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=stream):
            for _ in range(K):
                fn()
    return g


def time_graph(g, stream):
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    with torch.cuda.stream(stream):
        g.replay()
    e.record(stream)
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / K  # us per launch


def main():
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
    libs = [(os.path.basename(p), load(p)) for p in sys.argv[1:]]
    cases = []
    shapes = [("call", 1, 1024, 1024, 0, 0, 0), ("b8", 8, 1024, 1024, 0, 0, 0)]
    extra = os.environ.get("GT_SHAPES")  # e.g. "2,2,4;4,2,8" forced (q_waves,kv_waves,splits) for the call
    if extra:
        for s in extra.split(";"):
            qw, kw, sp = (int(x) for x in s.split(","))
            shapes.append((f"call_{qw}x{kw}s{sp}", 1, 1024, 1024, qw, kw, sp))
    cases_env = os.environ.get("GT_CASES")  # "name:B:nq:nkv:qw:kw:sp;..." replaces the default list
    if cases_env:
        shapes = []
        for c in cases_env.split(";"):
            f = c.split(":")
            shapes.append((f[0],) + tuple(int(x) for x in f[1:]))
    data = {}
    for name, b, nq, nkv, qw, kw, sp in shapes:
        qn, kn, vn = synth.qkv(5, nq, nkv, batch=b)
        q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in (qn, kn, vn))
        data[name] = (q, k, v, torch.empty_like(q))
    for lname, lib in libs:
        for name, b, nq, nkv, qw, kw, sp in shapes:
            q, k, v, o = data[name]
            tags = ((1, "main"), (3, "all"), (2, "comb"), (3, "all2k")) if os.environ.get("GT_ALL") else ((1, "main"),)
            for mask, tag in tags:
                # "all": the production form (split calls combine inside the main launch when the
                # library has that path); "all2k": main kernel + combine kernel
                fused = hasattr(lib, "mha_hd64_set_fused_combine")
                if fused:
                    lib.mha_hd64_set_fused_combine(0 if tag == "all2k" else 1)
                def fn(lib=lib, q=q, k=k, v=v, o=o, b=b, nq=nq, nkv=nkv, mask=mask, qw=qw, kw=kw, sp=sp):
                    st = lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), b, 4,
                                                    nq, nkv, 0, 0, qw, kw, sp, ws.data_ptr(), ws.numel(),
                                                    torch.cuda.current_stream().cuda_stream, mask)
                    assert st == 0
                cases.append((f"{lname}:{name}:{tag}", graph_of(fn, stream)))
                if fused:
                    lib.mha_hd64_set_fused_combine(1)
    x = torch.zeros(1, device=dev)
    cases.append(("torch_add1", graph_of(lambda: x.add_(1), stream)))
    res = {c: [] for c, _ in cases}
    for _ in range(ROUNDS):
        for c, g in cases:
            res[c].append(time_graph(g, stream))
    print(json.dumps({c: round(statistics.median(v), 3) for c, v in res.items()}, indent=0), flush=True)


if __name__ == "__main__":
    main()

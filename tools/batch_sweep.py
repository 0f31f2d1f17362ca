"""Diagnostic: per-launch graph-replay time of batched 1xBx4xNxN launches under the planner's
default plan (code 0), the 32-row single-pass kernel (21), the 16-row one (22) and the
streaming kernel (23); best of three interleaved passes.
    python tools/batch_sweep.py [BxN ...]"""
import json, os, sys
REPO = "/root/repo" if os.path.exists("/root/repo") else os.getcwd()
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd"), os.path.join(REPO, "tools")]
import torch
from lightglue_amd import _lib, synth
from direct_check import per_launch_us
lib = _lib.load()
dev = torch.device("cuda:0")
ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
res = {}
# cases: BxN (Nq = Nkv = N) or BxNQxNKV
cases = [tuple(int(x) for x in c.split("x")) for c in sys.argv[1:]] or [(8, 1024), (2, 1024), (4, 1024), (8, 512), (2, 512)]
for case in cases:
    batch, n = case[0], case[1]
    nkv = case[2] if len(case) > 2 else n
    qn, kn, vn = synth.qkv(5, n, nkv, batch=batch)
    q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in (qn, kn, vn))
    o = torch.empty_like(q)
    def run(code):
        st = lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), batch, 4, n, nkv, 0, 0,
                                        code, 0, 0, ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream, 3)
        assert st == 0
    row = {}
    for rep in range(3):  # three interleaved passes, the best of each (the first measured pays a warm-up)
        for c in (0, 21, 22, 23):
            try:
                t = round(per_launch_us(lambda: run(c)), 3)
                row[str(c)] = t if row.get(str(c)) is None else min(row[str(c)], t)
            except AssertionError:  # plan not applicable to this shape
                row[str(c)] = None
    res[f"b{batch}_n{n}" + (f"x{nkv}" if nkv != n else "")] = row
print(json.dumps(res))

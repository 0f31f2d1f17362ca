"""Scratch diagnostic: which output rows are NaN for a NaN in one Q element, per plan."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import numpy as np, torch
from lightglue_amd import _lib, synth
lib = _lib.load()
dev = torch.device("cuda:0")
ws = torch.empty(1 << 22, dtype=torch.uint8, device=dev)
n = 100
for val in (np.nan, np.inf):
    qn, kn, vn = synth.qkv(4711 + n, n, n)
    qn[0, 1, 33, 5] = val
    q16, k16, v16 = (synth.round_f16(a) for a in (qn, kn, vn))
    q, k, v = (torch.from_numpy(a).to(dev).half().contiguous() for a in (q16, k16, v16))
    for code, kw, sp in ((21, 0, 0), (23, 0, 0), (4, 2, 0), (22, 0, 0)):
        o = torch.empty(q.shape, dtype=torch.float16, device=dev)
        st = lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), 1, 4, n, n, 0, 0,
                                        code, kw, sp, ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream, 3)
        torch.cuda.synchronize()
        on = torch.isnan(o.float().cpu())
        idx = torch.nonzero(on.any(-1)).tolist()
        print(val, code, kw, st, "nan rows (b,h,row):", idx, "row33 head1:", o[0, 1, 33, :3].tolist(), flush=True)

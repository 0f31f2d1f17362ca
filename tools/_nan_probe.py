"""Scratch diagnostic: NaN propagation per plan (a NaN in one Q / K / V element)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import numpy as np, torch
from lightglue_amd import _lib, synth
lib = _lib.load()
dev = torch.device("cuda:0")
ws = torch.empty(1 << 22, dtype=torch.uint8, device=dev)
for b, n in ((1, 1024), (2, 1024), (2, 256), (1, 100)):
    for where in "qkv":
        qn, kn, vn = synth.qkv(4711 + n, n, n, batch=b)
        x = {"q": qn, "k": kn, "v": vn}[where]
        x[b - 1, 1, n // 3, 5] = np.nan
        q16, k16, v16 = (synth.round_f16(a) for a in (qn, kn, vn))
        qf, kf, vf = (torch.from_numpy(a) for a in (q16, k16, v16))
        ref = torch.softmax((qf @ kf.transpose(-1, -2)) * 0.125, -1) @ vf
        q, k, v = (torch.from_numpy(a).to(dev).half().contiguous() for a in (q16, k16, v16))
        row = {"b": b, "n": n, "where": where, "ref_nan": int(torch.isnan(ref).sum())}
        for code, kw, sp in ((0, 0, 0), (21, 0, 0), (22, 0, 0), (23, 0, 0), (4, 2, 0), (4, 1, 0), (2, 2, 2), (1, 8, 0), (12, 2, 0)):
            o = torch.empty(q.shape, dtype=torch.float16, device=dev)
            st = lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), b, 4, n, n, 0, 0,
                                            code, kw, sp, ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream, 3)
            torch.cuda.synchronize()
            if st:
                row[f'{code}/{kw}/{sp}'] = None
                continue
            on = torch.isnan(o.float().cpu())
            row[f'{code}/{kw}/{sp}'] = (int(on.sum()), bool(torch.equal(on, torch.isnan(ref))))
            if where == "q" and code == 23:
                row["row23"] = o[b - 1, 1, n // 3, :4].float().cpu().tolist()
        print(row, flush=True)

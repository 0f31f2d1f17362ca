"""Diagnostic: in-launch (ticketed) split combine vs the combine kernel, per shape: differing
elements, max-abs difference, and max-abs error of each against the C oracle on sampled rows."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

from lightglue_amd import _lib, synth  # noqa: E402
from oracle import oracle  # noqa: E402

SHAPES = [(1024, 1024, 2, 4, 0), (1024, 1024, 2, 2, 4), (300, 2048, 2, 2, 3), (100, 1000, 12, 2, 3),
          (64, 4000, 2, 4, 0), (33, 65, 4, 1, 2), (257, 1000, 4, 2, 2), (1024, 1024, 1, 8, 0), (300, 2000, 1, 8, 0),
          (100, 1000, 1, 4, 0)]


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
    for out_dt in (torch.float16, torch.float32):
        for nq, nkv, qw, kw, sp in SHAPES:
            qn, kn, vn = synth.qkv(77 + nq + nkv, nq, nkv)
            q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in (qn, kn, vn))
            outs = []
            for fused in (0, 1):
                lib.mha_hd64_set_fused_combine(fused)
                ws.fill_(255)  # NaN partials: a stale or missing read shows as NaN
                o = torch.full(q.shape, float("nan"), dtype=out_dt, device=dev)
                st = lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), 1, 4, nq,
                                                nkv, 0, int(out_dt == torch.float32), qw, kw, sp, ws.data_ptr(),
                                                ws.numel(), torch.cuda.current_stream().cuda_stream, 3)
                assert st == 0, _lib.last_error()
                outs.append(o.float())
            torch.cuda.synchronize()
            d = (outs[0] - outs[1]).abs()
            rows = np.unique(np.r_[np.arange(0, nq, max(1, nq // 32)), nq - 1])
            ref = oracle.attention_c(np.ascontiguousarray(synth.round_f16(qn)[:, :, rows]), synth.round_f16(kn),
                                     synth.round_f16(vn))
            e = [float(np.abs(x.cpu().numpy()[:, :, rows] - ref).max()) for x in outs]
            idx = torch.nonzero(d > 0)[:4].tolist()
            for i in idx:
                i = tuple(i)
                print("   at", i, "2k", float(outs[0][i]), "fused", float(outs[1][i]))
            print(out_dt, (nq, nkv, qw, kw, sp), "ndiff", int((d > 0).sum()), "of", d.numel(),
                  "maxdiff", float(d.max()), "nan", int(torch.isnan(outs[1]).sum()), "err2k/fused", e, flush=True)
    lib.mha_hd64_set_fused_combine(1)


if __name__ == "__main__":
    main()

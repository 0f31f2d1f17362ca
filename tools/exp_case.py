"""Diagnostic: run one forced plan against the C oracle with a chosen library build.
    python tools/exp_case.py <lib.so> nq nkv q_waves kv_waves splits"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

from lightglue_amd import _lib, synth  # noqa: E402
from oracle import oracle  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
lib = _lib.load()
nq, nkv, qw, kw, sp = (int(x) for x in sys.argv[2:7])
qn, kn, vn = synth.qkv(1000 + nq + 7 * nkv, nq, nkv)
q16, k16, v16 = (synth.round_f16(x) for x in (qn, kn, vn))
ref = oracle.attention_c(q16, k16, v16)
dev = torch.device("cuda:0")
q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in (q16, k16, v16))
ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
o = torch.full(q.shape, float("nan"), dtype=torch.float16, device=dev)
st = lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), 1, 4, nq, nkv, 0, 0, qw, kw,
                                sp, ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream, 3)
torch.cuda.synchronize()
got = o.float().cpu().numpy()
err = np.abs(got - ref)
print(os.path.basename(sys.argv[1]), (nq, nkv, qw, kw, sp), "status", st, "maxerr %.3e" % err.max(),
      "rows bad:", int((err.max(axis=-1) > 1e-2).sum()), "of", nq * 4,
      "first bad row per head:", [int(np.argmax(err[0, h].max(-1) > 1e-2)) for h in range(4)])

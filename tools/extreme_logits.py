"""Diagnostic: max-abs error vs the C oracle of each plan on extreme logits (|q| x 40)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import numpy as np, torch
from lightglue_amd import _lib, synth
from oracle import oracle
oracle.build()
lib = _lib.load()
dev = torch.device("cuda:0")
ws = torch.empty(1 << 22, dtype=torch.uint8, device=dev)
for scale in (4, 10, 20, 40):
    nq, nkv, b = 256, 700, 3
    qn, kn, vn = synth.qkv(4242, nq, nkv, batch=b)
    qn[:, :, :64] = -scale * np.abs(qn[:, :, :64]); kn = np.abs(kn)
    q16, k16, v16 = (synth.round_f16(x) for x in (qn, kn, vn))
    ref = oracle.attention_c(q16, k16, v16)
    q, k, v = (torch.from_numpy(x).to(dev).half().contiguous() for x in (q16, k16, v16))
    row = {"scale": scale}
    for code in (0, 21, 22, 23, 1):
        o = torch.empty(q.shape, dtype=torch.float32, device=dev)
        kw = 8 if code == 1 else 0
        st = lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), b, 4, nq, nkv, 0, 1,
                                        code, kw, 0, ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream, 3)
        torch.cuda.synchronize()
        row[code] = None if st else round(float(np.abs(o.cpu().numpy() - ref).max()), 5)
    print(row, flush=True)

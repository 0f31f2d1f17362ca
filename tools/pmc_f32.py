"""Profiling driver for the Float boundary: fp32 Q/K/V -> fp32 O calls of 1x4xNqxNkv through the
plugin path, eager, --steps times, with set_f32_inkernel(mode): 0 = convert launch + fp16 kernel,
1 = in-kernel rounding where the planner allows it (one-pass forms), 2 = also the two-pass forms.
    python tools/pmc_f32.py <mode> [nq] [nkv] [steps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

import lightglue_amd  # noqa: E402
from lightglue_amd import _lib, synth  # noqa: E402

mode = int(sys.argv[1])
nq = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
nkv = int(sys.argv[3]) if len(sys.argv) > 3 else 2048
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 50
_lib.load().mha_hd64_set_f32_inkernel(mode)
dev = torch.device("cuda:0")
q, k, v = (torch.from_numpy(x).to(dev).float().contiguous() for x in synth.qkv(11, nq, nkv))
o = torch.empty_like(q)
for _ in range(steps):
    lightglue_amd.mha_hd64(q, k, v, out=o)
torch.cuda.synchronize()

"""Profiling driver: lg_linear_cat_ffn at P pairs of n keypoints in form `mode` (lg_linear_set_ffn_fused:
0 two calls, 1 the one-launch ffn_rows_kernel), launched `steps` times eagerly, for rocprofv3 --pmc /
--kernel-trace passes.      python tools/ffn_driver.py [P] [n] [mode] [steps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

from lightglue_amd import _lib  # noqa: E402
from lightglue_amd import matcher as mt  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 1
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
mode = int(sys.argv[3]) if len(sys.argv) > 3 else 1
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
lib = _lib.load()
dev, dt, h = torch.device("cuda:0"), torch.float16, 4
g = torch.Generator().manual_seed(3)
rnd = lambda *s: torch.randn(*s, generator=g).to(dev, dt)  # noqa: E731
with torch.no_grad():
    x = rnd(1, P * 2 * n, 256) * 0.5
    c0, c1 = rnd(P, h, n, 64), rnd(P, h, n, 64)
    w, b, w2, b2 = rnd(512, 512) * 0.05, rnd(512) * 0.1, rnd(256, 512) * 0.05, rnd(256) * 0.1
    ln = torch.nn.LayerNorm(512).to(dev, dt)
    wp = mt.ffn_pack(w, w2)
    lib.lg_linear_set_ffn_fused(mode)
    for _ in range(steps):
        mt._Hip.ffn(x, c0, c1, w, b, ln, w2, b2, wp)
    torch.cuda.synchronize()
print(f"ffn P={P} n={n} mode={mode}: {steps} calls")

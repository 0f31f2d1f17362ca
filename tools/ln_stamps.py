"""Diagnostic: where the one-launch FFN kernel's time goes (linear_ln_kernel stamps build,
-DLG_LN_STAMPS: per wave, s_memtime cycles of chained segments; see csrc/lightglue_linear.hip).

    MHA_HD64_LIB=lib/ab/libmha_hd64_lnstamps.so python tools/ln_stamps.py [P=16] [n=1024]
"""
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lightglue_amd import _lib  # noqa: E402
from lightglue_amd import matcher as mt  # noqa: E402


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    lib = _lib.load()
    fn = lib.lg_diag_ln_stamps
    fn.restype = ctypes.c_int32
    fn.argtypes = [ctypes.c_void_p]
    dev, dt, h = torch.device("cuda:0"), torch.float16, 4
    M = P * 2 * n
    x = torch.randn(1, M, 256, device=dev, dtype=dt) * 0.5
    c0 = torch.randn(P, h, n, 64, device=dev, dtype=dt)
    c1 = torch.randn(P, h, n, 64, device=dev, dtype=dt)
    w, b = torch.randn(512, 512, device=dev, dtype=dt) * 0.05, torch.randn(512, device=dev, dtype=dt)
    ln = torch.nn.LayerNorm(512).to(dev, dt)
    names = ["prologue", "kstep_wait_barrier", "kstep_issue_mfma", "epi_stats", "epi_gelu_store"]
    rows = []
    for rep in range(6):
        for _ in range(3):  # back to back, as in a forward
            mt._Hip.linear_cat_ln_gelu(x, c0, c1, w, b, ln)
        torch.cuda.synchronize()
        buf = np.zeros(256 * 8 * 8, dtype=np.uint64)
        assert fn(buf.ctypes.data) == 0
        st = buf.reshape(256, 8, 8)
        used = st[:, :, 5] > 0
        seg = {nm: float(np.median(st[:, :, k][used])) for k, nm in enumerate(names)}
        seg["total"] = float(np.median(st[:, :, 5][used]))
        seg["total_max"] = float(np.max(st[:, :, 5][used]))
        seg["tiles_per_wg"] = float(np.median(st[:, :, 6][used]))
        rows.append(seg)
    out = {k: round(statistics.median(r[k] for r in rows)) for k in rows[0]}
    print(json.dumps({"P": P, "n": n, "M": M, "cycles_median_per_wave": out}))


if __name__ == "__main__":
    main()

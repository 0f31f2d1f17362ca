"""Diagnostic: where ffn_rows_kernel's time goes (stamps build, -DLG_FR_STAMPS: per wave, s_memtime
cycles of chained segments; see csrc/lightglue_linear.hip).

    MHA_HD64_LIB=lib/ab/libmha_hd64_frstamps.so python tools/fr_stamps.py [P=1] [n=1024] [kind=0]

kind 0: lg_linear_cat_ffn; 1 / 2 / 3: lg_linear_cat_ffn_proj with the split2 / qkv / plain projection
(segment "phase3": the projection and its epilogue). The kernel is the one lg_linear_cat_ffn picks
by size (ffn_rows16_kernel up to 4,096 rows).
"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lightglue_amd import _lib  # noqa: E402
from lightglue_amd import matcher as mt  # noqa: E402


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    kind = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    lib = _lib.load()
    fn = lib.lg_diag_fr_stamps
    fn.restype, fn.argtypes = ctypes.c_int32, [ctypes.c_void_p]
    dev, dt, h = torch.device("cuda:0"), torch.float16, 4
    M = P * 2 * n
    g = torch.Generator().manual_seed(3)
    rnd = lambda *s: torch.randn(*s, generator=g).to(dev, dt)  # noqa: E731
    x = rnd(1, M, 256) * 0.5
    c0, c1 = rnd(P, h, n, 64), rnd(P, h, n, 64)
    w, b, w2, b2 = rnd(512, 512) * 0.05, rnd(512) * 0.1, rnd(256, 512) * 0.05, rnd(256) * 0.1
    ln = torch.nn.LayerNorm(512).to(dev, dt)
    n3 = {0: 0, 1: 512, 2: 768, 3: 512}[kind]
    w3, b3 = (rnd(n3, 256) * 0.06, rnd(n3) * 0.1) if n3 else (None, None)
    wp = mt.ffn_pack(w, w2, w3)
    ang = rnd(1, M, 32).float()
    cs, sn = (torch.cos(ang).repeat_interleave(2, -1).to(dt).contiguous(), torch.sin(ang).repeat_interleave(2, -1).to(dt).contiguous())

    def call():
        if kind == 0:
            return mt._Hip.ffn(x, c0, c1, w, b, ln, w2, b2, wp)
        return mt._Hip.ffn_proj(x, c0, c1, b, ln, b2, wp, kind, b3, (n, n, P), cs, sn, 384)

    names = ["prologue", "phase1", "layernorm_gelu", "phase2", "epilogue", "total", "entry", "phase3"]
    mode = lib.lg_linear_set_ffn_fused(1)  # (the form in force; restored at once)
    lib.lg_linear_set_ffn_fused(mode)
    rows16 = mode == 3 or (mode != 2 and M <= 4096)
    wgs = min(256, (M + 15) // 16 if rows16 else (M + 31) // 32 if M <= 8192 else (M + 63) // 64)  # (the first 256)
    rows = []
    for rep in range(6):
        for _ in range(3):  # back to back, as in a forward
            call()
        torch.cuda.synchronize()
        buf = np.zeros(256 * 8 * 8, dtype=np.uint64)
        assert fn(buf.ctypes.data) == 0
        a = buf.reshape(256, 8, 8)[:wgs].astype(np.int64)
        if rep:
            rows.append(a)
    a = np.concatenate(rows, 0)
    if rows16:  # (ffn_rows16_kernel: slot 6 is the phase-3 epilogue; slot 7 its MFMA loop)
        names = names[:6] + ["phase3_epilogue", "phase3_mfma"]
    out = {"P": P, "n": n, "M": M, "kind": kind, "kernel": "ffn_rows16" if rows16 else "ffn_rows", "workgroups": wgs,
           "median_cycles": {k: float(np.median(a[:, :, i])) for i, k in enumerate(names) if k != "entry"},
           "max_total": float(a[:, :, 5].max()),
           **({} if rows16 else {"entry_spread_cycles": float(np.median(a[:, :, 6].max(1) - a[:, :, 6].min(1)))})}
    # per workgroup: how far apart its 8 waves finish phase 1 (cumulative prologue + phase 1), the
    # LayerNorm barrier's wait for the slowest
    ends = a[:, :, 0] + a[:, :, 1]
    out["phase1_end_spread_cycles"] = float(np.median(ends.max(1) - ends.min(1)))
    out["phase1_end_slowest_wave"] = int(np.bincount(ends.argmax(1), minlength=8).argmax())
    if not rows16:
        last = rows[-1]
        ent = last[:, :, 6]
        out["launch_entry_spread_cycles"] = float(ent.max() - ent.min())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

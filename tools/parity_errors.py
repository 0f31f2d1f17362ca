"""Observed max-abs errors of the three kernel paths on every golden fixture (calibrates the
regression bounds in tests/test_gpu_parity.py). One JSON line per case."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
from conftest import golden_cases, load_golden  # noqa: E402
from lightglue_amd import mha_hd64, mha_hd64_batched  # noqa: E402

dev = torch.device("cuda:0")
for name in golden_cases():
    g = load_golden(name)
    t = lambda x, dt: torch.from_numpy(np.ascontiguousarray(x)).to(dev).to(dt).contiguous()  # noqa: E731
    q, k, v = (t(x, torch.float16) for x in (g["q"], g["k"], g["v"]))
    o16 = mha_hd64(q, k, v).float().cpu().numpy()[:, :, g["rows"]]
    o32 = mha_hd64_batched(q, k, v, out_dtype=torch.float32).cpu().numpy()[:, :, g["rows"]]
    of = mha_hd64(*(t(x, torch.float32) for x in (g["q"], g["k"], g["v"]))).cpu().numpy()[:, :, g["rows"]]
    r16, r32 = g["o_ref16"].astype(np.float64), g["o_ref32"].astype(np.float64)
    d16 = np.abs(o16 - r16)
    print(json.dumps({"case": name, "q_std": float(g["q_std"]), "half_maxabs": float(d16.max()),
                      "half_excess_over_halfulp": float((d16 - np.abs(r16) * 2.0 ** -11).max()),
                      "f16in_f32out_maxabs": float(np.abs(o32 - r16).max()),
                      "float_path_maxabs": float(np.abs(of - r32).max()),
                      "max_abs_v": float(np.abs(g["v"]).max())}), flush=True)

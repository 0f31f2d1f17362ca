"""Diagnostic: max-abs errors of the GPU matcher (fp32 / fp16 models) vs the reference fixtures."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_matcher as tm  # noqa: E402
from lightglue_amd.matcher import filter_matches  # noqa: E402

for name in tm.CASES:
    g = np.load(os.path.join(tm.GOLD, f"{name}.npz"))
    for dt in ("float32", "float16"):
        _, d0, d1, sc = tm._gpu_run(name, getattr(torch, dt))
        e0 = float((d0 - torch.from_numpy(g["desc0"])).abs().max())
        e1 = float((d1 - torch.from_numpy(g["desc1"])).abs().max())
        es = float((sc - torch.from_numpy(g["scores"])).abs().max())
        got = tm._match_set(filter_matches(sc, 0.0)[0].numpy())
        ref = tm._match_set(g["matches_all"])
        print(f"{name:20s} {dt:8s} desc0 {e0:.4g} desc1 {e1:.4g} scores {es:.4g} "
              f"matches {len(got & ref)}/{len(ref)} (got {len(got)})", flush=True)

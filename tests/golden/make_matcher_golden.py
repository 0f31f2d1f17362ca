"""Golden fixtures for the LightGlue matcher around the op.

Run in the build container only (it reads /root/reference, absent on the GPU box):

    python tests/golden/make_matcher_golden.py [name ...]    (no names: every case)

Builds the reference model ``LightGlue(features=None, n_layers=L)`` from
/root/reference/lightglue_pytorch_no_plugin/lightglue.py (module file loaded directly; the
package __init__ needs cv2), loads the deterministic weights
``lightglue_amd.matcher.seeded_state_dict(seed, L)`` (strict: the parameter names must match),
runs ``forward(kpts0, kpts1, desc0, desc1)`` in float32 on CPU on
``lightglue_amd.matcher.synthetic_pair(seed, m, n)`` and the reference ``filter_matches``
(thresholds 0.1 and 0.0); SWEEP_CASES do the same at the BASELINE sweep sizes on pairs with
true correspondences and keep a row subset plus checksums. Weights and inputs are regenerated bit-exactly from their seeds, so only the
outputs are stored (with a sha256 of the regenerated inputs + weights).
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd"))
from lightglue_amd import matcher  # noqa: E402

REF = "/root/reference/lightglue_pytorch_no_plugin/lightglue.py"

# name: (seed, n_layers, m, n)
CASES = {
    "match_l2_64x48": (1, 2, 64, 48),
    "match_l9_120x97": (2, 9, 120, 97),
    "match_l3_300x257": (3, 3, 300, 257),
}
# BASELINE configs[3] sweep sizes, 9 layers, pairs with `overlap` true correspondences
# (matcher.synthetic_pair(..., overlap)); only a row subset of the m x n log-assignment, its first
# column and per-row / per-column sums are stored.
# name: (seed, n_layers, m, n, overlap, row_stride)
SWEEP_CASES = {
    "sweep_l9_512x512": (11, 9, 512, 512, 384, 16),
    "sweep_l9_1024x1024": (12, 9, 1024, 1024, 768, 32),
    "sweep_l9_2048x2048": (13, 9, 2048, 2048, 1536, 64),
}


def digest(sd, pair) -> str:
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(sd[k].numpy().tobytes())
    for t in pair:
        h.update(t.numpy().tobytes())
    return h.hexdigest()


def _merge_index(path, new):
    old = {}
    if os.path.exists(path):
        with open(path) as f:
            old = json.load(f)
    old.update(new)
    with open(path, "w") as f:
        json.dump(old, f, indent=1, sort_keys=True)


def main():
    want = set(sys.argv[1:])
    pick = lambda name: not want or name in want  # noqa: E731
    spec = importlib.util.spec_from_file_location("lg_ref", REF)
    lg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(lg)
    torch.manual_seed(0)
    index = {}
    for name, (seed, layers, m, n) in CASES.items():
        if not pick(name):
            continue
        model = lg.LightGlue(features=None, n_layers=layers).eval()
        sd = matcher.seeded_state_dict(seed, layers)
        model.load_state_dict(sd, strict=True)
        pair = matcher.synthetic_pair(seed, m, n)
        with torch.no_grad():
            d0, d1, scores = model(*pair)
            matches, mscores = lg.filter_matches(scores, 0.1)
            matches_all, mscores_all = lg.filter_matches(scores, 0.0)   # every mutual nearest neighbour
        out = {"desc0": d0.numpy(), "desc1": d1.numpy(), "scores": scores.numpy(),
               "matches": matches.numpy().astype(np.int64), "mscores": mscores.numpy(),
               "matches_all": matches_all.numpy().astype(np.int64), "mscores_all": mscores_all.numpy()}
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **out)
        index[name] = {"seed": seed, "n_layers": layers, "m": m, "n": n, "inputs_sha256": digest(sd, pair),
                       "n_matches": int(matches.shape[0])}
        print(name, {k: v.shape for k, v in out.items()}, "matches", int(matches.shape[0]))
    _merge_index(os.path.join(HERE, "matcher_index.json"), index)
    sweep = {}
    for name, (seed, layers, m, n, overlap, stride) in SWEEP_CASES.items():
        if not pick(name):
            continue
        model = lg.LightGlue(features=None, n_layers=layers).eval()
        sd = matcher.seeded_state_dict(seed, layers)
        model.load_state_dict(sd, strict=True)
        pair = matcher.synthetic_pair(seed, m, n, overlap=overlap)
        with torch.no_grad():
            d0, d1, scores = model(*pair)
            matches, mscores = lg.filter_matches(scores, 0.1)
            matches_all, mscores_all = lg.filter_matches(scores, 0.0)
        sc = scores[0].numpy()
        rows = np.arange(0, m, stride)
        out = {"rows": rows, "scores_rows": sc[rows], "scores_col0": sc[:, 0],
               "scores_row_sums": sc.astype(np.float64).sum(1), "scores_col_sums": sc.astype(np.float64).sum(0),
               "desc0_rows": d0[0].numpy()[rows], "desc1_rows": d1[0].numpy()[rows],
               "matches": matches.numpy().astype(np.int64), "mscores": mscores.numpy(),
               "matches_all": matches_all.numpy().astype(np.int64), "mscores_all": mscores_all.numpy()}
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
        sweep[name] = {"seed": seed, "n_layers": layers, "m": m, "n": n, "overlap": overlap,
                       "inputs_sha256": digest(sd, pair), "n_matches": int(matches.shape[0]),
                       "n_matches_all": int(matches_all.shape[0])}
        print(name, "matches", int(matches.shape[0]), "mutual", int(matches_all.shape[0]))
    _merge_index(os.path.join(HERE, "matcher_sweep_index.json"), sweep)


if __name__ == "__main__":
    main()

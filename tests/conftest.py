"""Test configuration: marker registration and import paths.

`-m "not gpu"` runs here (no GPU): oracle vs golden fixtures, the C-ABI library's
exports and the plugin's host-side contract. `-m gpu` runs on the MI355X box: parity
of the HIP kernels against the oracle and the reference's golden outputs.
"""
import glob
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")
for p in (REPO, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN_DIR = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def golden_cases():
    return sorted(os.path.basename(p)[5:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "attn_*.npz")))


def load_golden(name):
    """Load a fixture and regenerate its inputs (checked against the stored sha256)."""
    from lightglue_amd import synth

    with np.load(os.path.join(GOLDEN_DIR, f"attn_{name}.npz"), allow_pickle=False) as z:
        g = {k: z[k] for k in z.files}
    seed, nq, nkv = int(g["seed"]), int(g["nq"]), int(g["nkv"])
    q, k, v = synth.qkv(seed, nq, nkv, float(g["q_std"]), float(g["kv_std"]))
    spk = g["spike"]
    if spk[0] >= 0:
        k = synth.spike(q, k, int(spk[0]), int(spk[1]), float(spk[2]))
    assert synth.digest(q, k, v) == str(g["input_sha256"]), f"input generator drifted for {name}"
    g["q"], g["k"], g["v"] = q, k, v
    return g


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle

    oracle.build()
    return oracle

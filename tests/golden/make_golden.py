"""Generate the golden fixtures for the MHAHeadDim64 path from the reference itself.

Run in the build container only (it reads /root/reference, which is absent on the GPU box):

    python tests/golden/make_golden.py [case ...]   # all cases, or only the named ones

It loads the reference's oracle module file directly
(/root/reference/lightglue_pytorch_no_plugin/lightglue.py; importing the package fails
on its cv2 import) and evaluates ``Attention()(q, k, v)``
(lightglue.py:75-85) in float32 on CPU. The cross-check ``MHAHeadDim64.apply`` of the
with-plugin module (lightglue_pytorch_with_plugin/lightglue.py:16-46, an SDPA in eager
mode) is evaluated too.

Inputs are NOT stored: they are regenerated bit-exactly from (seed, shape, std) by
lightglue_amd.synth; each fixture stores the sha256 of the regenerated inputs so a
drift in the generator is caught. Stored expected outputs (float32):
  o_ref16  reference output on fp16-rounded inputs (what the fp16 kernels compute on)
  o_ref32  reference output on the raw fp32 inputs (the Float-boundary contract)
Large cases store a subset of query rows (``rows``) plus whole-tensor checksums.
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd"))
from lightglue_amd import synth  # noqa: E402

REF = "/root/reference"

# name: (seed, nq, nkv, q_std, kv_std, spike(q_row, k_row, gain) or None, full tensor?)
CASES = {
    "t1x1": (11, 1, 1, 1.0, 1.0, None, True),
    "t64": (12, 64, 64, 1.0, 1.0, None, True),
    "t100": (13, 100, 100, 1.0, 1.0, None, True),
    "t256": (14, 256, 256, 1.0, 1.0, None, True),          # BASELINE configs[0] shape
    "cross1000x777": (15, 1000, 777, 1.0, 1.0, None, False),
    "q2048xk64": (16, 2048, 64, 1.0, 1.0, None, False),
    "q64xk2048": (17, 64, 2048, 1.0, 1.0, None, True),
    "peaky192x160": (18, 192, 160, 3.0, 1.0, None, True),  # logit std ~3
    "spike128x300": (19, 128, 300, 1.0, 1.0, (5, 250, 4.0), True),
    "t1024": (20, 1024, 1024, 1.0, 1.0, None, False),      # BASELINE configs[1] shape
    "t33x65": (21, 33, 65, 1.0, 1.0, None, True),
    "t2048": (22, 2048, 2048, 1.0, 1.0, None, False),      # plugin maximum: the two-pass kernel
    "cross1536x1300": (23, 1536, 1300, 1.0, 1.0, None, False),
}
ROW_STRIDE = 16  # rows kept for non-full cases: 0, 16, 32, ... and the last row


def load_module(path: str, name: str):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def make_inputs(seed, nq, nkv, q_std, kv_std, spk):
    q, k, v = synth.qkv(seed, nq, nkv, q_std, kv_std)
    if spk is not None:
        k = synth.spike(q, k, *spk)
    return q, k, v


def main() -> None:
    torch.set_num_threads(8)
    ref_np = load_module(os.path.join(REF, "lightglue_pytorch_no_plugin", "lightglue.py"), "ref_lg_no_plugin")
    ref_wp = load_module(os.path.join(REF, "lightglue_pytorch_with_plugin", "lightglue.py"), "ref_lg_with_plugin")
    attn = ref_np.Attention()
    only = set(sys.argv[1:])
    index = {}
    index_path = os.path.join(HERE, "index.json")
    if only and os.path.exists(index_path):
        with open(index_path) as f:
            index = json.load(f)["cases"]
    for name, (seed, nq, nkv, q_std, kv_std, spk, full) in CASES.items():
        if only and name not in only:
            continue
        q, k, v = make_inputs(seed, nq, nkv, q_std, kv_std, spk)
        q16, k16, v16 = synth.round_f16(q), synth.round_f16(k), synth.round_f16(v)
        with torch.no_grad():
            o32 = attn(torch.from_numpy(q), torch.from_numpy(k), torch.from_numpy(v)).numpy()
            o16 = attn(torch.from_numpy(q16), torch.from_numpy(k16), torch.from_numpy(v16)).numpy()
            o_wp = ref_wp.MHAHeadDim64.apply(torch.from_numpy(q16), torch.from_numpy(k16),
                                             torch.from_numpy(v16)).numpy()
        sdpa_dev = float(np.abs(o_wp - o16).max())
        assert sdpa_dev < 1e-5, (name, sdpa_dev)
        rows = np.arange(nq) if full else np.unique(np.r_[np.arange(0, nq, ROW_STRIDE), nq - 1])
        rec = dict(
            name=np.array(name), seed=np.int64(seed), nq=np.int64(nq), nkv=np.int64(nkv),
            q_std=np.float64(q_std), kv_std=np.float64(kv_std),
            spike=np.array(spk if spk is not None else (-1, -1, 0.0), dtype=np.float64),
            input_sha256=np.array(synth.digest(q, k, v)),
            rows=rows.astype(np.int64),
            o_ref16=o16[:, :, rows, :].astype(np.float32),
            o_ref32=o32[:, :, rows, :].astype(np.float32),
            sum16=np.float64(o16.astype(np.float64).sum()),
            abssum16=np.float64(np.abs(o16.astype(np.float64)).sum()),
            sum32=np.float64(o32.astype(np.float64).sum()),
            sdpa_maxdev=np.float64(sdpa_dev),
        )
        path = os.path.join(HERE, f"attn_{name}.npz")
        np.savez_compressed(path, **rec)
        index[name] = dict(seed=seed, nq=nq, nkv=nkv, q_std=q_std, kv_std=kv_std, spike=spk,
                           rows=int(rows.size), sdpa_maxdev=sdpa_dev, bytes=os.path.getsize(path))
        print(f"{name:16s} nq={nq:5d} nkv={nkv:5d} rows={rows.size:5d} sdpa_dev={sdpa_dev:.2e} "
              f"{os.path.getsize(path)/1024:.0f} KiB")
    with open(index_path, "w") as f:
        json.dump(dict(generator="tests/golden/make_golden.py",
                       reference="lightglue_pytorch_no_plugin/lightglue.py:75-85 (Attention.forward)",
                       cross_check="lightglue_pytorch_with_plugin/lightglue.py:16-46 (MHAHeadDim64.apply, SDPA)",
                       torch=torch.__version__, cases=index), f, indent=1)


if __name__ == "__main__":
    main()

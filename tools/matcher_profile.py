"""Diagnostic driver for rocprofv3: eager fp16 LightGlue matcher forwards at N keypoints."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

from lightglue_amd import matcher  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
dev = torch.device("cuda:0")
model = matcher.LightGlueMatcher(n_layers=9).eval()
model.load_state_dict(matcher.seeded_state_dict(7, 9), strict=True)
model = model.to(dev, torch.float16)
k0, k1, d0, d1 = (t.to(dev, torch.float16) for t in matcher.synthetic_pair(40, n, n))
with torch.no_grad():
    for _ in range(12):
        model(k0, k1, d0, d1)
torch.cuda.synchronize()

"""Profiling driver: launch one forced plan of a 1x4xNqxNkv fp16 call --steps times (eager), for
rocprofv3 --pmc passes (plan codes as mha_hd64_launch_forced: 22 = 16-row single pass, 21 = 32-row,
23 = persistent streaming kernel, 0 = the planner's choice); batch calls stacked per launch.
    python tools/pmc_driver.py <plan> [nq] [nkv] [steps] [batch]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd")]
import torch  # noqa: E402

from lightglue_amd import _lib, synth  # noqa: E402

plan = int(sys.argv[1])
nq = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
nkv = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 50
batch = int(sys.argv[5]) if len(sys.argv) > 5 else 1
lib = _lib.load()
dev = torch.device("cuda:0")
q, k, v = (torch.from_numpy(x).to(dev).half().repeat(batch, 1, 1, 1).contiguous() for x in synth.qkv(11, nq, nkv))
o = torch.empty_like(q)
ws = torch.empty(5242880, dtype=torch.uint8, device=dev)
for _ in range(steps):
    assert lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), batch, 4, nq, nkv, 0, 0,
                                      plan, 0, 0, ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream, 3) == 0
torch.cuda.synchronize()

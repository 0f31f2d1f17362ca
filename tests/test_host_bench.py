"""The C++ host over the C ABI only (csrc/mha_hd64_host_bench.cpp): plugin lifecycle, one eager
enqueue checked against a double-precision CPU attention on sampled rows (<= 1e-2, in the
binary), then a captured graph of enqueues timed. Runs as a child process on the GPU box."""
import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "lightglue-with-flashattentionv2-tensorrt_amd", "lib", "mha_hd64_host_bench")


def test_host_bench_is_built():
    assert os.path.exists(BIN), "make -C lightglue-with-flashattentionv2-tensorrt_amd builds the C++ host"


@pytest.mark.gpu
@pytest.mark.parametrize("args", [["--nq", "1024", "--nkv", "1024"], ["--nq", "1000", "--nkv", "777"],
                                  ["--nq", "300", "--nkv", "2048", "--float"]])
def test_host_bench_parity_and_graph(args):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r = subprocess.run([BIN, "--steps", "200"] + args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["max_abs_err_sampled_rows"] <= 1e-2
    assert line["us_per_call"] > 0

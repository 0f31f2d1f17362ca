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


def _run(args, env=None, timeout=180):
    r = subprocess.run([BIN] + args, capture_output=True, text=True, timeout=timeout,
                       env=None if env is None else dict(os.environ, **env))
    assert r.returncode == 0, r.stderr + r.stdout
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{}, {"MHA_HD64_DIRECT": "0"}], ids=["default-plan", "ring-split-plan"])
def test_host_threads_share_one_device(env):
    """Two host threads on one GPU, each with its own plugin, stream and workspace, capturing and
    replaying graphs at the same time: per-(device, stream) tickets and the per-device capture arena
    are shared library state (ring-split-plan forces the split plans that use them)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    line = _run(["--steps", "200", "--streams", "2"], env)
    assert line["outputs_bitwise_identical"] is True and len(line["workers"]) == 2
    assert line["max_abs_err_sampled_rows"] <= 1e-2


@pytest.mark.gpu
def test_host_thread_per_device():
    """SURVEY.md §8e's host: one thread per GPU (hipSetDevice, one stream, one workspace each); the
    same pair gives bit-identical outputs on every device."""
    import torch

    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("needs >= 2 GPUs")
    line = _run(["--steps", "200", "--devices", str(n)])
    assert line["outputs_bitwise_identical"] is True
    assert sorted({w["device"] for w in line["workers"]}) == list(range(n))


def test_host_bench_refuses_missing_devices():
    """More devices than visible is an error, not a silent smaller run (no GPU here: 0 visible)."""
    import torch

    if torch.cuda.device_count() >= 64:
        pytest.skip("unexpected host")
    r = subprocess.run([BIN, "--devices", "64"], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0

"""Seeded random-shape parity sweep through the public operator surfaces (plugin enqueue, the L0
batched launcher, the grouped launcher), beyond the fixed fixture shapes: ragged query/key lengths
in [1, 2048], batches up to 24 (past one round of 128-row blocks, so the planner's streaming
kernel runs as well as the single-pass and split-KV forms), fp16 and fp32 inputs and outputs,
and logit scales from 0.25 to 3.

Reference: softmax(Q·Kᵀ/8)·V in float64 on the device, on the same (fp16-rounded) inputs
(lightglue_pytorch_no_plugin/lightglue.py:75-85). Bound: the north_star max-abs 1e-2, plus the
fp16-output regression guard of test_gpu_parity (1.5e-3 x logit scale + 2^-11 |ref|) and the
fp32-output guard 1.5e-3 x scale. Each case is printed with its seed so a failure reproduces alone.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL = 1e-2
REG_ABS = 1.5e-3
# cases per launcher (LG_FUZZ_CASES=n widens the sweep for a one-off run; the suite runs 64 / 64 / 48)
N_CASES = int(os.environ.get("LG_FUZZ_CASES", "64"))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from lightglue_amd import _lib

    _lib.load()
    return torch.device("cuda:0")


def _len(rng):
    """Mostly ragged lengths, with the edges (1, tile boundaries, the 2048 maximum) over-sampled."""
    r = rng.random()
    if r < 0.15:
        return int(rng.choice([1, 2, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129]))
    if r < 0.25:
        return int(rng.choice([255, 256, 257, 511, 512, 513, 1023, 1024, 1025, 2047, 2048]))
    return int(rng.integers(1, 2049))


def _inputs(seed, b, nq, nkv, dev, in_dt):
    g = torch.Generator(device="cpu").manual_seed(seed)
    scale = float(np.random.default_rng(seed).choice([0.25, 0.5, 1.0, 1.0, 2.0, 3.0]))
    q = torch.randn(b, 4, nq, 64, generator=g) * scale
    k = torch.randn(b, 4, nkv, 64, generator=g)
    v = torch.randn(b, 4, nkv, 64, generator=g)
    return [x.to(dev).to(in_dt).contiguous() for x in (q, k, v)], scale


def _ref(q, k, v):
    q, k, v = (x.double() for x in (q, k, v))
    return torch.softmax(q @ k.transpose(-1, -2) / 8.0, dim=-1) @ v


def _check(got, ref, scale, tag, v):
    got64 = got.double()
    assert torch.isfinite(got64).all(), tag
    d = (got64 - ref).abs()
    assert float(d.max()) <= TOL, (tag, float(d.max()))
    if got.dtype == torch.float16:
        bound = REG_ABS * scale + ref.abs() * 2.0 ** -11
    else:
        bound = torch.full_like(ref, REG_ABS * scale)
    # fewer than one 64-key tile, or peaked rows (logit scale >= 2: a row's mass on a few keys): the fp16
    # rounding of each P (2^-11 relative) no longer averages out over many keys, so a row's error
    # reaches 2^-11 max|v - o| (observed 1.6e-3 at nkv = 2; 5.1e-3 on the streaming kernel at scale 3,
    # 24 x 513 x 70 — seed 484 of the 600-case sweep, round 6 — within the 1e-2 contract)
    if v.shape[2] < 64 or scale >= 2.0:
        bound = bound + 2.0 ** -10 * float(v.double().abs().max())
    excess = float((d - bound).max())
    assert excess <= 0, (tag, f"regression excess {excess:.3e}, max-abs {float(d.max()):.3e}")


@pytest.mark.parametrize("seed", range(N_CASES))
def test_fuzz_plugin_enqueue(seed, dev):
    """The TensorRT-surface call ([1, 4, N, 64], all fp16 or all fp32), random ragged lengths."""
    from lightglue_amd import mha_hd64

    rng = np.random.default_rng(1000 + seed)
    nq, nkv = _len(rng), _len(rng)
    dt = torch.float16 if seed % 3 else torch.float32
    (q, k, v), scale = _inputs(1000 + seed, 1, nq, nkv, dev, dt)
    o = mha_hd64(q, k, v)
    torch.cuda.synchronize()
    assert o.dtype == dt and o.shape == q.shape
    _check(o, _ref(q.half(), k.half(), v.half()), scale, ("plugin", seed, nq, nkv, dt), v)


@pytest.mark.parametrize("seed", range(N_CASES))
def test_fuzz_batched_launcher(seed, dev):
    """L0 batched launcher: random batch 1-24 (the larger ones take the streaming kernel), random
    ragged lengths, fp16 or fp32 output from fp16 inputs, or fp32 inputs."""
    from lightglue_amd import mha_hd64_batched

    rng = np.random.default_rng(2000 + seed)
    b = int(rng.choice([1, 2, 3, 5, 8, 12, 16, 24]))
    nq, nkv = _len(rng), _len(rng)
    if b * nq * nkv > 16 * 1024 * 1024:  # keep the float64 reference small
        nkv = max(1, 16 * 1024 * 1024 // (b * nq))
    in_dt, out_dt = [(torch.float16, torch.float16), (torch.float16, torch.float32),
                     (torch.float32, torch.float32)][seed % 3]
    (q, k, v), scale = _inputs(2000 + seed, b, nq, nkv, dev, in_dt)
    o = mha_hd64_batched(q, k, v, out_dtype=out_dt)
    torch.cuda.synchronize()
    assert o.dtype == out_dt and o.shape == q.shape
    _check(o, _ref(q.half(), k.half(), v.half()), scale, ("batched", seed, b, nq, nkv, in_dt, out_dt), v)


@pytest.mark.parametrize("seed", range(N_CASES * 3 // 4))
def test_fuzz_grouped_launcher(seed, dev):
    """Grouped launcher: 1-7 independent calls of unrelated shapes and batches in one call
    (chunked by 4), each output against its own reference."""
    from lightglue_amd import mha_hd64_grouped

    rng = np.random.default_rng(3000 + seed)
    ncall = int(rng.integers(1, 8))
    in_dt, out_dt = [(torch.float16, torch.float16), (torch.float16, torch.float32),
                     (torch.float32, torch.float32)][seed % 3]
    calls, scales = [], []
    for i in range(ncall):
        b = int(rng.choice([1, 1, 2, 3]))
        nq, nkv = _len(rng), _len(rng)
        qkv, scale = _inputs(3000 + 37 * seed + i, b, nq, nkv, dev, in_dt)
        calls.append(tuple(qkv))
        scales.append(scale)
    outs = mha_hd64_grouped(calls, out_dtype=out_dt)
    torch.cuda.synchronize()
    assert len(outs) == ncall
    for i, ((q, k, v), o, s) in enumerate(zip(calls, outs, scales)):
        assert o.dtype == out_dt and o.shape == q.shape, (seed, i)
        _check(o, _ref(q.half(), k.half(), v.half()), s, ("grouped", seed, i, tuple(q.shape), tuple(k.shape)), v)

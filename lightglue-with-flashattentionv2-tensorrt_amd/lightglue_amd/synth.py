"""Deterministic synthetic Q/K/V for the MHAHeadDim64 path.

The reference ships no fixtures, so inputs are regenerated from a
portable recipe instead of being stored: splitmix64 counters -> 24-bit uniforms ->
Irwin-Hall(4) approximately-normal values. Every step is exact or a single
correctly-rounded IEEE operation, so the same (seed, shape, std) gives bit-identical
float32 tensors on any host (this container, the GPU box), which lets the golden
fixtures under tests/golden store only expected outputs.

Shapes follow the plugin contract: [batch=1, heads=4, N, 64], contiguous
(lightglue_attention_plugin/lightglue_attention_plugin.h:19-22).
"""
from __future__ import annotations

import hashlib

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_C1 = np.uint64(0xBF58476D1CE4E5B9)
_C2 = np.uint64(0x94D049BB133111EB)
_SQRT3 = float(np.sqrt(np.float64(3.0)))

HEADS = 4
HEAD_DIM = 64


def _splitmix64(counter: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = counter * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _C1
        z = (z ^ (z >> np.uint64(27))) * _C2
        return z ^ (z >> np.uint64(31))


def uniform24(seed: int, n: int) -> np.ndarray:
    """n exact multiples of 2**-24 in [0, 1) (float64)."""
    base = np.uint64((seed * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        ctr = base + np.arange(1, n + 1, dtype=np.uint64)
    bits = _splitmix64(ctr) >> np.uint64(40)
    return bits.astype(np.float64) * (1.0 / (1 << 24))


def normal(seed: int, shape, std: float = 1.0) -> np.ndarray:
    """Approximately N(0, std^2) float32 values, bit-reproducible across hosts."""
    n = int(np.prod(shape))
    u = uniform24(seed, 4 * n).reshape(4, n)
    x = (u[0] + u[1] + u[2] + u[3] - 2.0) * _SQRT3  # exact sum, one rounding
    if std != 1.0:
        x = x * float(std)
    return x.astype(np.float32).reshape(shape)


def qkv(seed: int, nq: int, nkv: int, q_std: float = 1.0, kv_std: float = 1.0, batch: int = 1,
        heads: int = HEADS):
    """Q [b,h,nq,64], K/V [b,h,nkv,64] float32."""
    q = normal(seed * 3 + 0, (batch, heads, nq, HEAD_DIM), q_std)
    k = normal(seed * 3 + 1, (batch, heads, nkv, HEAD_DIM), kv_std)
    v = normal(seed * 3 + 2, (batch, heads, nkv, HEAD_DIM), kv_std)
    return q, k, v


def spike(q: np.ndarray, k: np.ndarray, q_row: int, k_row: int, gain: float) -> np.ndarray:
    """Return K with row k_row of every head replaced by gain * Q[q_row].

    Forces the online-softmax running max of query q_row to jump at the KV tile
    holding k_row (cdna_hip_programming.md §5.4 rule 26)."""
    k = k.copy()
    k[:, :, k_row, :] = (q[:, :, q_row, :].astype(np.float64) * gain).astype(np.float32)
    return k


def round_f16(x: np.ndarray) -> np.ndarray:
    """fp32 -> fp16 (round-to-nearest-even) -> fp32, what the fp16 path computes on."""
    return x.astype(np.float16).astype(np.float32)


def digest(*arrays: np.ndarray) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()

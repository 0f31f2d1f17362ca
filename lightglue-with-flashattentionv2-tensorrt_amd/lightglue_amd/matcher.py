"""LightGlue matcher built around the MI355X attention op.

A restatement of the reference model (lightglue_pytorch_no_plugin/lightglue.py): input
projection, Fourier positional encoding applied as a rotary embedding (:32-52, :124-134),
``n_layers`` x (SelfBlock on each image with shared weights, CrossBlock in both directions)
(:88-194), MatchAssignment with the dual log-softmax (:197-233) and ``filter_matches``
(:236-262). Parameter names equal the reference's state-dict keys, so a reference checkpoint
(or ``seeded_state_dict``) loads unchanged.

What is different, and why:
* attention runs on the gfx950 kernel through the grouped launcher: per layer ONE launch for the
  two self-attention calls and ONE for the two cross directions (the reference makes four plugin
  enqueues per layer, TransformerLayer :186-194);
* the projections and FFNs whose weights both images share run once on the two images'
  rows concatenated (half the launches, twice the GEMM height); q/k/v are produced head-major
  in one copy (the reference splits an interleaved [N, H, 64, 3] projection and transposes);
* the column log-softmax of the assignment runs on a contiguous transpose (the reference's
  strided ``log_softmax(sim, 1)``);
* ``attention=`` lets tests substitute the oracle for the kernel on CPU; the default path
  requires GPU tensors and fails loudly otherwise (no CPU fallback).
"""
from __future__ import annotations

import zlib
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from . import synth
from .plugin import PluginError, mha_hd64_grouped

AttnFn = Callable[[Sequence[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]], List[torch.Tensor]]


def _kernel_attention(calls):
    for q, _, _ in calls:
        if not q.is_cuda:
            raise PluginError("LightGlueMatcher: the attention op runs on the GPU only (no CPU fallback)")
    return mha_hd64_grouped(calls)


class FourierPositionalEncoding(nn.Module):
    """lightglue.py:32-52: cos/sin of a learned projection of the keypoints, each repeated
    for the two members of a rotary pair. Returns (cos, sin), each [1, 1, N, head_dim]."""

    def __init__(self, m: int = 2, head_dim: int = 64) -> None:
        super().__init__()
        self.Wr = nn.Linear(m, head_dim // 2, bias=False)

    def forward(self, kpts: torch.Tensor):
        proj = self.Wr(kpts)                                   # [1, N, head_dim/2]
        cos = torch.cos(proj).repeat_interleave(2, dim=-1)     # (c0, c0, c1, c1, ...)
        sin = torch.sin(proj).repeat_interleave(2, dim=-1)
        return cos.unsqueeze(1), sin.unsqueeze(1)


def _rotary(t: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """t * cos + swap(t) * sin with swap((x0, x1)) = (-x1, x0) on consecutive pairs
    (lightglue.py:124-134)."""
    pairs = t.unflatten(-1, (-1, 2))
    swapped = torch.stack((-pairs[..., 1], pairs[..., 0]), dim=-1).flatten(-2)
    return t * cos + swapped * sin


def _ffn(d: int) -> nn.Sequential:
    return nn.Sequential(nn.Linear(2 * d, 2 * d), nn.LayerNorm(2 * d, elementwise_affine=True), nn.GELU(),
                         nn.Linear(2 * d, d))


class SelfBlock(nn.Module):
    """lightglue.py:88-134 (weights shared by both images of a pair)."""

    def __init__(self, d: int, heads: int) -> None:
        super().__init__()
        self.heads, self.head_dim = heads, d // heads
        self.Wqkv = nn.Linear(d, 3 * d)
        self.out_proj = nn.Linear(d, d)
        self.ffn = _ffn(d)

    def qkv(self, x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, splits: Sequence[int]):
        """x [1, N0+N1, d] (both images' rows) -> per image (q, k, v), each [1, H, Ni, 64]."""
        n = x.shape[1]
        # Wqkv output channel (h*64 + d)*3 + j  ->  [3, H, N, 64] head-major
        t = self.Wqkv(x).view(n, self.heads, self.head_dim, 3).permute(3, 1, 0, 2)
        q = _rotary(t[0], cos, sin)
        k = _rotary(t[1], cos, sin)
        out, a = [], 0
        for ni in splits:
            out.append(tuple(u[:, a:a + ni].unsqueeze(0).contiguous() for u in (q, k, t[2])))
            a += ni
        return out

    def finish(self, x: torch.Tensor, contexts: Sequence[torch.Tensor]) -> torch.Tensor:
        msg = self.out_proj(torch.cat([c[0].transpose(0, 1).reshape(c.shape[2], -1) for c in contexts], 0)[None])
        return x + self.ffn(torch.cat((x, msg), -1))


class CrossBlock(nn.Module):
    """lightglue.py:137-183: shared q/k projection, both directions."""

    def __init__(self, d: int, heads: int) -> None:
        super().__init__()
        self.heads, self.head_dim = heads, d // heads
        self.to_qk = nn.Linear(d, d)
        self.to_v = nn.Linear(d, d)
        self.to_out = nn.Linear(d, d)
        self.ffn = _ffn(d)

    def heads_of(self, t: torch.Tensor, splits: Sequence[int]) -> List[torch.Tensor]:
        """[1, N0+N1, d] -> per image [1, H, Ni, 64]."""
        h = t[0].view(t.shape[1], self.heads, self.head_dim).transpose(0, 1)
        out, a = [], 0
        for ni in splits:
            out.append(h[:, a:a + ni].unsqueeze(0).contiguous())
            a += ni
        return out

    def finish(self, x: torch.Tensor, ms: Sequence[torch.Tensor]) -> torch.Tensor:
        msg = self.to_out(torch.cat([m[0].transpose(0, 1).reshape(m.shape[2], -1) for m in ms], 0)[None])
        return x + self.ffn(torch.cat((x, msg), -1))


class TransformerLayer(nn.Module):
    def __init__(self, d: int, heads: int) -> None:
        super().__init__()
        self.self_attn = SelfBlock(d, heads)
        self.cross_attn = CrossBlock(d, heads)

    def forward(self, x, cos, sin, splits, attention: AttnFn):
        """x: both images' descriptors [1, N0+N1, d] (image 0 rows first)."""
        sa, ca = self.self_attn, self.cross_attn
        x = sa.finish(x, attention(sa.qkv(x, cos, sin, splits)))       # one grouped launch (self0, self1)
        qk0, qk1 = ca.heads_of(ca.to_qk(x), splits)
        v0, v1 = ca.heads_of(ca.to_v(x), splits)
        return ca.finish(x, attention([(qk0, qk1, v1), (qk1, qk0, v0)]))  # one grouped launch (cross)


def log_double_softmax(sim: torch.Tensor, z0: torch.Tensor, z1: torch.Tensor) -> torch.Tensor:
    """lightglue.py:197-205: log_softmax over both axes plus the matchability log-sigmoids
    (the column pass on a contiguous transpose)."""
    col = F.log_softmax(sim.transpose(1, 2).contiguous(), 2).transpose(1, 2)
    return F.log_softmax(sim, 2) + col + F.logsigmoid(z0) + F.logsigmoid(z1).transpose(1, 2)


class MatchAssignment(nn.Module):
    """lightglue.py:208-233."""

    def __init__(self, d: int) -> None:
        super().__init__()
        self.scale = d ** 0.25
        self.final_proj = nn.Linear(d, d)
        self.matchability = nn.Linear(d, 1)

    def forward(self, d0: torch.Tensor, d1: torch.Tensor) -> torch.Tensor:
        m0 = self.final_proj(d0) / self.scale
        m1 = self.final_proj(d1) / self.scale
        sim = m0 @ m1.transpose(1, 2)
        return log_double_softmax(sim.float(), self.matchability(d0).float(), self.matchability(d1).float())


def filter_matches(scores: torch.Tensor, th: float):
    """lightglue.py:236-262: mutual nearest neighbours of the log assignment above `th`.
    Returns (matches [K, 2] int64, scores [K])."""
    v0, m0 = scores.max(2)          # best column per row
    _, m1 = scores.max(1)           # best row per column
    rows = torch.arange(m0.shape[1], device=scores.device)
    mutual = m1[0].gather(0, m0[0]) == rows
    ms = torch.where(mutual, v0[0].exp(), torch.zeros((), device=scores.device, dtype=v0.dtype))
    keep = ms > th
    idx0 = rows[keep]
    return torch.stack([idx0, m0[0][idx0]], -1), ms[idx0]


class LightGlueMatcher(nn.Module):
    """LightGlue(features=None) of the reference with the MI355X attention (lightglue.py:265-353).

    forward(kpts0 [1,M,2], kpts1 [1,N,2], desc0 [1,M,in], desc1 [1,N,in])
        -> (desc0 [1,M,d], desc1 [1,N,d], log-assignment scores [1,M,N] fp32)"""

    def __init__(self, n_layers: int = 9, descriptor_dim: int = 256, input_dim: int = 256, num_heads: int = 4,
                 filter_threshold: float = 0.1, attention: Optional[AttnFn] = None) -> None:
        super().__init__()
        d = descriptor_dim
        self.n_layers, self.filter_threshold = n_layers, filter_threshold
        self.input_proj = nn.Linear(input_dim, d) if input_dim != d else nn.Identity()
        self.posenc = FourierPositionalEncoding(2, d // num_heads)
        self.transformers = nn.ModuleList([TransformerLayer(d, num_heads) for _ in range(n_layers)])
        self.log_assignment = nn.ModuleList([MatchAssignment(d) for _ in range(n_layers)])
        self.attention = attention or _kernel_attention

    def forward(self, kpts0, kpts1, desc0, desc1):
        splits = (desc0.shape[1], desc1.shape[1])
        x = self.input_proj(torch.cat((desc0, desc1), 1))
        cos, sin = self.posenc(torch.cat((kpts0, kpts1), 1).to(x.dtype))
        cos, sin = cos[0], sin[0]                                  # [1, N0+N1, 64], broadcast over heads
        for layer in self.transformers:
            x = layer(x, cos, sin, splits, self.attention)
        d0, d1 = x[:, :splits[0]], x[:, splits[0]:]
        return d0, d1, self.log_assignment[self.n_layers - 1](d0, d1)

    def match(self, kpts0, kpts1, desc0, desc1):
        """forward + filter_matches (the demo's post-processing)."""
        _, _, scores = self.forward(kpts0, kpts1, desc0, desc1)
        return filter_matches(scores, self.filter_threshold)


# --------------------------------------------------------------------------------------------
# Deterministic synthetic weights and inputs (no checkpoints offline): every parameter is drawn
# from lightglue_amd.synth (bit-reproducible on any host) with a seed derived from its name.
# --------------------------------------------------------------------------------------------
def seeded_state_dict(seed: int, n_layers: int = 9, descriptor_dim: int = 256, input_dim: int = 256,
                      num_heads: int = 4) -> dict:
    ref = LightGlueMatcher(n_layers, descriptor_dim, input_dim, num_heads)
    out = {}
    for name, p in ref.state_dict().items():
        s = (seed * 1_000_003 + zlib.crc32(name.encode())) & 0x7FFFFFFF
        shape = tuple(p.shape)
        if name.endswith("posenc.Wr.weight"):
            arr = synth.normal(s, shape, 1.0)                     # reference init: std gamma^-2 = 1
        elif ".ffn.1." in name:                                   # LayerNorm affine
            arr = (1.0 if name.endswith("weight") else 0.0) + synth.normal(s, shape, 0.1)
        elif name.endswith("weight"):
            arr = synth.normal(s, shape, 1.0 / np.sqrt(shape[-1]))
        else:
            arr = synth.normal(s, shape, 0.02)
        out[name] = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float32))
    return out


def synthetic_pair(seed: int, m: int, n: int, input_dim: int = 256):
    """Keypoints in the normalised [-1, 1] frame and unit-norm descriptors, fp32, batch 1."""
    k0 = synth.uniform24(seed * 4 + 0, m * 2).reshape(1, m, 2) * 2.0 - 1.0
    k1 = synth.uniform24(seed * 4 + 1, n * 2).reshape(1, n, 2) * 2.0 - 1.0
    d0 = synth.normal(seed * 4 + 2, (1, m, input_dim))
    d1 = synth.normal(seed * 4 + 3, (1, n, input_dim))
    d0 = d0 / np.linalg.norm(d0, axis=-1, keepdims=True)
    d1 = d1 / np.linalg.norm(d1, axis=-1, keepdims=True)
    return tuple(torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)) for x in (k0, k1, d0, d1))

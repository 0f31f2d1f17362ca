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
* ``glue="hip"`` (default) runs the layout/normalisation steps around the attention on gfx950
  kernels (include/lightglue_glue.h: q/k/v split + rotary + per-image head-major layout in one
  pass, head split/merge, LayerNorm+GELU, the dual log-softmax); ``glue="torch"`` is the same
  math in framework ops (the restatement the CPU tests pin to the reference);
* ``attention=`` lets tests substitute the oracle for the kernel on CPU; the default path
  requires GPU tensors and fails loudly otherwise (no CPU fallback).
"""
from __future__ import annotations

import ctypes
import os
import zlib
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from . import _lib, synth
from .plugin import PluginError, _check, _workspace

AttnFn = Callable[[Sequence[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]], List[torch.Tensor]]


_DT = {torch.float16: _lib.DT_HALF, torch.float32: _lib.DT_FLOAT}


def _sp(splits):
    """(n0, n1[, pairs]) -> (n0, n1, pairs): rows are `pairs` image pairs stacked pair-major."""
    return (splits[0], splits[1], splits[2] if len(splits) > 2 else 1)


class _Hip:
    """Thin wrappers of the gfx950 glue kernels (current stream, fail loudly on error). Row-major
    tensors hold P image pairs stacked pair-major ([1, P*(n0+n1), C]); per-image head-major
    tensors are [P, heads, ni, 64] (include/lightglue_glue.h)."""

    @staticmethod
    def _stream(t):
        return torch.cuda.current_stream(t.device).cuda_stream

    @staticmethod
    def qkv_rotary_split(qkv, cos, sin, heads, splits):
        n0, n1, pr = _sp(splits)
        mk = lambda n: torch.empty((pr, heads, n, 64), dtype=qkv.dtype, device=qkv.device)  # noqa: E731
        out = [tuple(mk(n) for _ in range(3)) for n in (n0, n1)]
        st = _lib.load().lg_qkv_rotary_split(_DT[qkv.dtype], qkv.data_ptr(), cos.data_ptr(), sin.data_ptr(), heads,
                                             n0, n1, pr, *(t.data_ptr() for t in out[0]),
                                             *(t.data_ptr() for t in out[1]), _Hip._stream(qkv))
        _check(st, "lg_qkv_rotary_split")
        return out

    @staticmethod
    def split_heads2(a, b, heads, splits):
        n0, n1, pr = _sp(splits)
        mk = lambda n: torch.empty((pr, heads, n, 64), dtype=a.dtype, device=a.device)  # noqa: E731
        a0, a1, b0, b1 = mk(n0), mk(n1), mk(n0), mk(n1)
        st = _lib.load().lg_split_heads2(_DT[a.dtype], a.data_ptr(), b.data_ptr(), heads, n0, n1, pr, a0.data_ptr(),
                                         a1.data_ptr(), b0.data_ptr(), b1.data_ptr(), _Hip._stream(a))
        _check(st, "lg_split_heads2")
        return (a0, a1), (b0, b1)

    @staticmethod
    def split_heads2_ld(ab, heads, splits):
        """ab [1, P*(N0+N1), 2*heads*64] = [a | b] (one GEMM's output) -> per image (a_i, b_i) heads."""
        n0, n1, pr = _sp(splits)
        mk = lambda n: torch.empty((pr, heads, n, 64), dtype=ab.dtype, device=ab.device)  # noqa: E731
        a0, a1, b0, b1 = mk(n0), mk(n1), mk(n0), mk(n1)
        half = heads * 64
        st = _lib.load().lg_split_heads2_ld(_DT[ab.dtype], ab.data_ptr(), ab.data_ptr() + half * ab.element_size(),
                                            2 * half, heads, n0, n1, pr, a0.data_ptr(), a1.data_ptr(), b0.data_ptr(),
                                            b1.data_ptr(), _Hip._stream(ab))
        _check(st, "lg_split_heads2_ld")
        return (a0, a1), (b0, b1)

    @staticmethod
    def merge_heads_cat(x, x0, x1):
        """[x | merge_heads(x0, x1)] -> [1, P*(N0+N1), 2*heads*64] (the FFN input)."""
        pr, heads, n0, n1 = x0.shape[0], x0.shape[1], x0.shape[2], x1.shape[2]
        out = torch.empty((1, pr * (n0 + n1), 2 * heads * 64), dtype=x.dtype, device=x.device)
        st = _lib.load().lg_merge_heads_cat(_DT[x.dtype], x.data_ptr(), x0.data_ptr(), x1.data_ptr(), heads, n0, n1,
                                            pr, out.data_ptr(), _Hip._stream(x))
        _check(st, "lg_merge_heads_cat")
        return out

    # ---- projections with their neighbours fused (fp16; csrc/lightglue_linear.hip) ----
    @staticmethod
    def linear(a, w, b, res=None):
        """a [1, M, K] -> a·wᵀ + b (+ res) [1, M, N]."""
        m, k = a.shape[1], a.shape[2]
        out = torch.empty((1, m, w.shape[0]), dtype=a.dtype, device=a.device)
        st = _lib.load().lg_linear(a.data_ptr(), w.data_ptr(), b.data_ptr(), res.data_ptr() if res is not None else None,
                                   m, w.shape[0], k, out.data_ptr(), _Hip._stream(a))
        _check(st, "lg_linear")
        return out

    @staticmethod
    def linear_cat(x, c0, c1, w, b):
        """[x | merge_heads(c0, c1)]·wᵀ + b."""
        pr, heads, n0, n1 = c0.shape[0], c0.shape[1], c0.shape[2], c1.shape[2]
        out = torch.empty((1, pr * (n0 + n1), w.shape[0]), dtype=x.dtype, device=x.device)
        st = _lib.load().lg_linear_cat(x.data_ptr(), c0.data_ptr(), c1.data_ptr(), heads, n0, n1, pr, w.data_ptr(),
                                       b.data_ptr(), w.shape[0], out.data_ptr(), _Hip._stream(x))
        _check(st, "lg_linear_cat")
        return out

    @staticmethod
    def ffn(x, c0, c1, w, b, ln: nn.LayerNorm, w2, b2, packed=None):
        """x + ffn([x | merge_heads(c0, c1)]) (lightglue.py:101-106 with the block's residual):
        with `packed` (ffn_pack(w, w2)) one launch (ffn_rows_kernel), else linear_cat_ln_gelu into
        the scratch h, then linear(h, w2, b2, res=x) (include/lightglue_glue.h, lg_linear_set_ffn_fused)."""
        pr, heads, n0, n1 = c0.shape[0], c0.shape[1], c0.shape[2], c1.shape[2]
        m = pr * (n0 + n1)
        h = torch.empty((1, m, w.shape[0]), dtype=x.dtype, device=x.device)
        out = torch.empty((1, m, w2.shape[0]), dtype=x.dtype, device=x.device)
        st = _lib.load().lg_linear_cat_ffn(x.data_ptr(), c0.data_ptr(), c1.data_ptr(), heads, n0, n1, pr,
                                           w.data_ptr(), b.data_ptr(), ln.weight.data_ptr(), ln.bias.data_ptr(),
                                           float(ln.eps), w2.data_ptr(), b2.data_ptr(),
                                           packed.data_ptr() if packed is not None else None, h.data_ptr(),
                                           out.data_ptr(), _Hip._stream(x))
        _check(st, "lg_linear_cat_ffn")
        return out

    @staticmethod
    def ffn_proj(x, c0, c1, b, ln: nn.LayerNorm, b2, packed, kind, b3, splits, cos=None, sin=None, n_store=0):
        """lg_linear_cat_ffn_proj: (x' = x + ffn([x | merge_heads(c0, c1)]), the next projection of x')
        in one launch; kind 1 -> ((a0, a1), (b0, b1)) per-image heads (to_qk | to_v), kind 2 -> q/k/v
        per image with the rotary, kind 3 -> [1, M, n_store] rows."""
        n0, n1, pr = _sp(splits)
        heads = c0.shape[1]
        m = pr * (n0 + n1)
        out = torch.empty((1, m, 256), dtype=x.dtype, device=x.device)
        mk = lambda n: torch.empty((pr, heads, n, 64), dtype=x.dtype, device=x.device)  # noqa: E731
        if kind == 1:
            outs = [mk(n0), mk(n1), mk(n0), mk(n1)]
        elif kind == 2:
            outs = [mk(n0), mk(n0), mk(n0), mk(n1), mk(n1), mk(n1)]
        else:
            outs = [torch.empty((1, m, n_store), dtype=x.dtype, device=x.device)]
        ptrs = (ctypes.c_void_p * 6)(*([t.data_ptr() for t in outs] + [None] * (6 - len(outs))))
        st = _lib.load().lg_linear_cat_ffn_proj(x.data_ptr(), c0.data_ptr(), c1.data_ptr(), heads, n0, n1, pr, b.data_ptr(),
                                                ln.weight.data_ptr(), ln.bias.data_ptr(), float(ln.eps), b2.data_ptr(),
                                                packed.data_ptr(), kind, b3.data_ptr(),
                                                cos.data_ptr() if cos is not None else None,
                                                sin.data_ptr() if sin is not None else None, n_store, ptrs, out.data_ptr(),
                                                _Hip._stream(x))
        _check(st, "lg_linear_cat_ffn_proj")
        if kind == 1:
            return out, ((outs[0], outs[1]), (outs[2], outs[3]))
        if kind == 2:
            return out, [tuple(outs[:3]), tuple(outs[3:])]
        return out, outs[0]

    @staticmethod
    def linear_cat_ln_gelu(x, c0, c1, w, b, ln: nn.LayerNorm):
        """GELU(LayerNorm([x | merge_heads(c0, c1)]·wᵀ + b)) in one launch (P pairs of equal sizes)."""
        pr, heads, n0, n1 = c0.shape[0], c0.shape[1], c0.shape[2], c1.shape[2]
        out = torch.empty((1, pr * (n0 + n1), w.shape[0]), dtype=x.dtype, device=x.device)
        st = _lib.load().lg_linear_cat_ln_gelu(x.data_ptr(), c0.data_ptr(), c1.data_ptr(), heads, n0, n1, pr,
                                               w.data_ptr(), b.data_ptr(), ln.weight.data_ptr(), ln.bias.data_ptr(),
                                               float(ln.eps), out.data_ptr(), _Hip._stream(x))
        _check(st, "lg_linear_cat_ln_gelu")
        return out

    @staticmethod
    def linear_qkv_rotary(x, w_perm, b_perm, cos, sin, heads, splits):
        n0, n1, pr = _sp(splits)
        mk = lambda n: torch.empty((pr, heads, n, 64), dtype=x.dtype, device=x.device)  # noqa: E731
        out = [tuple(mk(n) for _ in range(3)) for n in (n0, n1)]
        st = _lib.load().lg_linear_qkv_rotary(x.data_ptr(), w_perm.data_ptr(), b_perm.data_ptr(), cos.data_ptr(),
                                              sin.data_ptr(), heads, n0, n1, pr, x.shape[2],
                                              *(t.data_ptr() for t in out[0]), *(t.data_ptr() for t in out[1]),
                                              _Hip._stream(x))
        _check(st, "lg_linear_qkv_rotary")
        return out

    @staticmethod
    def linear_split2(x, w, b, heads, splits):
        n0, n1, pr = _sp(splits)
        mk = lambda n: torch.empty((pr, heads, n, 64), dtype=x.dtype, device=x.device)  # noqa: E731
        a0, a1, b0, b1 = mk(n0), mk(n1), mk(n0), mk(n1)
        st = _lib.load().lg_linear_split2(x.data_ptr(), w.data_ptr(), b.data_ptr(), heads, n0, n1, pr, x.shape[2],
                                          a0.data_ptr(), a1.data_ptr(), b0.data_ptr(), b1.data_ptr(), _Hip._stream(x))
        _check(st, "lg_linear_split2")
        return (a0, a1), (b0, b1)

    @staticmethod
    def merge_heads(x0, x1):
        pr, heads, n0, n1 = x0.shape[0], x0.shape[1], x0.shape[2], x1.shape[2]
        out = torch.empty((1, pr * (n0 + n1), heads * 64), dtype=x0.dtype, device=x0.device)
        st = _lib.load().lg_merge_heads(_DT[x0.dtype], x0.data_ptr(), x1.data_ptr(), heads, n0, n1, pr, out.data_ptr(),
                                        _Hip._stream(x0))
        _check(st, "lg_merge_heads")
        return out

    @staticmethod
    def layernorm_gelu(x, ln: nn.LayerNorm):
        y = torch.empty_like(x)
        rows, dim = x.numel() // x.shape[-1], x.shape[-1]
        st = _lib.load().lg_layernorm_gelu(_DT[x.dtype], x.data_ptr(), ln.weight.data_ptr(), ln.bias.data_ptr(), rows,
                                           dim, float(ln.eps), y.data_ptr(), _Hip._stream(x))
        _check(st, "lg_layernorm_gelu")
        return y

    @staticmethod
    def log_double_softmax(sim, z0, z1):
        """sim [P, m, n], z0 [P, m, 1], z1 [P, n, 1] (P pairs, one launch)."""
        pr, m, n = sim.shape[0], sim.shape[1], sim.shape[2]
        lib = _lib.load()
        out = torch.empty_like(sim)
        stream = _Hip._stream(sim)
        ws = _workspace(sim.device, stream, lib.lg_log_double_softmax_workspace(m, n, pr))
        st = lib.lg_log_double_softmax(sim.data_ptr(), z0.data_ptr(), z1.data_ptr(), m, n, pr, out.data_ptr(),
                                       ws.data_ptr(), stream)
        _check(st, "lg_log_double_softmax")
        return out


    @staticmethod
    def log_double_softmax_f16(sim, v, m, zc):
        """sim [P, m, n] fp16 (contiguous); the matchability logits at channel zc of v [P, m + n, C]
        (the assignment projection's output): one fp32 scores tensor [P, m, n], two launches."""
        pr, n, ch = sim.shape[0], sim.shape[2], v.shape[2]
        lib = _lib.load()
        out = torch.empty(sim.shape, dtype=torch.float32, device=sim.device)
        stream = _Hip._stream(sim)
        ws = _workspace(sim.device, stream, lib.lg_log_double_softmax_f16_workspace(m, n, pr))
        base = v.data_ptr() + zc * v.element_size()
        st = lib.lg_log_double_softmax_f16(sim.data_ptr(), base, base + m * ch * v.element_size(), (m + n) * ch, ch,
                                           m, n, pr, out.data_ptr(), ws.data_ptr(), stream)
        _check(st, "lg_log_double_softmax_f16")
        return out

    _last_assign_ws = None  # (tests read the similarity copy the kernel leaves in its workspace)

    @staticmethod
    def assign_scores(v, m, zc):
        """v [P, m + n, C] fp16: the assignment projection of both images' rows (scaled descriptors at
        channels 0..255, the matchability logit at zc) -> fp32 scores [P, m, n] (lg_assign_scores: the
        similarity and the dual log-softmax in two launches)."""
        pr, n, ch = v.shape[0], v.shape[1] - m, v.shape[2]
        lib = _lib.load()
        out = torch.empty((pr, m, n), dtype=torch.float32, device=v.device)
        stream = _Hip._stream(v)
        ws = _workspace(v.device, stream, lib.lg_assign_scores_workspace(m, n, pr))
        _Hip._last_assign_ws = ws
        st = lib.lg_assign_scores(v.data_ptr(), (m + n) * ch, ch, zc, m, n, pr, out.data_ptr(), ws.data_ptr(), stream)
        _check(st, "lg_assign_scores")
        return out

    @staticmethod
    def pair_inputs(desc0, desc1, kpts0, kpts1, wr):
        """x [1, P*(m+n), 256] pair-major and the rotary tables cos, sin [1, P*(m+n), 64] in one launch."""
        pr, m, n, d = desc0.shape[0], desc0.shape[1], desc1.shape[1], desc0.shape[2]
        rows = pr * (m + n)
        x = torch.empty((1, rows, d), dtype=desc0.dtype, device=desc0.device)
        cos = torch.empty((1, rows, 64), dtype=desc0.dtype, device=desc0.device)
        sin = torch.empty_like(cos)
        t = [u.contiguous() for u in (desc0, desc1, kpts0, kpts1, wr)]
        st = _lib.load().lg_pair_inputs(*(u.data_ptr() for u in t), m, n, pr, d, x.data_ptr(), cos.data_ptr(),
                                        sin.data_ptr(), _Hip._stream(desc0))
        _check(st, "lg_pair_inputs")
        return x, cos, sin


def _cached(module: nn.Module, name: str, params: Sequence[torch.Tensor], dtype: torch.dtype, build):
    """Derived weights cached on `module`, rebuilt when any source parameter changes (in-place
    updates bump ``_version``; load_state_dict does) or the dtype/device differs."""
    key = (dtype, params[0].device, tuple(p._version for p in params), tuple(p.data_ptr() for p in params))
    hit = module.__dict__.get(name)
    if hit is not None and hit[0] == key:
        return hit[1]
    with torch.no_grad():
        val = tuple(t.to(dtype).contiguous() for t in build())
    module.__dict__[name] = (key, val)
    return val


def _ffn_in_fused(block: nn.Module, proj: nn.Linear, dtype: torch.dtype):
    """The block's message projection folded into the FFN's first layer (hip path):
    ffn0(cat(x, proj(m))) = cat(x, m) @ [W_x | W_m·W_p]ᵀ + (b + W_m·b_p), computed in fp32.
    (lightglue.py:104-106, 181-183: the projection feeds only the FFN.)"""
    lin = block.ffn[0]

    def build():
        d = proj.weight.shape[0]
        w = lin.weight.float()
        wx, wm = w[:, :d], w[:, d:]
        return (torch.cat((wx, wm @ proj.weight.float()), 1), lin.bias.float() + wm @ proj.bias.float())

    return _cached(block, "_ffn_in_fused", (lin.weight, lin.bias, proj.weight, proj.bias), dtype, build)


def ffn_pack(w1: torch.Tensor, w2: torch.Tensor, w3: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The one-launch FFN's weight streams (lg_ffn_pack, include/lightglue_glue.h) by tensor ops, the
    32-row kernel's layout then the 16-row kernel's. 32-row: for wave w of 8, W1 rows 64w.. as pieces
    (step j, block b), then W2 rows 32w.. as pieces (step j), then (lg_linear_cat_ffn_proj) W3 rows
    (n3/8)w.. as pieces (step j, block b); each piece's 16-B lane l = W[row0 + 32b + l % 32][16j +
    8(l // 32) : + 8]. 16-row: the same rows per wave in 16-row blocks and k32 steps, lane l =
    W[row0 + 16b + l % 16][32j + 8(l // 16) : + 8]."""
    def layout(rows, k):  # W [8 waves * blocks * rows, steps * k] -> (w, step, block, lane group, row, e)
        def f(w):
            nb = w.shape[0] // (8 * rows)
            g = k // 8
            return w.reshape(8, nb, rows, w.shape[1] // k, g, 8).permute(0, 3, 1, 4, 2, 5).reshape(8, -1)
        return f
    parts32 = [layout(32, 16)(w1), layout(32, 16)(w2)]
    parts16 = [layout(16, 32)(w1), layout(16, 32)(w2)]
    if w3 is not None:
        parts32.append(layout(32, 16)(w3))
        parts16.append(layout(16, 32)(w3))
    return torch.cat([torch.cat(parts32, 1).reshape(-1), torch.cat(parts16, 1).reshape(-1)]).contiguous()


def _ffn_packed(block: nn.Module, proj: nn.Linear, dtype: torch.dtype, w3=None):
    """ffn_pack of the block's folded FFN input weight and its output weight (cached like them), and
    with w3 = (tag, source parameters, builder of W3) the next projection's weight appended."""
    lin, out = block.ffn[0], block.ffn[3]
    tag, src, w3_build = w3 if w3 is not None else ("", (), None)

    def build():
        w, _ = _ffn_in_fused(block, proj, dtype)
        return (ffn_pack(w, out.weight.to(dtype), w3_build().to(dtype) if w3_build else None),)

    return _cached(block, "_ffn_packed" + tag, (lin.weight, lin.bias, proj.weight, proj.bias, out.weight) + tuple(src), dtype,
                   build)[0]


def _cross_qkv(ca: nn.Module, dtype: torch.dtype):
    """CrossBlock to_qk | to_v stacked (one projection; lightglue.py:158-166)."""
    return _cached(ca, "_qkv_stacked", (ca.to_qk.weight, ca.to_qk.bias, ca.to_v.weight, ca.to_v.bias), dtype,
                   lambda: (torch.cat((ca.to_qk.weight, ca.to_v.weight), 0), torch.cat((ca.to_qk.bias, ca.to_v.bias), 0)))


def _qkv_perm(block: nn.Module, dtype: torch.dtype):
    """Wqkv's rows and bias in [q|k|v][head][dim] order (lg_linear_qkv_rotary's layout): new row
    j*H*64 + h*64 + d = reference row (h*64 + d)*3 + j (lightglue.py:111-114)."""
    lin = block.Wqkv

    def build():
        hd = block.heads * block.head_dim
        new = torch.arange(3 * hd, device=lin.weight.device)
        j, hd_idx = new // hd, new % hd
        old = hd_idx * 3 + j
        return lin.weight[old], lin.bias[old]

    return _cached(block, "_qkv_perm", (lin.weight, lin.bias), dtype, build)


def _fused_ok(x: torch.Tensor, block: nn.Module) -> bool:
    """The fused-projection kernels: fp16, 4 x 64 heads (k = 256 / 512)."""
    return x.dtype == torch.float16 and block.heads * block.head_dim == 256 and x.shape[-1] == 256


def _ffn_tail(block: nn.Module, x: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
    """x + Linear(GELU(LayerNorm(h))) with LayerNorm+GELU as one gfx950 kernel."""
    return x + block.ffn[3](_Hip.layernorm_gelu(h, block.ffn[1]))


def _ffn_apply(ffn: nn.Sequential, h: torch.Tensor, hip: bool) -> torch.Tensor:
    """Linear -> LayerNorm -> GELU -> Linear (the LN+GELU pair is one gfx950 kernel on the hip path)."""
    if not hip:
        return ffn(h)
    return ffn[3](_Hip.layernorm_gelu(ffn[0](h), ffn[1]))


def _kernel_attention(calls):
    for q, _, _ in calls:
        if not q.is_cuda:
            raise PluginError("LightGlueMatcher: the attention op runs on the GPU only (no CPU fallback)")
    qs, ks, vs = (list(t) for t in zip(*calls))
    return torch.ops.lightglue_amd.mha_hd64_grouped(qs, ks, vs)  # ops.py: grouped launches


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

    def qkv(self, x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, splits: Sequence[int], hip: bool = False):
        """x [1, N0+N1, d] (both images' rows) -> per image (q, k, v), each [1, H, Ni, 64]."""
        n = x.shape[1]
        if hip:
            return _Hip.qkv_rotary_split(self.Wqkv(x), cos, sin, self.heads, splits)
        # Wqkv output channel (h*64 + d)*3 + j  ->  [3, H, N, 64] head-major
        t = self.Wqkv(x).view(n, self.heads, self.head_dim, 3).permute(3, 1, 0, 2)
        q = _rotary(t[0], cos, sin)
        k = _rotary(t[1], cos, sin)
        out, a = [], 0
        for ni in splits[:2]:
            out.append(tuple(u[:, a:a + ni].unsqueeze(0).contiguous() for u in (q, k, t[2])))
            a += ni
        return out

    def finish(self, x: torch.Tensor, contexts: Sequence[torch.Tensor], hip: bool = False) -> torch.Tensor:
        if hip:  # [x | heads merged] in one pass, out_proj folded into ffn[0]
            w, b = _ffn_in_fused(self, self.out_proj, x.dtype)
            return _ffn_tail(self, x, F.linear(_Hip.merge_heads_cat(x, *contexts), w, b))
        merged = torch.cat([c[0].transpose(0, 1).reshape(c.shape[2], -1) for c in contexts], 0)[None]
        return x + _ffn_apply(self.ffn, torch.cat((x, self.out_proj(merged)), -1), hip)


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
        for ni in splits[:2]:
            out.append(h[:, a:a + ni].unsqueeze(0).contiguous())
            a += ni
        return out

    def qk_v(self, x: torch.Tensor, splits: Sequence[int]):
        """hip path: to_qk and to_v as ONE GEMM on stacked weights, heads split from its halves."""
        w, b = _cached(self, "_qkv_stacked", (self.to_qk.weight, self.to_qk.bias, self.to_v.weight, self.to_v.bias),
                       x.dtype, lambda: (torch.cat((self.to_qk.weight, self.to_v.weight), 0),
                                         torch.cat((self.to_qk.bias, self.to_v.bias), 0)))
        return _Hip.split_heads2_ld(F.linear(x, w, b), self.heads, splits)

    def finish(self, x: torch.Tensor, ms: Sequence[torch.Tensor], hip: bool = False) -> torch.Tensor:
        if hip:  # [x | heads merged] in one pass, to_out folded into ffn[0]
            w, b = _ffn_in_fused(self, self.to_out, x.dtype)
            return _ffn_tail(self, x, F.linear(_Hip.merge_heads_cat(x, *ms), w, b))
        merged = torch.cat([m[0].transpose(0, 1).reshape(m.shape[2], -1) for m in ms], 0)[None]
        return x + _ffn_apply(self.ffn, torch.cat((x, self.to_out(merged)), -1), hip)


class TransformerLayer(nn.Module):
    def __init__(self, d: int, heads: int) -> None:
        super().__init__()
        self.self_attn = SelfBlock(d, heads)
        self.cross_attn = CrossBlock(d, heads)

    def forward(self, x, cos, sin, splits, attention: AttnFn, hip: bool = False):
        """x: both images' descriptors [1, N0+N1, d] (image 0 rows first)."""
        sa, ca = self.self_attn, self.cross_attn
        if hip and _fused_ok(x, sa):
            return self._forward_fused(x, cos, sin, splits, attention)
        x = sa.finish(x, attention(sa.qkv(x, cos, sin, splits, hip)), hip)   # one grouped launch (self0, self1)
        if hip:
            (qk0, qk1), (v0, v1) = ca.qk_v(x, splits)
        else:
            qk0, qk1 = ca.heads_of(ca.to_qk(x), splits)
            v0, v1 = ca.heads_of(ca.to_v(x), splits)
        return ca.finish(x, attention([(qk0, qk1, v1), (qk1, qk0, v0)]), hip)  # one grouped launch (cross)


    def _forward_fused(self, x, cos, sin, splits, attention: AttnFn):
        """fp16 hip path per block: projection (+rotary/head split), grouped attention, and the FFN
        with its residual in one launch (lg_linear_cat_ffn with the packed weight stream: the input
        projection gathering [x | heads], LayerNorm+GELU, the output projection + residual); the
        message projection is folded into the FFN's first weight."""
        sa, ca = self.self_attn, self.cross_attn
        wq, bq = _qkv_perm(sa, x.dtype)
        qkv = _Hip.linear_qkv_rotary(x, wq, bq, cos, sin, sa.heads, splits)
        c0, c1 = attention(qkv)                                          # self0, self1: one launch
        w0, b0 = _ffn_in_fused(sa, sa.out_proj, x.dtype)
        x = _Hip.ffn(x, c0, c1, w0, b0, sa.ffn[1], sa.ffn[3].weight, sa.ffn[3].bias, _ffn_packed(sa, sa.out_proj, x.dtype))
        wc, bc = _cross_qkv(ca, x.dtype)
        (qk0, qk1), (v0, v1) = _Hip.linear_split2(x, wc, bc, ca.heads, splits)
        m0, m1 = attention([(qk0, qk1, v1), (qk1, qk0, v0)])            # cross: one launch
        w0, b0 = _ffn_in_fused(ca, ca.to_out, x.dtype)
        return _Hip.ffn(x, m0, m1, w0, b0, ca.ffn[1], ca.ffn[3].weight, ca.ffn[3].bias, _ffn_packed(ca, ca.to_out, x.dtype))


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

    def hip16_ok(self, x: torch.Tensor, m: int, n: int) -> bool:
        return x.dtype == torch.float16 and x.is_cuda and x.shape[-1] == 256 and n % 8 == 0 and n <= 2048 and m <= 2048

    def aug_weights(self, dtype: torch.dtype, rows: int = 384):
        """[W_final / scale ; w_match ; 0] [rows, d] and its bias (the head's one projection, cached)."""
        fp, mt = self.final_proj, self.matchability
        d = fp.weight.shape[1]

        def build():
            w = torch.zeros((rows, d), dtype=torch.float32, device=fp.weight.device)
            b = torch.zeros((rows,), dtype=torch.float32, device=fp.weight.device)
            w[:d], b[:d] = fp.weight.float() / self.scale, fp.bias.float() / self.scale
            w[d], b[d] = mt.weight.float()[0], mt.bias.float()[0]
            return w, b

        return _cached(self, f"_assign_aug{rows}", (fp.weight, fp.bias, mt.weight, mt.bias), dtype, build)

    def forward_rows(self, x: torch.Tensor, pr: int, m: int, n: int) -> torch.Tensor:
        """fp16 hip path on both images' rows x [1, P*(m+n), d] at once: ONE projection with
        [W_final / scale ; w_match ; 0], then lg_assign_scores: the similarity of its fp16 halves by
        MFMA with each row's and column's logsumexp, and the combine (two launches, no framework op;
        lightglue.py:208-233). d^0.25 = 4 for d = 256, a power of two: dividing W and b by it is
        exact unless a quotient falls below 2^-14 (fp16 subnormals), where it loses up to 2 bits; so
        the output equals the reference's fp16(final_proj(d)) / scale except for weights, biases or
        outputs that small, which differ by at most that subnormal rounding."""
        d = x.shape[-1]
        w, b = self.aug_weights(x.dtype, 384)
        v = _Hip.linear(x, w, b).view(pr, m + n, 384)
        return _Hip.assign_scores(v, m, d)   # sim (fp16) and the dual log-softmax: two launches

    def forward(self, d0: torch.Tensor, d1: torch.Tensor, hip: bool = False) -> torch.Tensor:
        m0 = self.final_proj(d0) / self.scale
        m1 = self.final_proj(d1) / self.scale
        sim = (m0 @ m1.transpose(1, 2)).float()
        z0, z1 = self.matchability(d0).float(), self.matchability(d1).float()
        if hip:
            return _Hip.log_double_softmax(sim.contiguous(), z0.contiguous(), z1.contiguous())
        return log_double_softmax(sim, z0, z1)


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

    forward(kpts0 [P,M,2], kpts1 [P,N,2], desc0 [P,M,in], desc1 [P,N,in])
        -> (desc0 [P,M,d], desc1 [P,N,d], log-assignment scores [P,M,N] fp32)

    P image pairs of equal sizes go through one forward (the reference's pair loop,
    demo/demo_mono.cpp:194-418, batched): on the hip path every projection, glue kernel and the
    dual log-softmax runs once on all pairs' rows, and each layer's self / cross attention is one
    grouped launch of P-batch calls. glue='torch' runs the pairs one by one."""

    def __init__(self, n_layers: int = 9, descriptor_dim: int = 256, input_dim: int = 256, num_heads: int = 4,
                 filter_threshold: float = 0.1, attention: Optional[AttnFn] = None, glue: str = "hip") -> None:
        super().__init__()
        d = descriptor_dim
        self.n_layers, self.filter_threshold = n_layers, filter_threshold
        self.input_proj = nn.Linear(input_dim, d) if input_dim != d else nn.Identity()
        self.posenc = FourierPositionalEncoding(2, d // num_heads)
        self.transformers = nn.ModuleList([TransformerLayer(d, num_heads) for _ in range(n_layers)])
        self.log_assignment = nn.ModuleList([MatchAssignment(d) for _ in range(n_layers)])
        self.attention = attention or _kernel_attention
        if glue not in ("hip", "torch"):
            raise ValueError("glue must be 'hip' or 'torch'")
        self.glue = glue

    def pair_inputs_ok(self, kpts0, kpts1, desc0, desc1) -> bool:
        """lg_pair_inputs reads both descriptor sets, both keypoint sets and posenc.Wr as raw fp16
        [.., 256] / [.., 2] / [32, 2] rows: take it only when every one of them is exactly that (an
        fp32 model or mixed-dtype inputs take the framework path, which casts or raises)."""
        f16 = torch.float16
        return (isinstance(self.input_proj, nn.Identity) and all(t.dtype == f16 for t in (kpts0, kpts1, desc0, desc1))
                and self.posenc.Wr.weight.dtype == f16 and desc0.shape[-1] == 256 and desc1.shape[-1] == 256
                and kpts0.shape[-1] == 2 and kpts1.shape[-1] == 2 and tuple(self.posenc.Wr.weight.shape) == (32, 2))

    def forward(self, kpts0, kpts1, desc0, desc1):
        pr, m, n = desc0.shape[0], desc0.shape[1], desc1.shape[1]
        hip = self.glue == "hip"
        if not hip and pr > 1:  # the framework-op restatement: one pair at a time
            outs = [self.forward(kpts0[i:i + 1], kpts1[i:i + 1], desc0[i:i + 1], desc1[i:i + 1]) for i in range(pr)]
            return tuple(torch.cat(t, 0) for t in zip(*outs))
        splits = (m, n, pr)
        rows = pr * (m + n)
        if hip and not desc0.is_cuda:
            raise PluginError("LightGlueMatcher(glue='hip') runs on the GPU only (no CPU fallback)")
        if hip and self.pair_inputs_ok(kpts0, kpts1, desc0, desc1):  # pair-major rows + posenc in one launch
            x, cos, sin = _Hip.pair_inputs(desc0, desc1, kpts0, kpts1, self.posenc.Wr.weight)
        else:
            x = self.input_proj(torch.cat((desc0, desc1), 1))          # [P, M+N, d], pair-major rows
            cos, sin = self.posenc(torch.cat((kpts0, kpts1), 1).to(x.dtype))
            x = x.reshape(1, rows, x.shape[-1])
            cos, sin = cos.reshape(1, rows, -1), sin.reshape(1, rows, -1)  # [1, P*(M+N), 64], broadcast over heads
            if hip:
                cos, sin = cos.contiguous(), sin.contiguous()
        head = self.log_assignment[self.n_layers - 1]
        if hip and self.chain_ok(x, m, n):
            x, scores = self._forward_chain(x, cos, sin, splits)
        else:
            for layer in self.transformers:
                x = layer(x, cos, sin, splits, self.attention, hip)
            scores = head.forward_rows(x, pr, m, n) if hip and head.hip16_ok(x, m, n) else None
        x = x.view(pr, m + n, x.shape[-1])
        d0, d1 = x[:, :m], x[:, m:]
        return d0, d1, scores if scores is not None else head(d0, d1, hip)

    # Which projections the chained path folds into the FFN launch before them (s: the cross block's
    # to_qk | to_v, q: the next layer's Wqkv, h: the head's projection). Measured
    # (profiles/r06/chain_kinds_forward_ab.jsonl, ms per forward, none / s / h / sh / sqh): P = 1 n = 1024
    # 0.496 / 0.481 / 0.494 / 0.480 / 0.492, P = 4 0.790 / 0.729 / 0.747 / 0.723 / 0.772, P = 16 2.165 /
    # 2.133 / 2.163 / 2.128 / 2.183: "sh" with the 32-row FFN kernel; folding Wqkv (768 channels, 384 KiB
    # more per workgroup's stream) cost the launch more than the separate projection took. With the
    # 16-row kernel (up to 4,096 rows: twice the workgroups) and the QKV epilogues' rotary factors read
    # from a conflict-free table (prefetched, in the 16-row kernel), "sqh" wins at every size
    # (profiles/r06/chain_kinds_rows16_ab.jsonl, chain_kinds_sqh_ab.jsonl; sh / sqh: P = 1 n = 512 0.372 /
    # 0.367, n = 1024 0.440 / 0.420, n = 2048 0.679 / 0.634, P = 2 0.560 / 0.513, P = 4 0.724 / 0.709,
    # P = 8 1.195 / 1.159, P = 16 2.140 / 2.124). Outputs bitwise equal in every form. LG_CHAIN (or this
    # attribute) overrides, for A/B.
    chain_kinds: Optional[str] = None

    def _chain_kinds(self, rows: int) -> str:
        if self.chain_kinds is not None:
            return self.chain_kinds
        return os.environ.get("LG_CHAIN", "sqh")

    def chain_ok(self, x: torch.Tensor, m: int, n: int) -> bool:
        """The chained fp16 path: every block fusable (4 x 64 heads, d = 256) and the fp16 head."""
        return (self.n_layers > 0 and all(_fused_ok(x, layer.self_attn) for layer in self.transformers) and
                self.log_assignment[self.n_layers - 1].hip16_ok(x, m, n))

    def _forward_chain(self, x, cos, sin, splits):
        """fp16 hip path with the layers chained (round 6): FFN launches also project their output for
        the attention that follows (lg_linear_cat_ffn_proj) — by default the self block's FFN the cross
        block's to_qk | to_v, the cross block's FFN the next layer's Wqkv (+ rotary) and the last FFN
        the assignment head's [W_final / scale ; w_match] (chain_kinds) — so a layer is 4 launches (self
        attention, FFN + cross projection, cross attention, FFN + next projection) and a forward
        2 + 4 L + 2 (inputs, layer 0's Wqkv, the layers, the head's two; lightglue.py:328-353)."""
        dt = x.dtype
        m, n, pr = _sp(splits)
        kinds = self._chain_kinds(x.shape[1])
        layers = self.transformers
        head = self.log_assignment[len(layers) - 1]
        qkv = None
        for li, layer in enumerate(layers):
            sa, ca = layer.self_attn, layer.cross_attn
            if qkv is None:
                wq, bq = _qkv_perm(sa, dt)
                qkv = _Hip.linear_qkv_rotary(x, wq, bq, cos, sin, sa.heads, splits)
            c0, c1 = self.attention(qkv)                                          # self0, self1: one launch
            _, b0 = _ffn_in_fused(sa, sa.out_proj, dt)
            wc, bc = _cross_qkv(ca, dt)
            if "s" in kinds:
                pk = _ffn_packed(sa, sa.out_proj, dt, ("_x", (ca.to_qk.weight, ca.to_qk.bias, ca.to_v.weight, ca.to_v.bias),
                                                       lambda ca=ca: _cross_qkv(ca, dt)[0]))
                x, ((qk0, qk1), (v0, v1)) = _Hip.ffn_proj(x, c0, c1, b0, sa.ffn[1], sa.ffn[3].bias, pk, 1, bc, splits)
            else:
                w0, _ = _ffn_in_fused(sa, sa.out_proj, dt)
                x = _Hip.ffn(x, c0, c1, w0, b0, sa.ffn[1], sa.ffn[3].weight, sa.ffn[3].bias, _ffn_packed(sa, sa.out_proj, dt))
                (qk0, qk1), (v0, v1) = _Hip.linear_split2(x, wc, bc, ca.heads, splits)
            m0, m1 = self.attention([(qk0, qk1, v1), (qk1, qk0, v0)])          # cross: one launch
            w0, b0 = _ffn_in_fused(ca, ca.to_out, dt)
            qkv = v = None
            if li + 1 < len(layers) and "q" in kinds:
                nsa = layers[li + 1].self_attn
                _, bq = _qkv_perm(nsa, dt)
                pk = _ffn_packed(ca, ca.to_out, dt, ("_q", (nsa.Wqkv.weight, nsa.Wqkv.bias),
                                                     lambda nsa=nsa: _qkv_perm(nsa, dt)[0]))
                x, qkv = _Hip.ffn_proj(x, m0, m1, b0, ca.ffn[1], ca.ffn[3].bias, pk, 2, bq, splits, cos, sin)
            elif li + 1 == len(layers) and "h" in kinds:
                _, b3 = head.aug_weights(dt, 512)
                hp = (head.final_proj.weight, head.final_proj.bias, head.matchability.weight, head.matchability.bias)
                pk = _ffn_packed(ca, ca.to_out, dt, ("_h", hp, lambda head=head: head.aug_weights(dt, 512)[0]))
                x, v = _Hip.ffn_proj(x, m0, m1, b0, ca.ffn[1], ca.ffn[3].bias, pk, 3, b3, splits, n_store=384)
            else:
                x = _Hip.ffn(x, m0, m1, w0, b0, ca.ffn[1], ca.ffn[3].weight, ca.ffn[3].bias, _ffn_packed(ca, ca.to_out, dt))
        if v is None:
            w, b = head.aug_weights(dt, 384)
            v = _Hip.linear(x, w, b)
        return x, _Hip.assign_scores(v.view(pr, m + n, 384), m, x.shape[-1])

    def match(self, kpts0, kpts1, desc0, desc1):
        """forward + filter_matches (the demo's post-processing); for P > 1 pairs a list of
        (matches, scores), one per pair."""
        _, _, scores = self.forward(kpts0, kpts1, desc0, desc1)
        if scores.shape[0] == 1:
            return filter_matches(scores, self.filter_threshold)
        return [filter_matches(scores[i:i + 1], self.filter_threshold) for i in range(scores.shape[0])]


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


def synthetic_pair(seed: int, m: int, n: int, input_dim: int = 256, overlap: int = 0):
    """Keypoints in the normalised [-1, 1] frame and unit-norm descriptors, fp32, batch 1.

    overlap > 0: the first `overlap` keypoints of image 1 re-observe distinct keypoints of image 0
    (a seeded permutation; positions moved by ~0.01, descriptors perturbed by 0.2-std noise and
    renormalised), so the pair has real correspondences for the matcher to find."""
    k0 = synth.uniform24(seed * 4 + 0, m * 2).reshape(1, m, 2) * 2.0 - 1.0
    k1 = synth.uniform24(seed * 4 + 1, n * 2).reshape(1, n, 2) * 2.0 - 1.0
    d0 = synth.normal(seed * 4 + 2, (1, m, input_dim))
    d1 = synth.normal(seed * 4 + 3, (1, n, input_dim))
    d0 = d0 / np.linalg.norm(d0, axis=-1, keepdims=True)
    if overlap > 0:
        assert overlap <= min(m, n)
        src = np.argsort(synth.uniform24(seed * 4 + 5, m), kind="stable")[:overlap]
        k1[0, :overlap] = k0[0, src] + 0.01 * synth.normal(seed * 4 + 6, (overlap, 2))
        d1[0, :overlap] = d0[0, src] + 0.2 * synth.normal(seed * 4 + 7, (overlap, input_dim)) / np.sqrt(input_dim)
    d1 = d1 / np.linalg.norm(d1, axis=-1, keepdims=True)
    return tuple(torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)) for x in (k0, k1, d0, d1))

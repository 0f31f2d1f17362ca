"""torch.library operators over the plugin C ABI ("the caller is its own
PyTorch-ROCm module via a torch.library op that invokes enqueue on torch.cuda.current_stream()").

* ``torch.ops.lightglue_amd.mha_hd64(q, k, v) -> o``: the plugin's ``enqueue`` (the TensorRT node
  ``CustomOp::MHAHeadDim64``, lightglue_pytorch_with_plugin/lightglue.py:16-46): [1, 4, N, 64],
  all fp16 (-> fp16) or all fp32 (-> fp32).
* ``torch.ops.lightglue_amd.mha_hd64_grouped(qs, ks, vs) -> os``: up to any number of independent
  calls in grouped launches (4 per launch), e.g. the self0/self1 or the two cross directions of a
  LightGlue layer.

Only a CUDA (HIP) kernel is registered: a CPU tensor has no implementation to dispatch to and
raises (no CPU fallback). The fake (meta) implementations give shapes/dtypes for tracing.
"""
from __future__ import annotations

from typing import List

import torch

from .plugin import mha_hd64 as _enqueue
from .plugin import mha_hd64_grouped as _grouped


@torch.library.custom_op("lightglue_amd::mha_hd64", mutates_args=(), device_types="cuda")
def mha_hd64_op(query: torch.Tensor, key: torch.Tensor, value: torch.Tensor) -> torch.Tensor:
    return _enqueue(query.contiguous(), key.contiguous(), value.contiguous())


@mha_hd64_op.register_fake
def _(query, key, value):
    return torch.empty_like(query, memory_format=torch.contiguous_format)


@torch.library.custom_op("lightglue_amd::mha_hd64_grouped", mutates_args=(), device_types="cuda")
def mha_hd64_grouped_op(queries: List[torch.Tensor], keys: List[torch.Tensor],
                        values: List[torch.Tensor]) -> List[torch.Tensor]:
    return _grouped([(q.contiguous(), k.contiguous(), v.contiguous()) for q, k, v in zip(queries, keys, values)])


@mha_hd64_grouped_op.register_fake
def _(queries, keys, values):
    return [torch.empty_like(q, memory_format=torch.contiguous_format) for q in queries]

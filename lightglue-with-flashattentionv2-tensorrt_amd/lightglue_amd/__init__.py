"""MI355X-native MHAHeadDim64: the fused FlashAttention-v2 (head_dim 64) hot path of
qdLMF/LightGlue-with-FlashAttentionV2-TensorRT, as hand-written gfx950 HIP kernels behind
the reference plugin's configurePlugin()/enqueue() surface (C ABI: include/mha_hd64.h).
"""
from ._lib import LIB_PATH, LibraryMissing, load as load_library  # noqa: F401
from .plugin import (  # noqa: F401
    Attention,
    LightGlueAttentionPlugin,
    LightGlueAttentionPluginCreator,
    MHAHeadDim64,
    PluginError,
    mha_hd64,
    mha_hd64_batched,
    mha_hd64_grouped,
    set_concurrency_hint,
    set_stream_mode,
)
from . import ops  # noqa: F401,E402  (registers torch.ops.lightglue_amd.*)

__all__ = [
    "Attention",
    "LightGlueAttentionPlugin",
    "LightGlueAttentionPluginCreator",
    "MHAHeadDim64",
    "PluginError",
    "mha_hd64",
    "mha_hd64_batched",
    "mha_hd64_grouped",
    "set_concurrency_hint",
    "set_stream_mode",
    "load_library",
    "LIB_PATH",
]

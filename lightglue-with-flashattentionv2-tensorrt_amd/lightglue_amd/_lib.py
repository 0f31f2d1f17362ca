"""ctypes binding of the C ABI in include/mha_hd64.h (lib/libmha_hd64.so).

This is the reference-side binding a Python host adds in place of TensorRT's
``trtexec --plugins=liblightglue_attention_plugin.so`` / ``dlopen`` (steps.txt:135-179,
demo/lightglue_trt.cpp:15). The library is built in-tree by ``make`` in the package
directory (``__graft_entry__.build()``); there is deliberately no fallback: if the
shared library is missing, ``load()`` raises.
"""
from __future__ import annotations

import ctypes
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# MHA_HD64_LIB: test a diagnostic build (e.g. lib/exp/…) through the same suite.
LIB_PATH = os.environ.get("MHA_HD64_LIB") or os.path.join(PKG_DIR, "lib", "libmha_hd64.so")

DT_FLOAT = 0  # nvinfer1::DataType::kFLOAT
DT_HALF = 1   # nvinfer1::DataType::kHALF
FMT_LINEAR = 0  # nvinfer1::TensorFormat::kLINEAR

STATUS_SUCCESS = 0
STATUS_BAD_PARAM = 1
STATUS_LAUNCH_FAILED = 2
STATUS_WORKSPACE = 3

BATCH = 1
NUM_HEADS = 4
MAX_SEQ_LEN = 2048
HEAD_DIM = 64


class Dims(ctypes.Structure):
    _fields_ = [("nb_dims", ctypes.c_int32), ("d", ctypes.c_int64 * 8)]

    @classmethod
    def of(cls, shape) -> "Dims":
        shape = tuple(int(x) for x in shape)
        d = cls()
        d.nb_dims = len(shape)
        for i, x in enumerate(shape):
            d.d[i] = x
        return d

    def shape(self):
        return tuple(int(self.d[i]) for i in range(self.nb_dims))


class TensorDesc(ctypes.Structure):
    _fields_ = [("dims", Dims), ("type", ctypes.c_int32), ("format", ctypes.c_int32), ("scale", ctypes.c_float)]

    @classmethod
    def of(cls, shape, dtype: int, fmt: int = FMT_LINEAR) -> "TensorDesc":
        t = cls()
        t.dims = Dims.of(shape)
        t.type = dtype
        t.format = fmt
        t.scale = 1.0
        return t


class DynamicTensorDesc(ctypes.Structure):
    _fields_ = [("desc", TensorDesc), ("min", Dims), ("max", Dims)]

    @classmethod
    def of(cls, shape, dtype: int, fmt: int = FMT_LINEAR) -> "DynamicTensorDesc":
        t = cls()
        t.desc = TensorDesc.of(shape, dtype, fmt)
        t.min = Dims.of(shape)
        t.max = Dims.of(shape)
        return t


class CallDesc(ctypes.Structure):
    """Mirrors mha_hd64_call_t (one call of a grouped launch)."""
    _fields_ = [("q", ctypes.c_void_p), ("k", ctypes.c_void_p), ("v", ctypes.c_void_p), ("o", ctypes.c_void_p),
                ("batch", ctypes.c_int32), ("heads", ctypes.c_int32), ("nq", ctypes.c_int32),
                ("nkv", ctypes.c_int32)]


# Every symbol include/mha_hd64.h declares, with its ctypes signature.
_P = ctypes.c_void_p
_I = ctypes.c_int32
_S = ctypes.c_size_t
_C = ctypes.c_char_p
SIGNATURES = {
    "mha_hd64_creator_plugin_name": ([], _C),
    "mha_hd64_creator_plugin_version": ([], _C),
    "mha_hd64_creator_nb_fields": ([], _I),
    "mha_hd64_create_plugin": ([_C], _P),
    "mha_hd64_deserialize_plugin": ([_C, _P, _S], _P),
    "mha_hd64_destroy": ([_P], None),
    "mha_hd64_clone": ([_P], _P),
    "mha_hd64_initialize": ([_P], _I),
    "mha_hd64_terminate": ([_P], None),
    "mha_hd64_get_serialization_size": ([_P], _S),
    "mha_hd64_serialize": ([_P, _P], None),
    "mha_hd64_get_plugin_type": ([_P], _C),
    "mha_hd64_get_plugin_version": ([_P], _C),
    "mha_hd64_set_plugin_namespace": ([_P, _C], None),
    "mha_hd64_get_plugin_namespace": ([_P], _C),
    "mha_hd64_attach_to_context": ([_P], None),
    "mha_hd64_detach_from_context": ([_P], None),
    "mha_hd64_get_nb_outputs": ([_P], _I),
    "mha_hd64_get_output_dimensions": ([_P, _I, ctypes.POINTER(Dims), _I, ctypes.POINTER(Dims)], _I),
    "mha_hd64_supports_format_combination": ([_P, _I, ctypes.POINTER(TensorDesc), _I, _I], _I),
    "mha_hd64_get_output_data_type": ([_P, _I, ctypes.POINTER(ctypes.c_int32), _I, ctypes.POINTER(ctypes.c_int32)], _I),
    "mha_hd64_configure_plugin": ([_P, ctypes.POINTER(DynamicTensorDesc), _I, ctypes.POINTER(DynamicTensorDesc), _I], _I),
    "mha_hd64_get_workspace_size": ([_P, ctypes.POINTER(TensorDesc), _I, ctypes.POINTER(TensorDesc), _I], _S),
    "mha_hd64_enqueue": ([_P, ctypes.POINTER(TensorDesc), ctypes.POINTER(TensorDesc),
                          ctypes.POINTER(_P), ctypes.POINTER(_P), _P, _P], _I),
    "mha_hd64_launch_fp16in_fp16out": ([_P, _P, _P, _P, _I, _I, _I, _I, _P, _S, _P], _I),
    "mha_hd64_launch_fp16in_fp32out": ([_P, _P, _P, _P, _I, _I, _I, _I, _P, _S, _P], _I),
    "mha_hd64_launch_fp32in_fp32out": ([_P, _P, _P, _P, _I, _I, _I, _I, _P, _S, _P], _I),
    "mha_hd64_launch_workspace_bytes": ([_I, _I, _I, _I], _S),
    "mha_hd64_launch_workspace_bytes_typed": ([_I, _I, _I, _I, _I], _S),
    "mha_hd64_launch_grouped": ([ctypes.POINTER(CallDesc), _I, _I, _I, _P, _S, _P], _I),
    "mha_hd64_grouped_workspace_bytes": ([ctypes.POINTER(CallDesc), _I], _S),
    "mha_hd64_grouped_workspace_bytes_typed": ([ctypes.POINTER(CallDesc), _I, _I], _S),
    "mha_hd64_set_concurrency_hint": ([_I], _I),
    "mha_hd64_last_error": ([], _C),
    "mha_hd64_set_abort_on_error": ([_I], None),
    "mha_hd64_build_info": ([], _C),
}
# include/lightglue_glue.h (matcher kernels around the op)
_F = ctypes.POINTER(ctypes.c_float)
SIGNATURES.update({
    "lg_qkv_rotary_split": ([_I, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P], _I),
    "lg_split_heads2": ([_I, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P], _I),
    "lg_merge_heads": ([_I, _P, _P, _I, _I, _I, _I, _P, _P], _I),
    "lg_split_heads2_ld": ([_I, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P], _I),
    "lg_merge_heads_cat": ([_I, _P, _P, _P, _I, _I, _I, _I, _P, _P], _I),
    "lg_linear": ([_P, _P, _P, _P, _I, _I, _I, _P, _P], _I),
    "lg_linear_cat": ([_P, _P, _P, _I, _I, _I, _I, _P, _P, _I, _P, _P], _I),
    "lg_linear_cat_ln_gelu": ([_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, ctypes.c_float, _P, _P], _I),
    "lg_linear_cat_ffn": ([_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, ctypes.c_float, _P, _P, _P, _P, _P, _P], _I),
    "lg_ffn_packed_bytes": ([_I, _I], _S),
    "lg_assign_scores_workspace": ([_I, _I, _I], _S),
    "lg_assign_scores": ([_P, ctypes.c_int64, _I, _I, _I, _I, _I, _P, _P, _P], _I),
    "lg_ffn_pack": ([_P, _P, _P, _I, _I, _P, _P], _I),
    "lg_linear_cat_ffn_proj": ([_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, ctypes.c_float, _P, _P, _I, _P, _P, _P, _I,
                                ctypes.POINTER(_P), _P, _P], _I),
    "lg_linear_qkv_rotary": ([_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P], _I),
    "lg_linear_split2": ([_P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P], _I),
    "lg_layernorm_gelu": ([_I, _P, _P, _P, _I, _I, ctypes.c_float, _P, _P], _I),
    "lg_log_double_softmax_workspace": ([_I, _I, _I], _S),
    "lg_log_double_softmax": ([_P, _P, _P, _I, _I, _I, _P, _P, _P], _I),
    "lg_linear_set_wide": ([_I], _I),
    "lg_glue_abi_version": ([], _I),
    "lg_log_double_softmax_f16_workspace": ([_I, _I, _I], _S),
    "lg_log_double_softmax_f16": ([_P, _P, _P, ctypes.c_int64, ctypes.c_int64, _I, _I, _I, _P, _P, _P], _I),
    "lg_pair_inputs": ([_P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P], _I),
    "lg_linear_set_ln_fused": ([_I], _I),
    "lg_linear_set_ffn_fused": ([_I], _I),
    # kernel-form switches (include/mha_hd64.h "kernel-form switches")
    "mha_hd64_set_fused_combine": ([_I], None),
    "mha_hd64_set_f32_inkernel": ([_I], None),
    "mha_hd64_set_stream_mode": ([_I], _I),
    # test and benchmark hooks (include/mha_hd64.h "test and benchmark hooks")
    "mha_hd64_launch_forced": ([_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _S, _P, _I], _I),
    "mha_hd64_plan": ([_I, _I, _I, _I, _S, ctypes.POINTER(ctypes.c_int32)], _S),
    "mha_hd64_set_stamp_buffer": ([_P], None),
    "mha_hd64_last_combine_form": ([], _I),
})
HOOKS = {}  # (every export is declared in include/mha_hd64.h since round 4)

_lib = None


class LibraryMissing(RuntimeError):
    pass


GLUE_ABI_VERSION = 4  # include/lightglue_glue.h LG_GLUE_ABI_VERSION


def load() -> ctypes.CDLL:
    """Load lib/libmha_hd64.so (build it with __graft_entry__.build()). Raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LibraryMissing(
            f"{LIB_PATH} not found: the MI355X HIP extension is not built "
            "(run `python -c 'import __graft_entry__ as g; g.build()'` or `make -C "
            f"{PKG_DIR}`). There is no CPU fallback.")
    try:  # bind to the HIP runtime torch already loaded, if torch is in use
        import torch  # noqa: F401
    except Exception:  # pragma: no cover
        pass
    lib = ctypes.CDLL(LIB_PATH)
    stale = (f"{LIB_PATH} is stale (built from older sources than this package binds): rebuild it with "
             f"`make -C {PKG_DIR}`")
    # the version first: a library older than the query lacks it (and other symbols bound below)
    try:
        ver_fn = lib.lg_glue_abi_version
    except AttributeError:
        raise LibraryMissing(f"{stale}; it has no lg_glue_abi_version") from None
    ver_fn.argtypes, ver_fn.restype = [], _I
    if ver_fn() != GLUE_ABI_VERSION:  # the argument lists below match this ABI only
        raise LibraryMissing(f"{stale}; glue ABI {ver_fn()}, this package binds {GLUE_ABI_VERSION}")
    for table in (SIGNATURES, HOOKS):
        for name, (args, res) in table.items():
            try:
                fn = getattr(lib, name)
            except AttributeError:
                raise LibraryMissing(f"{stale}; it does not export {name}") from None
            fn.argtypes = args
            fn.restype = res
    _lib = lib
    return lib


def last_error() -> str:
    msg = load().mha_hd64_last_error()
    return msg.decode() if msg else ""

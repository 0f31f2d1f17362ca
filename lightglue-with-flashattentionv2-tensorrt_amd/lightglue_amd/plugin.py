"""Host-side mirror of the reference's MHAHeadDim64 plugin and its PyTorch call site.

Reference interfaces mirrored here:

* ``LightGlueAttentionPlugin`` / ``LightGlueAttentionPluginCreator`` —
  lightglue_attention_plugin/lightglue_attention_plugin.h:28-159 (IPluginV2DynamicExt /
  IPluginCreator). Same method names (snake_case), argument meaning and results; each
  call goes through the C ABI of include/mha_hd64.h. Where the reference's
  PLUGIN_ASSERT would abort the process, these methods raise ``PluginError``.
* ``MHAHeadDim64`` — the autograd Function of lightglue_pytorch_with_plugin/lightglue.py:16-46:
  the same ONNX symbolic (``CustomOp::MHAHeadDim64``, output typed like the query) and a
  forward that runs the MI355X kernel through ``enqueue`` on the current HIP stream
  (the reference's eager forward is an SDPA; its TensorRT engine runs the plugin).
* ``Attention`` — lightglue_pytorch_with_plugin/lightglue.py:102-115.

There is no CPU fallback: CPU tensors raise, and a missing shared library raises.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Sequence, Tuple

import torch
from torch import nn

from . import _lib
from ._lib import DT_FLOAT, DT_HALF, FMT_LINEAR, Dims, DynamicTensorDesc, TensorDesc


class PluginError(RuntimeError):
    """A contract violation the reference would have turned into PLUGIN_ASSERT -> abort()."""


def _check(status: int, what: str) -> None:
    if status != _lib.STATUS_SUCCESS:
        raise PluginError(f"{what} failed (status {status}): {_lib.last_error()}")


def _desc_array(descs: Sequence[TensorDesc]):
    arr = (TensorDesc * len(descs))()
    for i, d in enumerate(descs):
        arr[i] = d
    return arr


def _dyn_array(descs: Sequence[DynamicTensorDesc]):
    arr = (DynamicTensorDesc * len(descs))()
    for i, d in enumerate(descs):
        arr[i] = d
    return arr


def torch_dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float16:
        return DT_HALF
    if t.dtype == torch.float32:
        return DT_FLOAT
    raise PluginError(f"unsupported dtype {t.dtype}: MHAHeadDim64 takes float16 or float32")


def tensor_desc(t: torch.Tensor) -> TensorDesc:
    fmt = FMT_LINEAR if t.is_contiguous() else 1  # anything but kLINEAR is rejected by the plugin
    return TensorDesc.of(t.shape, torch_dtype_code(t), fmt)


class LightGlueAttentionPlugin:
    """Python face of one ``mha_hd64_plugin_t`` (lightglue_attention_plugin.h:28-121)."""

    def __init__(self, handle=None):
        lib = _lib.load()
        self._lib = lib
        self._h = handle if handle is not None else lib.mha_hd64_create_plugin(b"")
        if not self._h:
            raise PluginError(f"createPlugin failed: {_lib.last_error()}")

    # -- lifetime / identity (.cpp:28-77) --
    def initialize(self) -> int:
        return self._lib.mha_hd64_initialize(self._h)

    def terminate(self) -> None:
        self._lib.mha_hd64_terminate(self._h)

    def destroy(self) -> None:
        if self._h:
            self._lib.mha_hd64_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass

    def clone(self) -> "LightGlueAttentionPlugin":
        return LightGlueAttentionPlugin(self._lib.mha_hd64_clone(self._h))

    def get_serialization_size(self) -> int:
        return self._lib.mha_hd64_get_serialization_size(self._h)

    def serialize(self) -> bytes:
        n = self.get_serialization_size()
        buf = ctypes.create_string_buffer(max(n, 1))
        self._lib.mha_hd64_serialize(self._h, buf)
        return buf.raw[:n]

    def get_plugin_type(self) -> str:
        return self._lib.mha_hd64_get_plugin_type(self._h).decode()

    def get_plugin_version(self) -> str:
        return self._lib.mha_hd64_get_plugin_version(self._h).decode()

    def set_plugin_namespace(self, ns: str) -> None:
        self._lib.mha_hd64_set_plugin_namespace(self._h, ns.encode())

    def get_plugin_namespace(self) -> str:
        return self._lib.mha_hd64_get_plugin_namespace(self._h).decode()

    def attach_to_context(self) -> None:
        self._lib.mha_hd64_attach_to_context(self._h)

    def detach_from_context(self) -> None:
        self._lib.mha_hd64_detach_from_context(self._h)

    def get_nb_outputs(self) -> int:
        return self._lib.mha_hd64_get_nb_outputs(self._h)

    # -- build-time queries (.cpp:79-112, 272-359) --
    def get_output_dimensions(self, output_index: int, inputs_dims: Sequence[Sequence[int]]) -> Tuple[int, ...]:
        arr = (Dims * len(inputs_dims))()
        for i, s in enumerate(inputs_dims):
            arr[i] = Dims.of(s)
        out = Dims()
        _check(self._lib.mha_hd64_get_output_dimensions(self._h, output_index, arr, len(inputs_dims),
                                                        ctypes.byref(out)), "getOutputDimensions")
        return out.shape()

    def supports_format_combination(self, pos: int, in_out: Sequence[TensorDesc], nb_inputs: int,
                                    nb_outputs: int) -> bool:
        r = self._lib.mha_hd64_supports_format_combination(self._h, pos, _desc_array(in_out), nb_inputs, nb_outputs)
        if r < 0:
            raise PluginError(f"supportsFormatCombination: {_lib.last_error()}")
        return bool(r)

    def get_output_data_type(self, output_index: int, inputs_type: Sequence[int]) -> int:
        arr = (ctypes.c_int32 * len(inputs_type))(*inputs_type)
        out = ctypes.c_int32(-1)
        _check(self._lib.mha_hd64_get_output_data_type(self._h, output_index, arr, len(inputs_type),
                                                       ctypes.byref(out)), "getOutputDataType")
        return out.value

    def configure_plugin(self, inputs: Sequence[DynamicTensorDesc], outputs: Sequence[DynamicTensorDesc]) -> None:
        _check(self._lib.mha_hd64_configure_plugin(self._h, _dyn_array(inputs), len(inputs), _dyn_array(outputs),
                                                   len(outputs)), "configurePlugin")

    def get_workspace_size(self, inputs: Sequence[TensorDesc], outputs: Sequence[TensorDesc]) -> int:
        return self._lib.mha_hd64_get_workspace_size(self._h, _desc_array(inputs), len(inputs),
                                                     _desc_array(outputs), len(outputs))

    # -- run time (.cpp:114-270) --
    def enqueue(self, inputs_desc: Sequence[TensorDesc], outputs_desc: Sequence[TensorDesc],
                inputs: Sequence[int], outputs: Sequence[int], workspace: int, stream: int) -> int:
        ins = (ctypes.c_void_p * len(inputs))(*inputs)
        outs = (ctypes.c_void_p * len(outputs))(*outputs)
        status = self._lib.mha_hd64_enqueue(self._h, _desc_array(inputs_desc), _desc_array(outputs_desc), ins, outs,
                                            workspace, stream)
        _check(status, "enqueue")
        return status


class LightGlueAttentionPluginCreator:
    """lightglue_attention_plugin.h:125-159."""

    def __init__(self):
        self._lib = _lib.load()
        self._namespace = ""

    def get_plugin_name(self) -> str:
        return self._lib.mha_hd64_creator_plugin_name().decode()

    def get_plugin_version(self) -> str:
        return self._lib.mha_hd64_creator_plugin_version().decode()

    def set_plugin_namespace(self, ns: str) -> None:
        self._namespace = ns

    def get_plugin_namespace(self) -> str:
        return self._namespace

    def get_field_names(self) -> list:
        return [None] * self._lib.mha_hd64_creator_nb_fields()

    def create_plugin(self, name: str = "", fields=None) -> LightGlueAttentionPlugin:
        p = LightGlueAttentionPlugin(self._lib.mha_hd64_create_plugin(name.encode()))
        p.set_plugin_namespace(self._namespace)
        return p

    def deserialize_plugin(self, name: str, data: bytes) -> LightGlueAttentionPlugin:
        buf = ctypes.create_string_buffer(data, max(len(data), 1))
        p = LightGlueAttentionPlugin(self._lib.mha_hd64_deserialize_plugin(name.encode(), buf, len(data)))
        p.set_plugin_namespace(self._namespace)
        return p


# ---------------------------------------------------------------------------------------
# Torch glue: one plugin object per process, one workspace per (device, stream), as the
# TensorRT execution context would own (the plugin itself owns nothing, .cpp:114-175).
# ---------------------------------------------------------------------------------------
_plugin = None
_workspaces: Dict[Tuple[int, int], torch.Tensor] = {}


def get_plugin() -> LightGlueAttentionPlugin:
    global _plugin
    if _plugin is None:
        _plugin = LightGlueAttentionPlugin()
    return _plugin


def _workspace(device: torch.device, stream: int, nbytes: int) -> torch.Tensor:
    key = (device.index if device.index is not None else torch.cuda.current_device(), stream)
    ws = _workspaces.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=device)
        _workspaces[key] = ws
    return ws


def set_concurrency_hint(streams: int) -> int:
    """Tell the planner how many independent enqueue streams are kept busy at once (C ABI
    mha_hd64_set_concurrency_hint): 1 = every call may fill the chip; 2 = calls take half the CUs
    so two streams overlap; >= 3 = half-LDS two-per-CU blocks so up to four share the chip.
    Process-wide; returns the previous value."""
    return int(_lib.load().mha_hd64_set_concurrency_hint(int(streams)))


def set_stream_mode(mode: int) -> int:
    """1 (default): fp16 launches of more than 256 128-row blocks (batched image-pair streams,
    large grouped layers) run the persistent streaming kernel (csrc/mha_hd64_stream.hip); 0: the
    planner's other plans (the LDS-ring kernel there). Same results within the contract (DESIGN.md
    section 3). Process-wide (MHA_HD64_STREAM=0 sets 0 at first use). Returns the previous mode."""
    return int(_lib.load().mha_hd64_set_stream_mode(int(mode)))


def _require_gpu(*ts: torch.Tensor) -> None:
    for t in ts:
        if not t.is_cuda:
            raise PluginError("MHAHeadDim64 runs on the GPU only (no CPU fallback); got a CPU tensor")


def mha_hd64(query: torch.Tensor, key: torch.Tensor, value: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """Run the plugin's enqueue() on the current stream: O = softmax(Q·Kᵀ/8)·V.

    Same contract as the TensorRT node ``CustomOp::MHAHeadDim64``: [1, 4, N, 64]
    contiguous tensors, all float16 or all float32, Nq, Nkv <= 2048."""
    _require_gpu(query, key, value)
    if out is None:
        out = torch.empty_like(query, memory_format=torch.contiguous_format)
    plugin = get_plugin()
    in_desc = [tensor_desc(query), tensor_desc(key), tensor_desc(value)]
    out_desc = [tensor_desc(out)]
    stream = torch.cuda.current_stream(query.device).cuda_stream
    nbytes = plugin.get_workspace_size(in_desc, out_desc)
    ws = _workspace(query.device, stream, nbytes)
    plugin.enqueue(in_desc, out_desc, [query.data_ptr(), key.data_ptr(), value.data_ptr()], [out.data_ptr()],
                   ws.data_ptr(), stream)
    return out


def bound_enqueue(query: torch.Tensor, key: torch.Tensor, value: torch.Tensor, out: torch.Tensor):
    """The enqueue() of mha_hd64 with its bindings prepared once, as a TensorRT execution context
    holds them between inferences: descriptors, pointer arrays, workspace and stream are fixed here
    (the current stream at bind time), and each call of the returned function is one C-ABI
    mha_hd64_enqueue of the plugin (lightglue_attention_plugin.cpp's enqueue) and nothing else."""
    _require_gpu(query, key, value)
    for t in (query, key, value, out):
        if not t.is_contiguous():
            raise PluginError("bound_enqueue needs contiguous tensors")
    plugin = get_plugin()
    in_desc = [tensor_desc(query), tensor_desc(key), tensor_desc(value)]
    out_desc = [tensor_desc(out)]
    stream = torch.cuda.current_stream(query.device).cuda_stream
    ws = _workspace(query.device, stream, plugin.get_workspace_size(in_desc, out_desc))
    args = (plugin._h, _desc_array(in_desc), _desc_array(out_desc),
            (ctypes.c_void_p * 3)(query.data_ptr(), key.data_ptr(), value.data_ptr()),
            (ctypes.c_void_p * 1)(out.data_ptr()), ws.data_ptr(), stream)
    fn = plugin._lib.mha_hd64_enqueue

    def enqueue() -> None:
        status = fn(*args)
        if status != _lib.STATUS_SUCCESS:
            _check(status, "enqueue")
    enqueue.keep = (query, key, value, out, ws)      # the bound buffers outlive the closure's users
    return enqueue


_LAUNCHERS = {
    (torch.float16, torch.float16): "mha_hd64_launch_fp16in_fp16out",
    (torch.float16, torch.float32): "mha_hd64_launch_fp16in_fp32out",
    (torch.float32, torch.float32): "mha_hd64_launch_fp32in_fp32out",
}


def mha_hd64_batched(query: torch.Tensor, key: torch.Tensor, value: torch.Tensor, out_dtype=None,
                     out: torch.Tensor = None) -> torch.Tensor:
    """L0 launcher path (AttentionHeadDim64::launch_*): [B, H, N, 64] for any B, H.

    Stacking the independent calls of several image pairs (or the self0/self1 and the
    two cross directions of one layer) into the batch dimension runs them as one launch."""
    _require_gpu(query, key, value)
    out_dtype = out_dtype or query.dtype
    fn_name = _LAUNCHERS.get((query.dtype, out_dtype))
    if fn_name is None:
        raise PluginError(f"no launcher for {query.dtype} -> {out_dtype}")
    for t in (query, key, value):
        if not t.is_contiguous() or t.dim() != 4 or t.shape[-1] != 64 or t.dtype != query.dtype:
            raise PluginError("expected contiguous [B, H, N, 64] tensors of one dtype")
    b, h, nq, _ = query.shape
    nkv = key.shape[2]
    if key.shape != value.shape or key.shape[:2] != query.shape[:2]:
        raise PluginError("key/value shape mismatch")
    if out is None:
        out = torch.empty(query.shape, dtype=out_dtype, device=query.device)
    lib = _lib.load()
    stream = torch.cuda.current_stream(query.device).cuda_stream
    # (fp32 inputs: room for the fp16 copies when the planner converts before a single-pass kernel)
    nbytes = lib.mha_hd64_launch_workspace_bytes_typed(b, h, nq, nkv, _DT[query.dtype])
    ws = _workspace(query.device, stream, nbytes) if nbytes else None
    status = getattr(lib, fn_name)(query.data_ptr(), key.data_ptr(), value.data_ptr(), out.data_ptr(), b, h, nq,
                                   nkv, ws.data_ptr() if ws is not None else None, nbytes, stream)
    _check(status, fn_name)
    return out


_DT = {torch.float16: _lib.DT_HALF, torch.float32: _lib.DT_FLOAT}


def mha_hd64_grouped(calls, out_dtype=None, outs=None):
    """Grouped launcher: several independent calls [(q, k, v), ...] of possibly different shapes
    ([B, H, Nq_i, 64] / [B, H, Nkv_i, 64]) in one launch (up to 4 per launch, chunked beyond).

    The four attention calls of a LightGlue layer (self0, self1, cross0->1, cross1->0;
    lightglue_pytorch_with_plugin/lightglue.py:137-152, 188-205) run as two such launches."""
    calls = list(calls)
    if not calls:
        return []
    in_dtype = calls[0][0].dtype
    out_dtype = out_dtype or in_dtype
    if in_dtype not in _DT or out_dtype not in _DT:
        raise PluginError(f"unsupported dtypes {in_dtype} -> {out_dtype}")
    if outs is None:
        outs = [torch.empty(q.shape, dtype=out_dtype, device=q.device) for q, _, _ in calls]
    descs = (_lib.CallDesc * len(calls))()
    for i, ((q, k, v), o) in enumerate(zip(calls, outs)):
        _require_gpu(q, k, v, o)
        for t in (q, k, v):
            if not t.is_contiguous() or t.dim() != 4 or t.shape[-1] != 64 or t.dtype != in_dtype:
                raise PluginError("expected contiguous [B, H, N, 64] tensors of one dtype")
        if k.shape != v.shape or k.shape[:2] != q.shape[:2] or o.shape != q.shape or o.dtype != out_dtype:
            raise PluginError("shape mismatch in grouped call")
        descs[i] = _lib.CallDesc(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), q.shape[0], q.shape[1],
                                 q.shape[2], k.shape[2])
    lib = _lib.load()
    device = calls[0][0].device
    stream = torch.cuda.current_stream(device).cuda_stream
    # (fp32 groups: includes the fp16 copies of Q/K/V the convert launch writes when a single-pass
    # kernel that does not round fp32 inputs itself runs them; largest chunk of 4 calls)
    nbytes = lib.mha_hd64_grouped_workspace_bytes_typed(descs, len(calls), _DT[in_dtype])
    ws = _workspace(device, stream, nbytes) if nbytes else None
    status = lib.mha_hd64_launch_grouped(descs, len(calls), _DT[in_dtype], _DT[out_dtype],
                                         ws.data_ptr() if ws is not None else None, nbytes, stream)
    _check(status, "mha_hd64_launch_grouped")
    return outs


class MHAHeadDim64(torch.autograd.Function):
    """lightglue_pytorch_with_plugin/lightglue.py:16-46, forward on the MI355X kernel."""

    @staticmethod
    def symbolic(g, query, key, value):
        return g.op("CustomOp::MHAHeadDim64", query, key, value).setType(
            query.type().with_sizes([
                torch.onnx.symbolic_helper._get_tensor_dim_size(query, 0),
                torch.onnx.symbolic_helper._get_tensor_dim_size(query, 1),
                torch.onnx.symbolic_helper._get_tensor_dim_size(query, 2),
                torch.onnx.symbolic_helper._get_tensor_dim_size(query, 3),
            ]))

    @staticmethod
    def forward(ctx, query, key, value):
        return torch.ops.lightglue_amd.mha_hd64(query, key, value)  # ops.py: enqueue on the current stream


class Attention(nn.Module):
    """lightglue_pytorch_with_plugin/lightglue.py:102-115."""

    def forward(self, query, key, value) -> torch.Tensor:
        return MHAHeadDim64.apply(query, key, value)

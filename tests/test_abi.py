"""C-ABI boundary tests that need no GPU: the library loads, exports every symbol that
include/mha_hd64.h declares, and the plugin's host-side contract mirrors the reference
(lightglue_attention_plugin/lightglue_attention_plugin.cpp:28-422)."""
import ctypes
import importlib.util
import os
import re
import shutil
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

HEADERS = [os.path.join(REPO, "include", h) for h in ("mha_hd64.h", "lightglue_glue.h")]


def header_functions():
    names = set()
    for h in HEADERS:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b((?:mha_hd64|lg)_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


@pytest.fixture(scope="module")
def lib():
    from lightglue_amd import _lib

    return _lib.load()


@pytest.fixture()
def plugin():
    from lightglue_amd import LightGlueAttentionPlugin

    p = LightGlueAttentionPlugin()
    yield p
    p.destroy()


def desc(shape, dt=1, fmt=0):
    from lightglue_amd._lib import TensorDesc

    return TensorDesc.of(shape, dt, fmt)


def dyn(shape, dt=1, fmt=0):
    from lightglue_amd._lib import DynamicTensorDesc

    return DynamicTensorDesc.of(shape, dt, fmt)


def test_every_header_symbol_is_exported(lib):
    from lightglue_amd import _lib

    names = header_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(lib, n), n
        assert n in _lib.SIGNATURES, f"{n} has no ctypes signature"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T ((?:mha_hd64|lg)_\w+)", out))
    assert set(names) <= exported
    # ... and the other way round: no exported C entry point lacks a prototype a C host can bind
    undeclared = sorted(exported - set(names))
    assert not undeclared, f"exported without a declaration in include/*.h: {undeclared}"


def test_library_is_gfx950_code_object(lib):
    from lightglue_amd import _lib

    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data, "no gfx950 code object in the fat binary"
    assert b"gfx950" in ctypes.string_at(lib.mha_hd64_build_info())


def test_identity(plugin):
    from lightglue_amd import LightGlueAttentionPluginCreator

    c = LightGlueAttentionPluginCreator()
    assert c.get_plugin_name() == "MHAHeadDim64" and c.get_plugin_version() == "1"
    assert c.get_field_names() == []
    assert plugin.get_plugin_type() == "MHAHeadDim64" and plugin.get_plugin_version() == "1"
    assert plugin.get_plugin_namespace() == ""
    plugin.set_plugin_namespace("ns")
    assert plugin.get_plugin_namespace() == "ns"
    assert plugin.clone().get_plugin_namespace() == "ns"
    assert plugin.get_nb_outputs() == 1
    assert plugin.initialize() == 0
    assert plugin.get_serialization_size() == 0 and plugin.serialize() == b""
    p2 = c.deserialize_plugin("MHAHeadDim64", b"")
    assert p2.get_plugin_type() == "MHAHeadDim64"
    plugin.attach_to_context()
    plugin.detach_from_context()


def test_output_dimensions(plugin):
    from lightglue_amd import PluginError

    assert plugin.get_output_dimensions(0, [(1, 4, 100, 64), (1, 4, 77, 64), (1, 4, 77, 64)]) == (1, 4, 100, 64)
    with pytest.raises(PluginError):
        plugin.get_output_dimensions(1, [(1, 4, 100, 64)] * 3)
    with pytest.raises(PluginError):
        plugin.get_output_dimensions(0, [(1, 4, 100, 64)] * 2)
    with pytest.raises(PluginError):
        plugin.get_output_dimensions(0, [(4, 100, 64), (1, 4, 1, 64), (1, 4, 1, 64)])


def test_output_data_type(plugin):
    assert plugin.get_output_data_type(0, [1, 1, 1]) == 1
    assert plugin.get_output_data_type(0, [0, 0, 0]) == 0


def test_supports_format_combination(plugin):
    from lightglue_amd import PluginError

    half = [desc((1, 4, 8, 64), 1)] * 4
    flt = [desc((1, 4, 8, 64), 0)] * 4
    for pos in range(4):
        assert plugin.supports_format_combination(pos, half, 3, 1)
        assert plugin.supports_format_combination(pos, flt, 3, 1)
    mixed = [desc((1, 4, 8, 64), 1), desc((1, 4, 8, 64), 0), desc((1, 4, 8, 64), 1), desc((1, 4, 8, 64), 1)]
    assert not plugin.supports_format_combination(1, mixed, 3, 1)
    int8 = [desc((1, 4, 8, 64), 2)] + half[1:]
    assert not plugin.supports_format_combination(0, int8, 3, 1)
    chw = [desc((1, 4, 8, 64), 1, fmt=1)] + half[1:]
    assert not plugin.supports_format_combination(0, chw, 3, 1)
    with pytest.raises(PluginError):
        plugin.supports_format_combination(4, half, 3, 1)


def test_workspace_size_is_fixed(plugin):
    for n in (1, 64, 1000, 2048):
        ins = [desc((1, 4, n, 64))] * 3
        assert plugin.get_workspace_size(ins, [desc((1, 4, n, 64))]) == 5242880


GOOD = ((1, 4, 1000, 64), (1, 4, 777, 64), (1, 4, 777, 64), (1, 4, 1000, 64))


def _cfg(plugin, shapes, types=(1, 1, 1, 1), fmts=(0, 0, 0, 0)):
    ins = [dyn(s, t, f) for s, t, f in zip(shapes[:3], types[:3], fmts[:3])]
    return plugin.configure_plugin(ins, [dyn(shapes[3], types[3], fmts[3])])


BAD = {
    "batch2": ((2, 4, 10, 64), (2, 4, 10, 64), (2, 4, 10, 64), (2, 4, 10, 64)),
    "heads8": ((1, 8, 10, 64), (1, 8, 10, 64), (1, 8, 10, 64), (1, 8, 10, 64)),
    "nq2049": ((1, 4, 2049, 64), (1, 4, 10, 64), (1, 4, 10, 64), (1, 4, 2049, 64)),
    "nkv2049": ((1, 4, 10, 64), (1, 4, 2049, 64), (1, 4, 2049, 64), (1, 4, 10, 64)),
    "k_ne_v": ((1, 4, 10, 64), (1, 4, 11, 64), (1, 4, 10, 64), (1, 4, 10, 64)),
    "o_ne_q": ((1, 4, 10, 64), (1, 4, 10, 64), (1, 4, 10, 64), (1, 4, 11, 64)),
    "d128": ((1, 4, 10, 128), (1, 4, 10, 128), (1, 4, 10, 128), (1, 4, 10, 128)),
    "rank3": ((4, 10, 64), (1, 4, 10, 64), (1, 4, 10, 64), (1, 4, 10, 64)),
    "nkv0": ((1, 4, 10, 64), (1, 4, 0, 64), (1, 4, 0, 64), (1, 4, 10, 64)),
}


def test_configure_accepts_reference_shapes(plugin):
    _cfg(plugin, GOOD)
    _cfg(plugin, GOOD, types=(0, 0, 0, 0))
    _cfg(plugin, ((1, 4, 2048, 64),) * 4)
    _cfg(plugin, ((1, 4, 1, 64),) * 4)


@pytest.mark.parametrize("case", sorted(BAD))
def test_configure_rejects(plugin, case):
    from lightglue_amd import PluginError

    with pytest.raises(PluginError):
        _cfg(plugin, BAD[case])


def test_configure_rejects_mixed_types_and_formats(plugin):
    from lightglue_amd import PluginError

    with pytest.raises(PluginError):
        _cfg(plugin, GOOD, types=(1, 0, 1, 1))
    with pytest.raises(PluginError):
        _cfg(plugin, GOOD, types=(1, 1, 1, 0))
    with pytest.raises(PluginError):
        _cfg(plugin, GOOD, types=(2, 2, 2, 2))
    with pytest.raises(PluginError):
        _cfg(plugin, GOOD, fmts=(0, 0, 1, 0))


@pytest.mark.parametrize("case", sorted(BAD))
def test_enqueue_rejects_before_touching_the_device(plugin, case):
    """enqueue() validates exactly like configurePlugin and returns before any launch."""
    from lightglue_amd import PluginError

    s = BAD[case]
    with pytest.raises(PluginError):
        plugin.enqueue([desc(x) for x in s[:3]], [desc(s[3])], [16, 32, 48], [64], 128, 0)


def test_enqueue_rejects_null_workspace(plugin):
    from lightglue_amd import PluginError

    with pytest.raises(PluginError, match="workspace"):
        plugin.enqueue([desc(x) for x in GOOD[:3]], [desc(GOOD[3])], [16, 32, 48], [64], 0, 0)


def test_empty_query_is_a_noop(lib):
    # Nq == 0: nothing to launch, success without a device.
    assert lib.mha_hd64_launch_fp16in_fp16out(None, None, None, None, 1, 4, 0, 10, None, 0, None) == 0


def test_launch_rejects_misaligned_and_null(lib):
    assert lib.mha_hd64_launch_fp16in_fp16out(None, None, None, None, 1, 4, 8, 8, None, 0, None) == 1
    assert lib.mha_hd64_launch_fp16in_fp16out(16, 16, 16, 18, 1, 4, 8, 8, None, 0, None) == 1
    assert lib.mha_hd64_launch_fp16in_fp16out(16, 16, 16, 16, 1, 4, 8, 0, None, 0, None) == 1


def test_plan_fills_the_chip_and_fits_the_reference_workspace(lib):
    out = (ctypes.c_int32 * 4)()
    # metric shape 1x4x1024x1024 inside the fixed 5,242,880 B workspace
    # (16-row single-pass kernel, plan code 22: 256 workgroups of 16 rows x all 1024 keys, no
    # split, no workspace)
    need = lib.mha_hd64_plan(1, 4, 1024, 1024, 5242880, out)
    qw, kw, splits, tps = list(out)
    assert need == 0 and (qw, kw, splits) == (22, 4, 1)
    # 1024 < nkv <= 2048 on <= 256 16-row blocks: the 16-row kernel's two-pass form, no split
    need = lib.mha_hd64_plan(1, 4, 1024, 2048, 5242880, out)
    qw, kw, splits, tps = list(out)
    assert need == 0 and splits == 1 and qw == 22
    # max length still fits
    need = lib.mha_hd64_plan(1, 4, 2048, 2048, 5242880, out)
    assert need <= 5242880
    # no workspace -> no split
    lib.mha_hd64_plan(1, 4, 1024, 2048, 0, out)
    assert out[2] == 1
    # a big batch needs no split: past one round of 128-row blocks the persistent streaming
    # kernel (plan code 23) takes it (the default stream mode)
    lib.mha_hd64_plan(64, 4, 1024, 1024, 1 << 30, out)
    assert out[2] == 1 and out[0] == 23


@pytest.mark.parametrize("batch,nq,nkv,code", [
    (1, 1024, 1024, 22),     # the metric call: 256 blocks of 16 rows, 1024 keys
    (1, 2048, 1024, 21),     # 512 16-row blocks, 256 of 32 rows: the 32-row kernel
    (2, 2048, 1024, 21),     # 512 32-row blocks: two rounds of the 32-row kernel
    (6, 1024, 1024, 21),     # 768: three rounds
    (7, 1024, 1024, None),   # 896 32-row blocks: the LDS ring kernel
    (1, 1024, 1025, 22),     # more keys than 4 waves x 4 tiles: the 16-row kernel's two passes
    (1, 256, 2048, 22),      # two passes on 64 16-row blocks
    (1, 2048, 2048, 21),     # 512 16-row blocks: two passes on 256 32-row blocks
    (1, 2048, 1536, 21),
    (2, 2048, 2048, 21),     # 512 32-row blocks: 4 passes x 2 tiles, two workgroups per CU
    (4, 2048, 2048, None),   # 1024 of them: the LDS ring kernel
    (1, 1024, 2049, None),   # past 4 waves x 2 x 4 tiles
    (1, 256, 256, 22),
    (1, 1, 1, 22),
    (8, 1024, 1024, None),   # batched: 1024 blocks
    (2, 1024, 512, 21),
    (2, 512, 1000, 22),
])
def test_planner_single_pass_rule(lib, batch, nq, nkv, code):
    """Single-pass kernels iff fp16 and nkv <= 1024: plan code 22 (16-row blocks) when at most 256
    of them, else 21 (32-row blocks) when at most 768 of those; 1024 < nkv <= 2048 (two passes):
    22 on <= 256 16-row blocks, else 21 on 96..768 32-row blocks; they need no workspace and
    never split."""
    out = (ctypes.c_int32 * 4)()
    need = lib.mha_hd64_plan(batch, 4, nq, nkv, 5242880, out)
    if code is None:
        assert out[0] not in (21, 22)
    else:
        assert out[0] == code and need == 0 and out[2] == 1


def test_abort_mode_aborts_like_plugin_assert():
    """mha_hd64_set_abort_on_error(1) reproduces PLUGIN_ASSERT's abort() (checkMacrosPlugin.cpp:118-128)."""
    code = (
        "import sys; sys.path.insert(0, %r);"
        "from lightglue_amd import _lib; l=_lib.load(); l.mha_hd64_set_abort_on_error(1);"
        "l.mha_hd64_launch_fp16in_fp16out(None,None,None,None,1,4,8,8,None,0,None)" % os.path.join(
            REPO, "lightglue-with-flashattentionv2-tensorrt_amd"))
    r = subprocess.run(["python", "-c", code], capture_output=True, text=True)
    assert r.returncode != 0 and "assertion failed" in r.stderr


def test_error_message_names_the_assertion(lib):
    from lightglue_amd import _lib

    lib.mha_hd64_launch_fp16in_fp16out(None, None, None, None, 1, 4, 8, 8, None, 0, None)
    assert "assertion failed" in _lib.last_error()


def test_cpu_tensors_fail_loudly():
    import torch
    from lightglue_amd import PluginError, mha_hd64, mha_hd64_batched

    q = torch.zeros(1, 4, 8, 64, dtype=torch.float16)
    with pytest.raises(PluginError, match="GPU"):
        mha_hd64(q, q, q)
    with pytest.raises(PluginError, match="GPU"):
        mha_hd64_batched(q, q, q)


def test_typed_launch_workspace_query(lib):
    """mha_hd64_launch_workspace_bytes_typed: HALF equals the untyped query; FLOAT includes the
    fp16 copies exactly where the planner converts before a single-pass kernel (1x4x1024x2048:
    Q + K + V in fp16), nothing for the in-kernel one-pass form (1x4x1024^2) or the ring
    kernel's convert-on-load (4x4x1024^2, past one round of 32-row blocks); 0 for bad types."""
    HALF, FLOAT = 1, 0
    for shape in ((1, 4, 1024, 1024), (1, 4, 1024, 2048), (2, 4, 512, 512), (4, 4, 1024, 1024), (1, 4, 33, 65)):
        assert lib.mha_hd64_launch_workspace_bytes_typed(*shape, HALF) == lib.mha_hd64_launch_workspace_bytes(*shape)
    assert lib.mha_hd64_launch_workspace_bytes_typed(1, 4, 1024, 1024, FLOAT) == 0
    assert lib.mha_hd64_launch_workspace_bytes_typed(1, 4, 1024, 2048, FLOAT) == 4 * (1024 + 2 * 2048) * 64 * 2
    assert lib.mha_hd64_launch_workspace_bytes_typed(4, 4, 1024, 1024, FLOAT) == \
        lib.mha_hd64_launch_workspace_bytes(4, 4, 1024, 1024)
    assert lib.mha_hd64_launch_workspace_bytes_typed(1, 4, 1024, 1024, 7) == 0
    assert lib.mha_hd64_launch_workspace_bytes_typed(0, 4, 1024, 1024, FLOAT) == 0


def test_planner_invariants_fuzzed(lib):
    """Host-only property test of the planner (no GPU): for seeded random shapes (batch 1-64,
    heads 1-8, nq/nkv 1-4096) and workspace sizes, the plan code is one the launchers compile,
    the split count is 1..16 with tiles_per_split covering every key tile, the workspace the plan
    asks for fits the workspace given, and the typed queries are consistent (HALF = untyped,
    FLOAT >= 0, both 0 only for empty shapes)."""
    rng = np.random.default_rng(77)
    out = (ctypes.c_int32 * 4)()
    codes = {1, 2, 4, 12, 21, 22, 23}
    for _ in range(400):
        b, h = int(rng.integers(1, 65)), int(rng.integers(1, 9))
        nq, nkv = int(rng.integers(1, 4097)), int(rng.integers(1, 4097))
        ws = int(rng.choice([0, 1 << 16, 1 << 20, 5242880, 1 << 30]))
        need = lib.mha_hd64_plan(b, h, nq, nkv, ws, out)
        qw, kw, splits, tps = list(out)
        assert qw in codes, (b, h, nq, nkv, ws, qw)
        assert 1 <= splits <= 16 and tps >= 1, (b, h, nq, nkv, ws, splits, tps)
        if qw not in (21, 22, 23):
            super_tiles = -(-nkv // (64 * kw))
            assert splits * tps >= super_tiles, (b, h, nq, nkv, ws, kw, splits, tps)
        assert need <= ws or splits == 1, (b, h, nq, nkv, ws, need)
        half = lib.mha_hd64_launch_workspace_bytes_typed(b, h, nq, nkv, 1)
        assert half == lib.mha_hd64_launch_workspace_bytes(b, h, nq, nkv)
        assert lib.mha_hd64_launch_workspace_bytes_typed(b, h, nq, nkv, 0) >= 0


def _dma_checker():
    import importlib.util

    spec = importlib.util.spec_from_file_location("check_dma_hazards", os.path.join(REPO, "tools", "check_dma_hazards.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_dma_hazard_rules_on_synthetic_sequences():
    """tools/check_dma_hazards.py flags a VALU write of an LDS-DMA load's SGPR operand (soffset,
    descriptor, M0) fewer than 5 wait states before it and a SALU write of M0 right before it."""
    c = _dma_checker()

    def seq(*ins):
        return [("k", [(op, dst, src) for op, dst, src in ins])]

    load = ("buffer_load_dwordx4", "v1", " s[8:11], s4 offen lds")
    assert c.check(seq(("v_readfirstlane_b32", "s4", " v2"), ("s_nop", "0", ""), load)) == (1, 1)
    assert c.check(seq(("v_readfirstlane_b32", "s4", " v2"), ("s_nop", "4", ""), load)) == (1, 0)
    assert c.check(seq(("v_readfirstlane_b32", "s9", " v2"), ("s_add_i32", "s5", " s5, 1"), load)) == (1, 1)
    assert c.check(seq(("s_mov_b32", "m0", " s3"), load)) == (1, 1)
    assert c.check(seq(("s_mov_b32", "m0", " s3"), ("s_nop", "0", ""), load)) == (1, 0)
    assert c.check(seq(("v_readfirstlane_b32", "s3", " v2"), ("s_mov_b32", "m0", " s3"), ("s_nop", "0", ""), load)) == (1, 0)

    # branch targets: the walk stops at an instruction another block jumps to, and
    # counts it unless the load already has its 5 wait states after the target
    def seq_t(targets, *ins):
        return [("k", [(op, dst, src) for op, dst, src in ins], set(targets))]

    body = (("s_add_i32", "s6", " s6, 1"), ("s_nop", "0", ""), load)
    assert c.check(seq_t((), *body)) == (1, 0)  # straight line: fine
    assert c.check(seq_t((1,), *body)) == (1, 1)  # s_nop 0 is a jump target: 1 wait state only
    assert c.check(seq_t((0,), ("s_nop", "4", ""), load)) == (1, 0)  # padded after the target
    assert c.check(seq_t((2,), ("v_readfirstlane_b32", "s4", " v2"), ("s_nop", "4", ""), load)) == (1, 1)


def test_dma_hazard_parser_finds_branch_targets():
    """parse() maps an s_cbranch's `<func+0x..>` target to the instruction at that address."""
    c = _dma_checker()
    lines = [
        "0000000000001000 <k>:",
        "\ts_mov_b32 s4, 0  // 000000001000: BEEF0000",
        "\ts_cbranch_scc1 1  // 000000001004: BF850001 <k+0x10>",
        "\tv_readfirstlane_b32 s4, v2  // 00000000100C: 7E080502",
        "\ts_nop 0  // 000000001010: BF800000",
        "\tbuffer_load_dwordx4 v1, s[8:11], s4 offen lds  // 000000001014: E05D1000 02020001",
    ]
    funcs = c.parse(lines)
    assert funcs[0][0] == "k" and funcs[0][2] == {3}
    # the load sits 1 wait state after a jump target: flagged there (the walk stops at it)
    assert c.check(funcs) == (1, 1)
    # without the branch, the same code is flagged for the VALU write of s4 one wait state away
    assert c.check([(funcs[0][0], funcs[0][1], set())]) == (1, 1)
    assert c.check([(funcs[0][0], funcs[0][1][3:], set())]) == (1, 0)


def test_built_library_dma_wait_states():
    """Every LDS-DMA load of the built gfx950 code objects keeps the wait states (inline asm: the
    compiler's hazard recognizer does not see inside it)."""
    import shutil

    if not shutil.which("objcopy") or not os.path.exists(os.path.join("/opt/rocm", "lib", "llvm", "bin", "llvm-objdump")):
        pytest.skip("needs objcopy and the ROCm llvm-objdump")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "check_dma_hazards.py")], capture_output=True,
                       text=True, timeout=300)
    m = re.search(r"checked (\d+) LDS-DMA loads; (\d+) wait-state", r.stdout)
    assert r.returncode == 0 and m and int(m.group(1)) > 1000 and int(m.group(2)) == 0, r.stdout[-2000:]


def test_mfma_hazard_audit_flags_an_early_read():
    """tools/check_mfma_hazards.py: a VALU read of an MFMA destination needs the form's wait states
    (gfx950 16x16x32 f16: 4 passes, 7); MFMAs and s_nop count toward them; a read of other
    registers is not a hazard."""
    spec = importlib.util.spec_from_file_location("check_mfma_hazards", os.path.join(REPO, "tools", "check_mfma_hazards.py"))
    c = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(c)
    k = "kern"

    def seq(*body):
        return [(k, mn, ops, 4 * i) for i, (mn, ops) in enumerate(body)]

    mfma = ("v_mfma_f32_16x16x32_f16", "v[32:35], v[128:131], v[156:159], v[32:35]")
    assert len(c.audit(seq(mfma, ("v_mov_b32_e32", "v33, v32")), set())) == 1       # round 6's flush
    assert len(c.audit(seq(mfma, ("s_nop", "5"), ("v_mov_b32_e32", "v33, v32")), set())) == 1
    assert c.audit(seq(mfma, ("s_nop", "6"), ("v_mov_b32_e32", "v33, v32")), set()) == []
    assert c.audit(seq(mfma, ("v_mfma_f32_32x32x16_f16", "v[0:15], v[1:4], v[5:8], v[0:15]"),
                       ("v_mov_b32_e32", "v33, v32")), set()) == []
    assert c.audit(seq(mfma, ("v_mov_b32_e32", "v40, v41")), set()) == []


def test_built_library_mfma_result_wait_states():
    """No VALU instruction of the built gfx950 code objects reads or overwrites an MFMA result
    sooner than the form's wait states (inline asm on an accumulator gets none from the compiler:
    round 6's missed overflow in the streaming kernel's flush)."""
    import shutil

    if not shutil.which("objcopy") or not os.path.exists(os.path.join("/opt/rocm", "lib", "llvm", "bin", "llvm-objdump")):
        pytest.skip("needs objcopy and the ROCm llvm-objdump")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "check_mfma_hazards.py")], capture_output=True,
                       text=True, timeout=600)
    m = re.search(r"checked (\d+) VALU instructions; (\d+) MFMA-result", r.stdout)
    assert r.returncode == 0 and m and int(m.group(1)) > 100000 and int(m.group(2)) == 0, r.stdout[-3000:]


def test_ffn_and_form_hooks_validate_before_touching_the_device(lib):
    """lg_linear_cat_ffn (include/lightglue_glue.h) rejects bad arguments and returns success for an
    empty launch without a device call; the form hooks return the previous value and clamp."""
    A = 4096  # a fake 16-B aligned address: never dereferenced on these paths
    args = dict(x=A, c0=A, c1=A, heads=4, n0=8, n1=8, pairs=1, w1=A, b1=A, g=A, be=A, eps=1e-5, w2=A, b2=A, wp=A, h=A,
                out=2 * A)

    def call(**kw):
        a = {**args, **kw}
        return lib.lg_linear_cat_ffn(a["x"], a["c0"], a["c1"], a["heads"], a["n0"], a["n1"], a["pairs"], a["w1"], a["b1"],
                                     a["g"], a["be"], a["eps"], a["w2"], a["b2"], a["wp"], a["h"], a["out"], None)

    assert call(pairs=0) == 0 and call(pairs=0, wp=None) == 0  # nothing to launch
    for bad in (dict(x=None), dict(w2=None), dict(h=None), dict(out=A), dict(out=A + 4), dict(heads=0),
                dict(heads=3), dict(pairs=-1), dict(eps=-1.0), dict(x=A + 8), dict(wp=A + 8)):
        assert call(**{**bad, "pairs": 0 if "pairs" not in bad else bad["pairs"]}) == 1, bad
    # (two layouts: the 32-row kernel's, then the 16-row kernel's)
    assert lib.lg_ffn_packed_bytes(4, 0) == 2 * (512 * 512 + 256 * 512) * 2 and lib.lg_ffn_packed_bytes(3, 0) == 0
    assert lib.lg_ffn_packed_bytes(4, 768) == 2 * (512 * 512 + 256 * 512 + 768 * 256) * 2
    assert lib.lg_ffn_packed_bytes(4, 384) == 0
    for bad in ((A, A, None, 0, 3, A), (None, A, None, 0, 4, A), (A, A, None, 0, 4, None), (A, A + 4, None, 0, 4, A),
                (A, A, None, 512, 4, A), (A, A, A + 8, 768, 4, A), (A, A, A, 256, 4, A)):
        assert lib.lg_ffn_pack(*bad, None) == 1, bad
    # lg_linear_cat_ffn_proj: kind, the outputs its kind needs, n_store, alignment
    import ctypes
    outs = (ctypes.c_void_p * 6)(*([A] * 6))

    def proj(**kw):
        a = dict(x=A, c0=A, c1=A, heads=4, n0=8, n1=8, pairs=0, b1=A, g=A, be=A, eps=1e-5, b2=A, wp=A, kind=1, b3=A,
                 cs=A, sn=A, ns=0, outs=outs, out=2 * A)
        a.update(kw)
        return lib.lg_linear_cat_ffn_proj(a["x"], a["c0"], a["c1"], a["heads"], a["n0"], a["n1"], a["pairs"], a["b1"],
                                          a["g"], a["be"], a["eps"], a["b2"], a["wp"], a["kind"], a["b3"], a["cs"],
                                          a["sn"], a["ns"], a["outs"], a["out"], None)

    assert proj() == 0 and proj(kind=2) == 0 and proj(kind=3, ns=384) == 0
    for bad in (dict(kind=0), dict(kind=4), dict(heads=2), dict(wp=None), dict(out=A), dict(kind=2, cs=None),
                dict(kind=3, ns=0), dict(kind=3, ns=12), dict(kind=3, ns=520), dict(b3=None),
                dict(outs=(ctypes.c_void_p * 6)(A, A, A, None, A, A))):
        assert proj(**bad) == 1, bad
    prev = lib.lg_linear_set_wide(7)              # clamped to 5
    try:
        assert lib.lg_linear_set_wide(-5) == 5    # clamped to -1
        assert lib.lg_linear_set_wide(4) == -1
    finally:
        lib.lg_linear_set_wide(prev)
    prev = lib.lg_linear_set_ffn_fused(7)         # outside 0..3: 1
    try:
        assert lib.lg_linear_set_ffn_fused(0) == 1
        assert lib.lg_linear_set_ffn_fused(3) == 0
        assert lib.lg_linear_set_ffn_fused(2) == 3
        assert lib.lg_linear_set_ffn_fused(-1) == 2
        assert lib.lg_linear_set_ffn_fused(1) == 1
    finally:
        lib.lg_linear_set_ffn_fused(prev)


@pytest.mark.parametrize("version", [None, 1])
def test_stale_library_is_reported_as_missing(tmp_path, monkeypatch, version):
    """A library built from older sources (no lg_glue_abi_version, or an older ABI) raises
    LibraryMissing naming the rebuild, not an AttributeError from the binding loop."""
    if not shutil.which("gcc"):
        pytest.skip("needs gcc")
    from lightglue_amd import _lib

    src = tmp_path / "stale.c"
    body = "int mha_hd64_get_nb_outputs(void) { return 1; }\n"
    if version is not None:
        body += f"int lg_glue_abi_version(void) {{ return {version}; }}\n"
    src.write_text(body)
    so = tmp_path / "libstale.so"
    subprocess.run(["gcc", "-shared", "-fPIC", str(src), "-o", str(so)], check=True)
    monkeypatch.setattr(_lib, "LIB_PATH", str(so))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.LibraryMissing, match="stale"):
        _lib.load()

"""Parity of the persistent streaming kernel (csrc/mha_hd64_stream.hip; forced plan code 23 with
kv_waves 4 / 8 for its two forms, or mha_hd64_set_stream_mode(1) for the planner) with the C oracle.

The kernel walks items (call, batch*head, 128- or 256-row block) with every key of the call per item; a
workgroup takes a contiguous range of items and its K/V ring runs on across item seams, so the
cases below vary: items per workgroup (1 to 3; the grid is at most 512 workgroups), calls of
different nkv in one launch (the MULTI form), partial last key tiles, one-tile items (nkv <= 64),
a running-max move inside an item and at its first tile, and NaN inputs. Tolerances as
test_gpu_parity.py (north_star: max-abs <= 1e-2; fp32 output 5e-3)."""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL = 1e-2
TOL_F32OUT = 5e-3
STREAM = 23


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from lightglue_amd import _lib

    _lib.load()
    return torch.device("cuda:0")


@pytest.fixture
def stream_mode(dev):
    import lightglue_amd

    prev = lightglue_amd.set_stream_mode(1)
    lightglue_amd.set_stream_mode(prev)
    yield lightglue_amd.set_stream_mode
    lightglue_amd.set_stream_mode(prev)


def _t(x, dev, dtype):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev).to(dtype).contiguous()


def _maxdiff(a, b):
    return float(np.abs(a.astype(np.float64) - b.astype(np.float64)).max())


def _launch(lib, q, k, v, o, code=STREAM, ws=None, waves=0):
    from lightglue_amd import _lib

    b, h, nq, _ = q.shape
    nkv = k.shape[2]
    ws = ws if ws is not None else torch.empty(1 << 20, dtype=torch.uint8, device=q.device)
    st = lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), b, h, nq, nkv,
                                    int(q.dtype == torch.float32), int(o.dtype == torch.float32), code, waves, 0,
                                    ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream, 3)
    assert st == 0, _lib.last_error()


def _rows(nq, n=40):
    return np.unique(np.r_[np.arange(0, nq, max(1, nq // n)), nq - 1])


def _oracle_rows(oracle_mod, q16, k16, v16, rows):
    return oracle_mod.attention_c(np.ascontiguousarray(q16[:, :, rows]), k16, v16)


# (batch, nq, nkv): one-tile items, partial tiles, items per workgroup 1..3, ragged last blocks
STREAM_SHAPES = [(1, 1, 1), (1, 100, 77), (1, 33, 65), (1, 129, 1), (1, 1000, 3), (5, 257, 63), (2, 300, 1000),
                 (3, 1000, 777), (1, 64, 2048), (1, 1024, 1024), (16, 1024, 1024), (40, 128, 128), (2, 2048, 2048),
                 (24, 1024, 1100), (36, 1000, 129)]


@pytest.mark.parametrize("waves", [4, 8])
@pytest.mark.parametrize("batch,nq,nkv", STREAM_SHAPES)
def test_stream_kernel_matches_oracle(batch, nq, nkv, waves, dev, oracle_mod):
    from lightglue_amd import _lib, synth

    lib = _lib.load()
    qn, kn, vn = synth.qkv(2300 + 7 * batch + nq + 3 * nkv, nq, nkv, batch=batch)
    q16, k16, v16 = (synth.round_f16(x) for x in (qn, kn, vn))
    rows = _rows(nq)
    bsel = sorted({0, batch // 2, batch - 1})
    ref = _oracle_rows(oracle_mod, q16[bsel], k16[bsel], v16[bsel], rows)
    q, k, v = (_t(x, dev, torch.float16) for x in (q16, k16, v16))
    for out_dt, tol in ((torch.float16, TOL), (torch.float32, TOL_F32OUT)):
        o = torch.full(q.shape, float("nan"), dtype=out_dt, device=dev)
        _launch(lib, q, k, v, o, waves=waves)
        torch.cuda.synchronize()
        got = o.float().cpu().numpy()
        assert np.isfinite(got).all(), "unwritten or NaN output rows"
        d = _maxdiff(got[bsel][:, :, rows], ref)
        assert d <= tol, (batch, nq, nkv, waves, out_dt, d)


@pytest.mark.parametrize("waves", [4, 8])
def test_stream_kernel_running_max_moves(waves, dev, oracle_mod):
    """A spike key moves a query's running max at the item's first tile (key 10), in a middle tile
    past the lazy-rescale threshold (key 300, gain 6), barely (gain 0.5: no rescale), and in the
    partial last tile (nkv 1100, key 1090); batch 40 gives every workgroup 2-3 items, so the
    moves land at item seams of the continuous K/V ring too."""
    from lightglue_amd import _lib, synth

    lib = _lib.load()
    batch, nq = 40, 512
    for nkv, krow, gain in ((1024, 10, 6.0), (1024, 300, 6.0), (1024, 700, 0.5), (1100, 1090, 6.0), (2048, 1900, 3.0)):
        qn, kn, vn = synth.qkv(909 + nkv + krow, nq, nkv, batch=batch)
        kn = synth.spike(qn, kn, 5, krow, gain)
        kn = synth.spike(qn, kn, 300, (krow * 7 + 64) % nkv, gain)
        q16, k16, v16 = (synth.round_f16(x) for x in (qn, kn, vn))
        rows = np.unique(np.r_[_rows(nq, 24), 5, 300])
        bsel = [0, 17, batch - 1]
        ref = _oracle_rows(oracle_mod, q16[bsel], k16[bsel], v16[bsel], rows)
        q, k, v = (_t(x, dev, torch.float16) for x in (q16, k16, v16))
        for out_dt, tol in ((torch.float16, TOL), (torch.float32, TOL_F32OUT)):
            o = torch.full(q.shape, float("nan"), dtype=out_dt, device=dev)
            _launch(lib, q, k, v, o, waves=waves)
            torch.cuda.synchronize()
            got = o.float().cpu().numpy()
            assert np.isfinite(got).all()
            d = _maxdiff(got[bsel][:, :, rows], ref)
            assert d <= tol, (nkv, krow, gain, waves, out_dt, d)


@pytest.mark.parametrize("waves", [4, 8])
@pytest.mark.parametrize("nkv", [200, 1100, 2048])
def test_stream_kernel_every_item_recomputed(nkv, waves, dev, oracle_mod):
    """The speculative running max's rare path on every item: each 128-row block of every head has
    one query row whose spike key (gain 8, past tile 0) beats tile 0's max by far more than 2^16, so
    every item's row sum overflows, every item is marked and every wave re-runs its rows of all of
    them through its own ring slot after the workgroup's last barrier (csrc/mha_hd64_stream.hip,
    exact_item). nkv 200 and 1100: a partial last tile; batch 40: 2-3 items per workgroup,
    so the re-runs follow each other through the same slot. Every row of three heads is checked.
    Both output types take the 1e-2 contract: on these peaked rows fp16 P's rounding alone puts the
    fp32 output 6.1e-3 from the fp64 oracle, in the lazy-rescale form (no rare path) as in this one
    (profiles/r06/stream_rare_path_errors.jsonl, tools/rare_path_errors.py)."""
    from lightglue_amd import _lib, synth

    lib = _lib.load()
    batch, nq = 40, 512
    qn, kn, vn = synth.qkv(4242 + nkv, nq, nkv, batch=batch)
    for blk in range(nq // 128):
        kn = synth.spike(qn, kn, 128 * blk + 9 + 11 * blk, 64 + 37 * blk, 8.0)
    q16, k16, v16 = (synth.round_f16(x) for x in (qn, kn, vn))
    bsel = [0, 23, batch - 1]
    ref = oracle_mod.attention_c(q16[bsel], k16[bsel], v16[bsel])
    q, k, v = (_t(x, dev, torch.float16) for x in (q16, k16, v16))
    for out_dt in (torch.float16, torch.float32):
        o = torch.full(q.shape, float("nan"), dtype=out_dt, device=dev)
        _launch(lib, q, k, v, o, waves=waves)
        torch.cuda.synchronize()
        got = o.float().cpu().numpy()
        assert np.isfinite(got).all()
        d = _maxdiff(got[bsel], ref)
        assert d <= TOL, (nkv, waves, out_dt, d)


@pytest.mark.parametrize("waves", [4, 8])
def test_stream_kernel_matcher_overflow_head(waves, dev, oracle_mod):
    """A head of the seeded fp16 matcher (P = 8 pairs, n = 1024; the layer-7 self-attention launch,
    tools/matcher_nan_probe.py) whose rows 131, 361 and 816 beat their tile-0 max by just past 2^16:
    the speculative max overflows there and, through the row-sum MFMA, in the partner rows 147, 377
    and 800. The overflow of an item whose epilogue is the flush's (the workgroup's last item) was
    missed until round 6: the check read the row sums with an inline-asm move that the compiler gave
    no MFMA wait states. Every row against the fp64 oracle (tests/golden/stream_spec_overflow_head.npz)."""
    import os

    from conftest import REPO
    from lightglue_amd import _lib

    lib = _lib.load()
    d = np.load(os.path.join(REPO, "tests", "golden", "stream_spec_overflow_head.npz"))
    q16, k16, v16 = (d[n].astype(np.float32) for n in "qkv")
    ref = oracle_mod.attention_c(q16, k16, v16)
    q, k, v = (_t(x, dev, torch.float16) for x in (q16, k16, v16))
    for out_dt, tol in ((torch.float16, TOL), (torch.float32, TOL_F32OUT)):
        o = torch.full(q.shape, float("nan"), dtype=out_dt, device=dev)
        _launch(lib, q, k, v, o, waves=waves)
        torch.cuda.synchronize()
        got = o.float().cpu().numpy()
        assert np.isfinite(got).all(), np.nonzero(~np.isfinite(got).all(-1))
        d_ = _maxdiff(got, ref)
        assert d_ <= tol, (waves, out_dt, d_)


@pytest.mark.parametrize("waves", [4, 8])
def test_stream_kernel_large_negative_logits(waves, dev, oracle_mod):
    """Scores far below zero everywhere (~ -200 raw, as test_gpu_parity.py's case) in a launch of
    several items per workgroup: each item's first tile must set its max (no underflow to l = 0).
    At this logit scale the fp16 operands of Q·Kᵀ alone put every plan ~6e-3 from the fp64 oracle
    (tools/extreme_logits.py: identical errors across plans 0/1/21/22/23), so both output types
    take the 1e-2 contract here, and the stream kernel must agree with the planner's plan."""
    from lightglue_amd import _lib, synth

    lib = _lib.load()
    nq, nkv, batch = 256, 700, 40
    qn, kn, vn = synth.qkv(808, nq, nkv, batch=batch)
    qn = np.abs(qn) * 4
    kn = -np.abs(kn) * 4
    q16, k16, v16 = (synth.round_f16(x) for x in (qn, kn, vn))
    bsel = [0, 21, batch - 1]
    ref = oracle_mod.attention_c(q16[bsel], k16[bsel], v16[bsel])
    q, k, v = (_t(x, dev, torch.float16) for x in (q16, k16, v16))
    for out_dt in (torch.float16, torch.float32):
        o = torch.empty(q.shape, dtype=out_dt, device=dev)
        _launch(lib, q, k, v, o, waves=waves)
        o2 = torch.empty(q.shape, dtype=out_dt, device=dev)
        _launch(lib, q, k, v, o2, code=0)
        torch.cuda.synchronize()
        got = o.float().cpu().numpy()
        assert np.isfinite(got).all()
        d = _maxdiff(got[bsel], ref)
        dp = _maxdiff(got, o2.float().cpu().numpy())
        assert d <= TOL and dp <= 2e-3, (out_dt, d, dp)


@pytest.mark.parametrize("out_dt,tol", [(torch.float16, TOL), (torch.float32, TOL_F32OUT)])
def test_stream_mode_grouped_calls(out_dt, tol, dev, oracle_mod, stream_mode):
    """set_stream_mode(1): a grouped launch of calls with different nq/nkv (the kernel's MULTI
    form: per-call bases and key counts selected per item) and a batched call go through the
    streaming kernel; both match the oracle and the planner's default plan within the contract."""
    from lightglue_amd import _lib, mha_hd64_batched, mha_hd64_grouped, synth

    lib = _lib.load()
    shapes = [(12, 1024, 1024), (6, 512, 700), (3, 1000, 77), (9, 200, 1500)]
    host = []
    for i, (b, nq, nkv) in enumerate(shapes):
        qn, kn, vn = synth.qkv(5150 + 13 * i, nq, nkv, batch=b)
        host.append(tuple(synth.round_f16(x) for x in (qn, kn, vn)))
    dev_t = [tuple(_t(x, dev, torch.float16) for x in c) for c in host]
    stream_mode(0)
    base = mha_hd64_grouped(dev_t, out_dtype=out_dt)
    stream_mode(1)
    plan = (ctypes.c_int32 * 4)()
    lib.mha_hd64_plan(16, 4, 1024, 1024, 5242880, plan)
    assert plan[0] == STREAM
    outs = mha_hd64_grouped(dev_t, out_dtype=out_dt)
    torch.cuda.synchronize()
    for (q16, k16, v16), o, ob in zip(host, outs, base):
        rows = _rows(q16.shape[2], 24)
        b = q16.shape[0]
        bsel = sorted({0, b - 1})
        ref = _oracle_rows(oracle_mod, q16[bsel], k16[bsel], v16[bsel], rows)
        got = o.float().cpu().numpy()
        assert np.isfinite(got).all()
        d, db = _maxdiff(got[bsel][:, :, rows], ref), _maxdiff(got, ob.float().cpu().numpy())
        assert d <= tol and db <= tol, (q16.shape, d, db)
    (q, k, v) = dev_t[0]
    a = mha_hd64_batched(q, k, v, out_dtype=out_dt)
    torch.cuda.synchronize()
    assert torch.equal(a, outs[0])  # one call alone: same items, same bits


@pytest.mark.parametrize("waves", [4, 8])
def test_stream_kernel_deterministic_and_capturable(waves, dev):
    from lightglue_amd import _lib, synth

    lib = _lib.load()
    qn, kn, vn = synth.qkv(99, 1024, 1024, batch=16)
    q, k, v = (_t(x, dev, torch.float16) for x in (qn, kn, vn))
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    a = torch.empty_like(q)
    b = torch.empty_like(q)
    _launch(lib, q, k, v, a, ws=ws, waves=waves)
    _launch(lib, q, k, v, b, ws=ws, waves=waves)
    out = torch.empty_like(q)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        _launch(lib, q, k, v, out, ws=ws, waves=waves)
        with torch.cuda.graph(g, stream=s):
            _launch(lib, q, k, v, out, ws=ws, waves=waves)
    torch.cuda.current_stream().wait_stream(s)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(out, a)


@pytest.mark.parametrize("waves", [4, 8])
@pytest.mark.parametrize("where", ["q", "k", "v"])
def test_stream_kernel_nan_inputs(where, waves, dev):
    """NaNs reach the outputs the reference's PyTorch math gives them (a NaN query row -> that
    row; a NaN key row -> every row of the head; a NaN value element -> its column)."""
    from lightglue_amd import _lib, synth

    lib = _lib.load()
    n = 1024
    qn, kn, vn = synth.qkv(4711 + n, n, n, batch=2)
    x = {"q": qn, "k": kn, "v": vn}[where]
    x[1, 1, n // 3, 5] = np.nan
    q16, k16, v16 = (synth.round_f16(a) for a in (qn, kn, vn))
    qf, kf, vf = (torch.from_numpy(a) for a in (q16, k16, v16))
    ref = torch.softmax((qf @ kf.transpose(-1, -2)) * 0.125, -1) @ vf
    q, k, v = (_t(a, dev, torch.float16) for a in (q16, k16, v16))
    for out_dt in (torch.float16, torch.float32):
        o = torch.empty(q.shape, dtype=out_dt, device=dev)
        _launch(lib, q, k, v, o, waves=waves)
        torch.cuda.synchronize()
        assert torch.equal(torch.isnan(o.float().cpu()), torch.isnan(ref)), (where, waves, out_dt)


def test_stream_plan_reported_and_fp32_inputs_fall_back(dev, stream_mode):
    """The plan query names code 23 for large fp16 launches under stream mode 1 and never below one
    round of 128-row blocks; fp32 inputs forced to 23 are rejected and under stream mode 1 keep the
    planner's other plans (bitwise the stream-mode-0 result)."""
    from lightglue_amd import _lib, mha_hd64_batched, synth

    lib = _lib.load()
    plan = (ctypes.c_int32 * 4)()
    stream_mode(1)
    lib.mha_hd64_plan(1, 4, 1024, 1024, 5242880, plan)
    assert plan[0] != STREAM  # 32 items: the single-pass kernel
    lib.mha_hd64_plan(16, 4, 1024, 1024, 5242880, plan)
    assert plan[0] == STREAM and plan[1] == 8  # 256 items of 256 rows: the 8-wave form
    lib.mha_hd64_plan(12, 4, 1024, 1024, 5242880, plan)
    assert plan[0] == STREAM and plan[1] == 8  # 192 of them: one round, 3/4 full
    lib.mha_hd64_plan(24, 4, 1024, 1024, 5242880, plan)
    assert plan[0] == STREAM and plan[1] == 4  # 384: a half-full second round -> 768 items of 128 rows
    stream_mode(0)
    lib.mha_hd64_plan(16, 4, 1024, 1024, 5242880, plan)
    assert plan[0] != STREAM
    qn, kn, vn = synth.qkv(5, 300, 500, batch=2)
    q, k, v = (_t(x, dev, torch.float32) for x in (qn, kn, vn))
    o = torch.empty(q.shape, dtype=torch.float32, device=dev)
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    st = lib.mha_hd64_launch_forced(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), 2, 4, 300, 500, 1, 1,
                                    STREAM, 0, 0, ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream, 3)
    assert st == 1  # BAD_PARAM: the streaming kernel takes fp16 inputs only
    stream_mode(1)
    a = mha_hd64_batched(q.repeat(8, 1, 1, 1), k.repeat(8, 1, 1, 1), v.repeat(8, 1, 1, 1), out_dtype=torch.float32)
    stream_mode(0)
    b = mha_hd64_batched(q.repeat(8, 1, 1, 1), k.repeat(8, 1, 1, 1), v.repeat(8, 1, 1, 1), out_dtype=torch.float32)
    torch.cuda.synchronize()
    assert torch.equal(a, b)  # fp32 inputs never take the streaming kernel


def test_stream_mode_grouped_with_one_tile_calls(dev, oracle_mod, stream_mode):
    """Grouped MULTI launch mixing long items with one-tile items (nkv <= 64: the next item's Q
    is fetched and waited for inside the seam step) and a one-key call, both output types."""
    from lightglue_amd import _lib, mha_hd64_grouped, synth

    lib = _lib.load()
    stream_mode(1)
    shapes = [(12, 1024, 1024), (8, 300, 50), (6, 128, 1), (10, 640, 64)]
    host = []
    for i, (b, nq, nkv) in enumerate(shapes):
        qn, kn, vn = synth.qkv(6200 + 11 * i, nq, nkv, batch=b)
        host.append(tuple(synth.round_f16(x) for x in (qn, kn, vn)))
    dev_t = [tuple(_t(x, dev, torch.float16) for x in c) for c in host]
    plan = (ctypes.c_int32 * 4)()
    lib.mha_hd64_plan(12, 4, 1024, 1024, 5242880, plan)
    assert plan[0] == STREAM
    for out_dt, tol in ((torch.float16, TOL), (torch.float32, TOL_F32OUT)):
        outs = [torch.full(q.shape, float("nan"), dtype=out_dt, device=dev) for q, _, _ in dev_t]
        mha_hd64_grouped(dev_t, out_dtype=out_dt, outs=outs)
        torch.cuda.synchronize()
        for (q16, k16, v16), o in zip(host, outs):
            got = o.float().cpu().numpy()
            assert np.isfinite(got).all()
            rows = _rows(q16.shape[2], 24)
            bsel = sorted({0, q16.shape[0] - 1})
            ref = _oracle_rows(oracle_mod, q16[bsel], k16[bsel], v16[bsel], rows)
            d = _maxdiff(got[bsel][:, :, rows], ref)
            assert d <= tol, (q16.shape, k16.shape, out_dt, d)


@pytest.mark.parametrize("waves,batch", [(8, 32), (8, 12), (4, 24), (4, 32)])
def test_stream_kernel_bitwise_repeatable(waves, batch, dev):
    """Ten launches of one forced form give identical bits (the K/V ring's barrier schedule leaves
    no read of a slot racing a refill: a race shows up as launch-to-launch differences)."""
    from lightglue_amd import _lib, synth

    lib = _lib.load()
    qn, kn, vn = synth.qkv(5150, 1024, 1024, batch=batch)
    q, k, v = (_t(x, dev, torch.float16) for x in (qn, kn, vn))
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    first = torch.empty_like(q)
    _launch(lib, q, k, v, first, ws=ws, waves=waves)
    o = torch.empty_like(q)
    for _ in range(9):
        _launch(lib, q, k, v, o, ws=ws, waves=waves)
        torch.cuda.synchronize()
        assert torch.equal(o, first)


# ---- the reference's golden fixtures through plan 23 ----
from conftest import golden_cases, load_golden  # noqa: E402


def _fixture_batch(nq, waves):
    """Copies of a fixture stacked in the batch so that every workgroup of the forced form walks at
    least two items (grid = min(items, 512 / 256 workgroups for 4 / 8 waves))."""
    items = 4 * -(-nq // (32 * waves))
    cap = 512 if waves == 4 else 256
    return -(-(2 * cap + cap // 4) // items)


@pytest.mark.parametrize("waves", [4, 8])
@pytest.mark.parametrize("name", golden_cases())
def test_stream_kernel_matches_reference_fixtures(name, waves, dev):
    """Every golden fixture (outputs of the reference's PyTorch Attention) through the streaming
    kernel, both forms, both output types, under the single-call kernels' regression guards
    (test_gpu_parity.py: fp16 out |d| <= 1.5e-3 s + 2^-11 |ref|, fp32 out 1.5e-3 s); the fixture is
    copied B times into the batch so items sit at every seam position of the K/V ring, and every
    copy must give the same bits (an item's result may not depend on its neighbours)."""
    from test_gpu_parity import REG_F32OUT, _regress16, _scale

    from lightglue_amd import _lib

    lib = _lib.load()
    g = load_golden(name)
    nq = g["q"].shape[2]
    B = _fixture_batch(nq, waves)
    q16, k16, v16 = (np.ascontiguousarray(np.repeat(g[x], B, axis=0)) for x in ("q", "k", "v"))
    q, k, v = (_t(x, dev, torch.float16) for x in (q16, k16, v16))
    for out_dt in (torch.float16, torch.float32):
        o = torch.full(q.shape, float("nan"), dtype=out_dt, device=dev)
        _launch(lib, q, k, v, o, waves=waves)
        torch.cuda.synchronize()
        assert torch.equal(o, o[:1].expand_as(o)), "batch copies of one fixture differ"
        got = o[:1].float().cpu().numpy()[:, :, g["rows"]]
        assert np.isfinite(got).all()
        if out_dt == torch.float16:
            _regress16(got, g["o_ref16"], _scale(g))
        else:
            assert _maxdiff(got, g["o_ref16"]) <= REG_F32OUT * _scale(g)

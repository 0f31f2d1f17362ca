"""torch.library operators (lightglue_amd/ops.py): registration, CPU refusal, fake shapes (CPU),
and equality with the direct enqueue / grouped launcher (GPU)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")


def test_ops_registered_and_cpu_refused():
    import lightglue_amd  # noqa: F401  (registers the ops)

    q = torch.randn(1, 4, 8, 64)
    with pytest.raises(NotImplementedError):
        torch.ops.lightglue_amd.mha_hd64(q, q, q)
    with pytest.raises(NotImplementedError):
        torch.ops.lightglue_amd.mha_hd64_grouped([q], [q], [q])


def test_ops_fake_shapes():
    import lightglue_amd  # noqa: F401

    with torch.device("meta"):
        q = torch.empty(1, 4, 37, 64, dtype=torch.float16)
        k = torch.empty(1, 4, 50, 64, dtype=torch.float16)
    o = torch.ops.lightglue_amd.mha_hd64(q, k, k)
    assert o.shape == q.shape and o.dtype == torch.float16
    outs = torch.ops.lightglue_amd.mha_hd64_grouped([q, k], [k, q], [k, q])
    assert [t.shape for t in outs] == [q.shape, k.shape]


@pytest.mark.gpu
def test_ops_match_direct_calls():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from lightglue_amd import mha_hd64, mha_hd64_grouped, synth

    dev = torch.device("cuda:0")
    qn, kn, vn = synth.qkv(17, 300, 211)
    q, k, v = (torch.from_numpy(np.ascontiguousarray(x)).to(dev).half() for x in (qn, kn, vn))
    a = torch.ops.lightglue_amd.mha_hd64(q, k, v)
    b = mha_hd64(q, k, v)
    (c, d) = torch.ops.lightglue_amd.mha_hd64_grouped([q, k], [k, q], [v, q])
    (e, f) = mha_hd64_grouped([(q, k, v), (k, q, q)])
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(c, e) and torch.equal(d, f)

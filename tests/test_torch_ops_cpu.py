"""The ste:: custom-op layer (torch_ops.py) without a GPU: every op is registered
with its schema, and its fake (meta) implementation propagates shapes and dtypes, so the ops
trace under FakeTensorMode / torch.compile.  The kernels themselves run in
tests/test_torch_ops_gpu.py."""
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

import speech_transcript_embeddings_amd  # noqa: F401  (registers torch.ops.ste.*)
from speech_transcript_embeddings_amd import torch_ops


def test_ops_registered_with_schemas():
    for name in torch_ops.OPS:
        op = getattr(torch.ops.ste, name).default
        assert op._schema.name == f"ste::{name}"
    s = str(torch.ops.ste.adamw_.default._schema)
    assert "Tensor(a0!) p" in s and "Tensor(a2!) m" in s and "Tensor(a3!) v" in s  # in-place state
    assert "Tensor? rel_E" in str(torch.ops.ste.attention.default._schema)


def test_fake_implementations_propagate_shapes():
    with FakeTensorMode():
        f, m = torch.ops.ste.fbank(torch.empty(3, 160000), torch.empty(3, dtype=torch.int32), 499)
        assert f.shape == (3, 499, 160) and f.dtype == torch.float32 and m.shape == (3, 499) and m.dtype == torch.int64
        y = torch.ops.ste.linear(torch.empty(2, 5, 64), torch.empty(32, 64), torch.empty(32))
        assert y.shape == (2, 5, 32) and y.dtype == torch.float32
        y, mu, rs = torch.ops.ste.layer_norm(torch.empty(4, 7, 96), torch.empty(96), torch.empty(96), 1e-5)
        assert y.shape == (4, 7, 96) and mu.shape == (28,) and rs.shape == (28,)
        q = torch.empty(2, 99, 128, dtype=torch.bfloat16)
        o, lse, olo = torch.ops.ste.attention(q, q, q, None, torch.empty(73, 64), 0.125, 64, 8)
        assert o.shape == q.shape and o.dtype == torch.bfloat16 and lse.shape == (2 * 2 * 99,) and olo.shape == q.shape
        loss = torch.ops.ste.pair_loss(torch.empty(8), torch.empty(8), None, 0.1, 0.5, 0.35)
        assert loss.shape == () and loss.dtype == torch.float32

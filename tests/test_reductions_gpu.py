"""The ordered (run-to-run deterministic) reductions one by one, each run twice on ragged shapes
while a second stream keeps our own GEMMs busy on the same CUs, so co-residency and timing differ
between the runs: results must be bit-identical and match an fp64 torch reference (DESIGN §4
"Determinism"; the whole training step is tests/test_determinism_gpu.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    from speech_transcript_embeddings_amd import ops as _ops
    assert not _ops.ATOMIC_SUMS
    return _ops


@pytest.fixture(scope="module")
def busy(ops):
    """Queue 30 GEMMs on a side stream (returns a function)."""
    s = torch.cuda.Stream()
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(2048, 768, device=DEV, generator=g).bfloat16()
    w = (torch.randn(3072, 768, device=DEV, generator=g) * 0.02).bfloat16()

    def run():
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(30):
                ops.linear(x, w, out_bf16=True)
    yield run
    torch.cuda.synchronize()


def _twice(fn, busy):
    outs = []
    for _ in range(2):
        busy()
        outs.append([t.clone() for t in fn()])
        torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    return outs[0]


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


@pytest.mark.parametrize("M,N,K", [(1000, 520, 256),      # 128x128 kernel, ragged tiles
                                   (8000, 4096, 1024)])   # 8-phase kernel (512 tiles)
def test_gemm_bias_gradient_columns(ops, busy, M, N, K):
    """GEMM epilogue column sums (a Linear's bias gradient) through per-wave partial rows and
    ste_rowsum_ordered."""
    torch.manual_seed(M)
    a = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()

    def fn():
        out = torch.empty(M, N, device=DEV)
        cs = torch.zeros(N, device=DEV)
        ops.linear(a, w, out=out, colsum=cs)
        return out, cs
    out, cs = _twice(fn, busy)
    assert _rel(cs, out.double().sum(0)) < 1e-5


@pytest.mark.parametrize("rows,cols,bf16", [(4999, 1000, True), (31936, 1024, False), (77, 3072, True)])
def test_colsum(ops, busy, rows, cols, bf16):
    torch.manual_seed(rows)
    x = torch.randn(rows, cols, device=DEV)
    if bf16:
        x = x.bfloat16()
    out = _twice(lambda: [ops.colsum(x, torch.zeros(cols, device=DEV))], busy)[0]
    assert _rel(out, x.double().sum(0)) < 1e-6


def test_sumsq(ops, busy):
    torch.manual_seed(3)
    g = torch.randn(10_000_123, device=DEV) * 1e-3
    part = torch.empty(ops.SUMSQ_PARTS, device=DEV, dtype=torch.float64)

    def fn():
        acc = torch.zeros(1, device=DEV, dtype=torch.float64)
        ops.sumsq(g, acc, part)
        return [acc]
    acc = _twice(fn, busy)[0]
    ref = (g.double() ** 2).sum()
    # fp32 squares (2^-24 relative each) summed in fp64: measured 9e-11
    assert abs(float(acc[0]) - float(ref)) / float(ref) < 1e-7


def test_text_embedding_rows(ops, busy):
    """Word / position table gradients with heavily repeated ids: one writer per row, the row's
    tokens summed in token order."""
    torch.manual_seed(6)
    B, L, D, V, pad = 64, 64, 768, 50, 1
    ids = torch.randint(5, V, (B, L), device=DEV)
    ids[:, 50:] = pad
    pid = torch.empty(B * L, dtype=torch.int32, device=DEV)
    ops.text_embed_fwd(ids, pad, torch.randn(V, D, device=DEV), torch.randn(514, D, device=DEV),
                       torch.randn(1, D, device=DEV), torch.empty(B * L, D, device=DEV), pid)
    do = torch.randn(B * L, D, device=DEV)

    def fn():
        dw, dp, dt = torch.zeros(V, D, device=DEV), torch.zeros(514, D, device=DEV), torch.zeros(1, D, device=DEV)
        ops.text_embed_bwd(ids, pid, do, pad, dw, dp, dt)
        return dw, dp, dt
    dw, dp, dt = _twice(fn, busy)
    ref_w = torch.zeros(V, D, device=DEV, dtype=torch.float64).index_add_(0, ids.reshape(-1), do.double())
    ref_w[pad] = 0
    assert _rel(dw, ref_w) < 1e-6
    assert _rel(dt[0], do.double().sum(0)) < 1e-6


def test_glu_dwconv_weight_gradient(ops, busy):
    torch.manual_seed(9)
    B, T, C, K = 8, 499, 1024, 31
    pre = torch.randn(B * T, 2 * C, device=DEV).bfloat16()
    w = torch.randn(C, K, device=DEV) * 0.1
    dcv = torch.randn(B * T, C, device=DEV).bfloat16()

    def fn():
        dpre = torch.empty(B * T, 2 * C, device=DEV, dtype=torch.bfloat16)
        dw = torch.zeros(C, K, device=DEV)
        ops.glu_dwconv_bwd(pre, w, dcv, dpre, dw, B, T)
        return dpre, dw
    _twice(fn, busy)

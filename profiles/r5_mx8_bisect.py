"""Which tree's persistent 8-phase MX-fp8 GEMM is right?  python profiles/r5_mx8_bisect.py ROOT:
imports speech_transcript_embeddings_amd from ROOT (the current tree or an old one extracted by
git archive) and compares the MX GEMM at 252 tiles (8-phase plan) and 128 tiles (single-stage)
with the dequantised operands' fp64 product, for the QKV epilogue (bias, bf16 out)."""
import json
import sys

root = sys.argv[1]
sys.path.insert(0, root)
import torch  # noqa: E402
from speech_transcript_embeddings_amd import ops  # noqa: E402


def deq(q, sc):
    v = q.view(torch.float8_e4m3fn).double()
    e = sc.long().repeat_interleave(32, dim=1) - 127
    return v * torch.pow(2.0, e.double())


res = {"root": root, "lib": str(getattr(ops._lib, "LIB_PATH", "?"))}
for M in (8000, 16000, 95936):
    torch.manual_seed(10)
    N, K = 1024, 1024
    x = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.03).bfloat16()
    bias = torch.randn(N, device="cuda")
    xq, wq = ops.mx8_quant(x), ops.mx8_quant(w)
    ref = deq(*xq) @ deq(*wq).T + bias.double()
    y = ops.linear_mx8(xq, wq, bias, out_bf16=True)
    err = ((y.double() - ref).norm() / ref.norm()).item()
    rows_bad = int(((y.double() - ref).abs().amax(1) > 0.1 * ref.abs().amax()).sum())
    res[f"M{M}"] = {"rel_err": err, "bad_rows": rows_bad}
    del x, xq, y, ref
    torch.cuda.synchronize()
print(json.dumps(res))

"""GEMM-run LayerNorm (EF_LNF) vs the residual GEMM + separate LayerNorm launch, isolated at c2 rows.
Round-6 experiment, not in the tree: apply profiles/r6_lnf.patch (ops.linear_ln, gemm.hip EF_LNF) first.

    python profiles/lnf_probe.py [--iters 20]
Per shape: the residual GEMM alone, the LayerNorm alone, and the fused ste_gemm call (ops.linear_ln),
HIP events around --iters launches each; one JSON line."""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from speech_transcript_embeddings_amd import ops  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / iters, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    M, N = 31936, 1024
    res = {}
    for name, K, pair in (("o_proj", 1024, False), ("ffn_out", 4096, False), ("ffn_out_pair", 4096, True)):
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16()
        b = torch.randn(N, device="cuda") * 0.1
        r = torch.randn(M, N, device="cuda")
        out = torch.empty(M, N, device="cuda")
        g1, b1 = torch.ones(N, device="cuda"), torch.zeros(N, device="cuda")
        yb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        yb2 = torch.empty_like(yb)
        ln1 = dict(gamma=g1, beta=b1, eps=1e-5, yb=yb)
        ln2 = dict(gamma=g1, beta=b1, eps=1e-5, yb=yb2) if pair else None
        t_gemm = timed(lambda: ops.linear(x, w, b, residual=r, out=out), a.iters)
        if pair:
            t_ln = timed(lambda: ops.layernorm_fwd_pair(dict(x=out, **ln1), ln2), a.iters)
        else:
            t_ln = timed(lambda: ops.layernorm_fwd(out, **ln1), a.iters)
        t_fused = timed(lambda: ops.linear_ln(x, w, b, residual=r, out=out, ln=ln1, ln2=ln2), a.iters)
        res[name] = dict(K=K, gemm_us=t_gemm, ln_us=t_ln, separate_us=round(t_gemm + t_ln, 1), fused_us=t_fused)
        print(json.dumps({name: res[name]}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

"""The encoder GEMMs of the c2 step, timed in isolation (HIP events): ste_gemm with the
epilogue the step uses, ste_gemm with a plain bf16 output, and torch.mm (hipBLASLt) on the
same operands — the A/B harness behind DESIGN §3's GEMM numbers.

    python profiles/gemm_probe.py [--rows 31936] [--iters 20] [--only NAME] [--mx8]

--mx8: the forward GEMMs on MX-fp8 operands (ste_gemm_mx8, config 5) with the step's epilogues
(FFN-in: pre-activation + fp8 copy of the output only, as in a frozen layer), next to the bf16
kernel with the same epilogue (run twice, STE_MX8_8PH=0 / 1, to compare the two MX kernels).

Shapes (M = b·T rows of c2 = 64 x 499): forward QKV / O / FFN-in / FFN-out, the input-gradient
(dX = dY·W through the cached Wᵀ) and the weight-gradient (dW = dYᵀX, k-major operands,
split-K) GEMMs of one Conformer layer."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=64 * 499)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default=None)
    ap.add_argument("--mx8", action="store_true")
    ap.add_argument("--text", action="store_true")
    a = ap.parse_args()
    from speech_transcript_embeddings_amd import _lib, ops
    M = a.rows
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*s, dt=torch.bfloat16, sc=1.0):
        return (torch.randn(*s, device=dev, generator=g) * sc).to(dt)

    ws = torch.empty((80 << 20) // 4, device=dev)
    D, F = 1024, 4096
    x = rnd(M, D)
    h = rnd(M, F)
    res = rnd(M, D, dt=torch.float32)
    cases = {}
    for name, (k, n, epi) in {"qkv": (D, 3 * D, "bias_bf16"), "o_proj": (D, D, "bias_res"),
                              "ffn_in": (D, F, "bias_swish_c2"), "ffn_out": (F, D, "bias_res"),
                              "dx_ffn_out": (F, D, "dx_bf16"), "dx_qkv": (3 * D, D, "dx_bf16"),
                              "dx_ffn_in_dz": (D, F, "dz_swish")}.items():
        cases[name] = (k, n, epi)
    out = {"rows": M}

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.iters

    if a.text:
        return text_shapes(a, ops, timed, rnd, ws)
    if a.mx8:
        for name, (K, N, epi) in cases.items():
            if not epi.startswith("bias") or (a.only and not name.startswith(a.only)):
                continue
            A = x if K == D else (h if K == F else rnd(M, K))
            W = rnd(N, K, sc=0.02)
            bias = torch.randn(N, device=dev, generator=g) * 0.1
            Aq, Wq = ops.mx8_quant(A), ops.mx8_quant(W)
            kw = dict(bias=bias)
            if epi == "bias_bf16":
                kw.update(out_bf16=True)
            elif epi == "bias_res":
                kw.update(residual=res if N == D else rnd(M, N, dt=torch.float32))
            else:   # FFN-in of a frozen layer: bf16 pre-activation + the fp8 copy only
                kw.update(act=_lib.ACT_SWISH, pre_out=torch.empty(M, N, device=dev, dtype=torch.bfloat16), out=False,
                          q_out=(torch.empty(M, N, device=dev, dtype=torch.uint8),
                                 torch.empty(M, N // 32, device=dev, dtype=torch.uint8)))
            t_mx = timed(lambda: ops.linear_mx8(Aq, Wq, **kw))
            kwb = {k: v for k, v in kw.items() if k not in ("q_out", "out")}
            if epi == "bias_swish_c2":
                kwb.update(out_bf16=True)
            t_bf = timed(lambda: ops.linear(A, W, **kwb))
            fl = 2.0 * M * N * K
            out[name] = {"M": M, "N": N, "K": K, "epilogue": epi, "mx8_us": round(t_mx, 1),
                         "mx8_tflops": round(fl / t_mx / 1e6, 1), "bf16_us": round(t_bf, 1),
                         "bf16_tflops": round(fl / t_bf / 1e6, 1)}
            print(json.dumps({name: out[name]}), flush=True)
        print(json.dumps(out), flush=True)
        return
    for name, (K, N, epi) in cases.items():
        if a.only and not name.startswith(a.only):
            continue
        A = x if K == D else (h if K == F else rnd(M, K))
        W = rnd(N, K, sc=0.02)
        bias = torch.randn(N, device=dev, generator=g) * 0.1
        kw = {}
        if epi == "bias_bf16":
            kw = dict(bias=bias, out_bf16=True)
        elif epi == "bias_res":
            kw = dict(bias=bias, residual=res if N == D else rnd(M, N, dt=torch.float32))
        elif epi == "bias_swish_c2":
            kw = dict(bias=bias, act=_lib.ACT_SWISH, pre_out=torch.empty(M, N, device=dev, dtype=torch.bfloat16),
                      out_bf16=True)
        elif epi == "dx_bf16":
            kw = dict(out_bf16=True)
        elif epi == "dz_swish":
            kw = dict(act=_lib.ACT_SWISH_BWD, z=rnd(M, N), out_bf16=True,
                      colsum=torch.zeros(N, device=dev))
        o_epi = torch.empty(M, N, device=dev, dtype=torch.bfloat16 if kw.get("out_bf16") else torch.float32)
        o_plain = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        t_epi = timed(lambda: ops.linear(A, W, out=o_epi, **{k: v for k, v in kw.items() if k != "out_bf16"}))
        t_plain = timed(lambda: ops.linear(A, W, out=o_plain))
        Wt = W.t().contiguous()
        t_blas = timed(lambda: torch.mm(A, Wt, out=o_plain))
        fl = 2.0 * M * N * K
        out[name] = {"M": M, "N": N, "K": K, "epilogue": epi,
                     "ste_epilogue_us": round(t_epi, 1), "ste_epilogue_tflops": round(fl / t_epi / 1e6, 1),
                     "ste_plain_us": round(t_plain, 1), "ste_plain_tflops": round(fl / t_plain / 1e6, 1),
                     "hipblaslt_plain_us": round(t_blas, 1), "hipblaslt_plain_tflops": round(fl / t_blas / 1e6, 1)}
        print(json.dumps({name: out[name]}), flush=True)
    # weight gradients: dW[N,K] = dYᵀ·X over M rows (k-major operands, split-K slabs)
    for name, (N, K) in {"dw_ffn_in": (F, D), "dw_ffn_out": (D, F), "dw_qkv": (3 * D, D), "dw_o": (D, D)}.items():
        if a.only and not name.startswith(a.only):
            continue
        dy = rnd(M, N)
        X = x if K == D else h
        dw = torch.zeros(N, K, device=dev)
        t_ste = timed(lambda: ops.linear_dw(dy, X, out=dw, beta=1.0, ws=ws))
        dwb = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        t_blas = timed(lambda: torch.mm(dy.t(), X, out=dwb))
        fl = 2.0 * M * N * K
        out[name] = {"M": N, "N": K, "K": M, "kernel": ops.gemm_kernel_name(_dw_args(ops, dy, X, dw, ws)),
                     "ste_us": round(t_ste, 1), "ste_tflops": round(fl / t_ste / 1e6, 1),
                     "hipblaslt_us": round(t_blas, 1), "hipblaslt_tflops": round(fl / t_blas / 1e6, 1)}
        print(json.dumps({name: out[name]}), flush=True)
    print(json.dumps(out), flush=True)


def text_shapes(a, ops, timed, rnd, ws):
    """--text: the text encoder's N = 768 outputs at M = 8,192 rows (c2: 64 pairs x 2 x 64
    tokens), 96 tiles of 256 x 256: the forward O-proj / FFN-out of the split-bf16 (precise)
    forward (K doubled: [hi | lo]) and the QKV / FFN-in input gradients, each with the step's
    epilogue, timed with and without the workspace (the few-tile split-K plan needs it).  Run
    under STE_GEMM_MIN_TILES / STE_GEMM_FEW_SPLIT to compare the kernel choices."""
    M, D = 8192, 768
    dev = "cuda"
    out = {"rows": M, "min_tiles": os.environ.get("STE_GEMM_MIN_TILES", "240"),
           "few_split": os.environ.get("STE_GEMM_FEW_SPLIT", "1")}
    res = rnd(M, D, dt=torch.float32)
    bias = torch.randn(D, device=dev) * 0.1
    for name, (K, epi) in {"o_fwd_precise": (2 * D, "BRD"), "ffn_out_fwd_precise": (8 * D, "BRD"),
                           "dx_qkv": (3 * D, "R"), "dx_ffn_in": (4 * D, "R"), "dx_o": (D, "bf16")}.items():
        A = rnd(M, K)
        W = rnd(D, K, sc=0.02)
        if epi == "BRD":
            kw = dict(bias=bias, residual=res, drop_p=0.1, seed=7)
            o = torch.empty(M, D, device=dev)
        elif epi == "R":
            kw = dict(residual=res)
            o = torch.empty(M, D, device=dev)
        else:
            kw = {}
            o = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
        ref = ops.linear(A, W, out=torch.empty_like(o), **kw).float()
        t0 = timed(lambda: ops.linear(A, W, out=o, **kw))
        t1 = timed(lambda: ops.linear(A, W, out=o, ws=ws, **kw))
        err = ((o.float() - ref).abs().max() / ref.abs().max()).item()
        fl = 2.0 * M * D * K
        out[name] = {"K": K, "epilogue": epi, "no_ws_us": round(t0, 1), "no_ws_tflops": round(fl / t0 / 1e6, 1),
                     "ws_us": round(t1, 1), "ws_tflops": round(fl / t1 / 1e6, 1), "ws_vs_no_ws_rel": err}
        print(json.dumps({name: out[name]}), flush=True)
    print(json.dumps(out), flush=True)


def _dw_args(ops, dy, x, dw, ws):
    from speech_transcript_embeddings_amd._lib import GemmArgs, ptr
    a = GemmArgs()
    a.M, a.N, a.K, a.batch = dy.shape[1], x.shape[1], dy.shape[0], 1
    a.A, a.lda, a.a_kc = ptr(dy), dy.stride(0), 0
    a.B, a.ldb, a.b_kc = ptr(x), x.stride(0), 0
    a.C, a.ldc = ptr(dw), dw.stride(0)
    a.alpha, a.beta = 1.0, 1.0
    a.ws, a.ws_bytes = ptr(ws), ws.numel() * 4
    return a


if __name__ == "__main__":
    main()

"""Time one libste.so kernel configuration in isolation with HIP events (GPU, scratch probe).
    python profiles/kernel_timer.py text_attn_f32      # the precise text forward's attention at c2
"""
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from speech_transcript_embeddings_amd import ops  # noqa: E402

ops.LN_ATOMIC_COLSUMS = os.environ.get("STE_LN_ATOMIC") == "1"   # A/B: LN column sums by fp32 atomics


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def text_attn_f32():
    B, T, H, D = 128, 64, 12, 64
    W = H * D
    qkv = torch.randn(B * T, 3 * W, device="cuda")
    mask = torch.ones(B * T, dtype=torch.int32, device="cuda")
    os_ = torch.empty(B * T, 2 * W, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H * T, device="cuda")
    for p in (0.0, 0.1):
        us = timeit(lambda: ops.attention_fwd_f32(qkv[:, :W], qkv[:, W:2 * W], qkv[:, 2 * W:], B=B, T=T, H=H, o32=None,
                                                  lse=lse, o=os_[:, :W], o_lo=os_[:, W:], key_mask=mask, drop_p=p,
                                                  seed=1))
        qb = qkv.bfloat16()
        o = torch.empty(B * T, W, device="cuda", dtype=torch.bfloat16)
        us_b = timeit(lambda: ops.attention_fwd(qb[:, :W], qb[:, W:2 * W], qb[:, 2 * W:], B=B, T=T, H=H, o=o, lse=lse,
                                                key_mask=mask, drop_p=p, seed=1, o_lo=os_[:, W:]))
        print(f"text attention fwd B={B} T={T} H={H} drop={p}: fp32 {us:.1f} us, bf16 kernel {us_b:.1f} us")




def layernorm():
    """c2 Conformer LayerNorms (rows 31,936 x 1,024): forward to bf16, the chained pair, backward
    with the residual gradient (dx fp32 + dxb bf16); GB/s of algorithmic bytes."""
    R, D = 64 * 499, 1024
    x = torch.randn(R, D, device="cuda")
    g, b = torch.rand(D, device="cuda") + 0.5, torch.randn(D, device="cuda") * 0.1
    yb = torch.empty(R, D, device="cuda", dtype=torch.bfloat16)
    y = torch.empty(R, D, device="cuda")
    yb2 = torch.empty_like(yb)
    st = ops.layernorm_fwd(x, g, b, 1e-5, yb=yb)
    us = timeit(lambda: ops.layernorm_fwd(x, g, b, 1e-5, yb=yb, mean=st[0], rstd=st[1]))
    print(f"ln fwd -> bf16: {us:.1f} us, {R * D * 6 / us / 1e3:.0f} GB/s", flush=True)
    us = timeit(lambda: ops.layernorm_fwd_pair(dict(x=x, gamma=g, beta=b, eps=1e-5, y=y, yb=yb),
                                               dict(gamma=g, beta=b, eps=1e-5, yb=yb2)))
    print(f"ln fwd pair (y fp32 + bf16, then bf16): {us:.1f} us, {R * D * 12 / us / 1e3:.0f} GB/s", flush=True)
    dy = torch.randn(R, D, device="cuda").bfloat16()
    dres = torch.randn(R, D, device="cuda")
    dx = torch.empty(R, D, device="cuda")
    dxb = torch.empty(R, D, device="cuda", dtype=torch.bfloat16)
    us = timeit(lambda: ops.layernorm_bwd(dy, x, st[0], st[1], g, beta=b, dres=dres, dx=dx, dxb=dxb))
    print(f"ln bwd (dy bf16, x, dres -> dx, dxb): {us:.1f} us, {R * D * 16 / us / 1e3:.0f} GB/s", flush=True)
    us = timeit(lambda: ops.layernorm_bwd(dy, x, st[0], st[1], g, beta=b, dres=dres, dx=dx, dxb=dxb,
                                          dgamma=torch.zeros(D, device="cuda"), dbeta=torch.zeros(D, device="cuda")))
    print(f"ln bwd + dgamma/dbeta: {us:.1f} us, {R * D * 16 / us / 1e3:.0f} GB/s", flush=True)
    y1 = torch.empty_like(x)
    (ma, ra), (mb, rb) = ops.layernorm_fwd_pair(dict(x=x, gamma=g, beta=b, eps=1e-5, y=y1),
                                                dict(gamma=g, beta=b, eps=1e-5, yb=yb2))
    Z = lambda: torch.zeros(D, device="cuda")  # noqa: E731
    us = timeit(lambda: ops.layernorm_bwd_pair(
        dict(x=x, mean=ma, rstd=ra, gamma=g, beta=b, dxb=dxb, dgamma=Z(), dbeta=Z(), dsum=Z()),
        dict(dy=dy, x=y1, mean=mb, rstd=rb, gamma=g, beta=b, dres=dres, dgamma=Z(), dbeta=Z())))
    print(f"ln bwd pair + column sums (both LNs): {us:.1f} us", flush=True)


def fbank():
    """c2 batch: 64 clips of 10 s at 16 kHz -> [64, 499, 160] features (three launches)."""
    B, N = 64, 160000
    wav = torch.randn(B, N, device="cuda") * 0.1
    lens = torch.full((B,), N, device="cuda", dtype=torch.int32)
    T = ((1 + (N - 400) // 160) + 1) // 2
    feats = torch.empty(B, T, 160, device="cuda")
    mask = torch.empty(B, T, device="cuda", dtype=torch.int64)
    work = torch.empty(B * 2 * T * 80 + B * 160, device="cuda")
    us = timeit(lambda: ops.fbank(wav, lens, T, feats=feats, mask=mask, work=work))
    nbytes = 4 * B * N + feats.numel() * 4 + mask.numel() * 8
    print(f"fbank (3 launches): {us:.1f} us, {nbytes / us / 1e3:.0f} GB/s algorithmic", flush=True)


if __name__ == "__main__":
    globals()[sys.argv[1]]()

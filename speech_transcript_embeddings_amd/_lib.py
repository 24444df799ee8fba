"""ctypes binding of libste.so (the C ABI declared in include/ste.h).

This module is the only place that touches the shared library.  It fails loudly:
if libste.so is missing or a call returns a non-zero status, a RuntimeError is
raised — there is no CPU or eager-PyTorch fallback anywhere in the product path.

torch is imported first on purpose: torch ships its own libamdhip64.so.7 and
the dynamic loader then resolves libste.so's HIP dependency (same SONAME) to
that already-loaded runtime, so kernels launched here and torch's allocator /
streams share one HIP runtime.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("STE_LIB", _PKG / "libste.so"))
# the A/B build (_build.py --ab: libste_ab.so) is the only configuration whose STE_* switches read
# the environment, on both sides of the ABI; with the shipped libste.so every switch is its default
AB_BUILD = LIB_PATH.name == "libste_ab.so"


def ab_env(name: str, default: str) -> str:
    """An A/B switch's value: the environment's under the A/B build, else `default`."""
    return os.environ.get(name, default) if AB_BUILD else default

c_void_p, c_int, c_int64, c_float, c_uint64, c_char_p = C.c_void_p, C.c_int, C.c_int64, C.c_float, C.c_uint64, C.c_char_p
c_i32p = C.POINTER(C.c_int32)

ACT_NONE, ACT_SWISH, ACT_GELU, ACT_TANH, ACT_RELU = 0, 1, 2, 3, 4
ACT_SWISH_BWD, ACT_GELU_BWD, ACT_TANH_BWD_OUT, ACT_RELU_BWD = 11, 12, 13, 14


class GemmArgs(C.Structure):
    _fields_ = [
        ("M", c_int), ("N", c_int), ("K", c_int), ("batch", c_int),
        ("A", c_void_p), ("lda", c_int64), ("a_kc", c_int),
        ("B", c_void_p), ("ldb", c_int64), ("b_kc", c_int),
        ("strideA", c_int64), ("strideB", c_int64), ("strideC", c_int64), ("strideR", c_int64),
        ("C", c_void_p), ("ldc", c_int64), ("c_bf16", c_int),
        ("C2", c_void_p), ("ldc2", c_int64),
        ("C3", c_void_p), ("ldc3", c_int64),
        ("bias", c_void_p),
        ("R", c_void_p), ("ldr", c_int64), ("r_bf16", c_int),
        ("Z", c_void_p), ("ldz", c_int64),
        ("colsum", c_void_p),
        ("row_scale", c_void_p),
        ("alpha", c_float), ("beta", c_float),
        ("act", c_int),
        ("drop_p", c_float), ("seed", c_uint64), ("drop_ld", c_int64),
        ("ws", c_void_p), ("ws_bytes", c_int64),
        ("c3_lo", c_int),
    ]


class LnFwdArgs(C.Structure):
    _fields_ = [
        ("rows", c_int), ("cols", c_int),
        ("x", c_void_p), ("ldx", c_int64), ("x_bf16", c_int),
        ("gamma", c_void_p), ("beta", c_void_p), ("eps", c_float),
        ("y", c_void_p), ("ldy", c_int64),
        ("yb", c_void_p), ("ldyb", c_int64),
        ("mean", c_void_p), ("rstd", c_void_p),
        ("row_scale", c_void_p),
        ("act", c_int),
        ("drop_p", c_float), ("seed", c_uint64),
        ("q8", c_void_p), ("q8s", c_void_p), ("ldq8", c_int64),
        ("ylo", c_void_p), ("ldylo", c_int64),
    ]


class LnBwdArgs(C.Structure):
    _fields_ = [
        ("rows", c_int), ("cols", c_int),
        ("dy", c_void_p), ("lddy", c_int64), ("dy_bf16", c_int),
        ("x", c_void_p), ("ldx", c_int64), ("x_bf16", c_int),
        ("mean", c_void_p), ("rstd", c_void_p),
        ("gamma", c_void_p), ("beta", c_void_p),
        ("row_scale", c_void_p),
        ("act", c_int),
        ("dres", c_void_p), ("lddres", c_int64),
        ("dx", c_void_p), ("lddx", c_int64),
        ("dxb", c_void_p), ("lddxb", c_int64),
        ("dgamma", c_void_p), ("dbeta", c_void_p),
        ("drop_p", c_float), ("seed", c_uint64), ("out_scale", c_float),
        ("in_drop_p", c_float), ("in_seed", c_uint64),
        ("out_row_scale", c_void_p),
        ("dsum", c_void_p),
        ("ws", c_void_p), ("ws_floats", c_int64),
    ]


class AttnArgs(C.Structure):
    _fields_ = [
        ("B", c_int), ("T", c_int), ("H", c_int),
        ("q", c_void_p), ("ldq", c_int64),
        ("k", c_void_p), ("ldk", c_int64),
        ("v", c_void_p), ("ldv", c_int64),
        ("o", c_void_p), ("ldo", c_int64),
        ("lse", c_void_p),
        ("key_mask", c_void_p),
        ("rel_E", c_void_p), ("rel_left", c_int), ("rel_right", c_int),
        ("scale", c_float),
        ("drop_p", c_float), ("seed", c_uint64),
        ("dout", c_void_p), ("lddo", c_int64),
        ("dq", c_void_p), ("lddq", c_int64),
        ("dk", c_void_p), ("lddk", c_int64),
        ("dv", c_void_p), ("lddv", c_int64),
        ("delta", c_void_p),
        ("dE", c_void_p),
        ("gwork", c_void_p),
        ("o_lo", c_void_p), ("ldolo", c_int64),
        ("zero_masked_rows", c_int),
    ]


# name -> (restype, argtypes); every symbol declared in include/ste.h
_SIGS = {
    "ste_gemm": (c_int, [C.POINTER(GemmArgs), c_void_p]),
    "ste_gemm_f32": (c_int, [C.POINTER(GemmArgs), c_void_p]),
    "ste_gemm_kernel": (c_int, [C.POINTER(GemmArgs)]),
    "ste_gemm_colsum_ws_floats": (c_int64, [C.POINTER(GemmArgs)]),
    "ste_gemm_tile_map": (c_int, [c_int, c_int, c_int, C.POINTER(c_int), C.POINTER(c_int)]),
    "ste_gemm_kernel_name": (c_int, [C.POINTER(GemmArgs), c_char_p, c_int]),
    "ste_rows_extract": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                 c_void_p, c_void_p]),
    "ste_rows_accumulate": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_float, c_void_p]),
    "ste_layernorm_fwd": (c_int, [C.POINTER(LnFwdArgs), c_void_p]),
    "ste_layernorm_bwd": (c_int, [C.POINTER(LnBwdArgs), c_void_p]),
    "ste_layernorm_fwd_pair": (c_int, [C.POINTER(LnFwdArgs), C.POINTER(LnFwdArgs), c_void_p]),
    "ste_layernorm_bwd_pair": (c_int, [C.POINTER(LnBwdArgs), C.POINTER(LnBwdArgs), c_void_p]),
    "ste_layernorm_bwd_ws_floats": (c_int64, [c_int, c_int]),
    "ste_attention_fwd": (c_int, [C.POINTER(AttnArgs), c_void_p]),
    "ste_attention_bwd": (c_int, [C.POINTER(AttnArgs), c_void_p]),
    "ste_attention_fwd_f32": (c_int, [C.POINTER(AttnArgs), c_void_p, c_int64, c_void_p]),
    "ste_attention_bwd_f32": (c_int, [C.POINTER(AttnArgs), c_void_p]),
    "ste_split_bf16": (c_int, [c_void_p, c_int64, c_int64, c_int, c_void_p, c_int, c_int, c_void_p]),
    "ste_glu_dwconv_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "ste_glu_dwconv_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                   c_void_p, c_int64, c_void_p]),
    "ste_glu_dwconv_bwd_ws_floats": (c_int64, [c_int, c_int, c_int, c_int]),
    "ste_fbank": (c_int, [c_void_p, c_int64, c_void_p, c_int, c_int, c_float, c_void_p, c_void_p, c_int, c_void_p,
                          c_void_p]),
    "ste_gemm_mx8": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "ste_gemm_mx8_kernel": (c_int, [C.POINTER(GemmArgs), c_int]),
    "ste_gemm_plan_min_tiles": (c_int, [c_int, c_int, C.POINTER(c_int), C.POINTER(c_int)]),
    "ste_mx8_quant": (c_int, [c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "ste_attn_pool_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                  c_void_p, c_void_p, c_void_p, c_void_p]),
    "ste_attn_pool_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                  c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p]),
    "ste_attn_pool_bwd_work_floats": (c_int, [c_int, c_int, c_int]),
    "ste_attn_pool_fwd_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                      c_void_p, c_void_p, c_void_p, c_void_p]),
    "ste_attn_pool_bwd_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                      c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p]),
    "ste_mean_pool_fwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                  c_void_p]),
    "ste_mean_pool_fwd_f32": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                      c_void_p]),
    "ste_weighted_pool_bwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "ste_xattn1_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int, c_int, c_int, c_int, c_float,
                               c_float, c_uint64, c_void_p, c_void_p, c_void_p]),
    "ste_xattn1_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int, c_int,
                               c_int, c_int, c_float, c_float, c_uint64, c_void_p, c_void_p, c_void_p, c_int64,
                               c_void_p]),
    "ste_xattn_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int, c_int, c_int, c_int, c_int,
                              c_float, c_float, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p]),
    "ste_xattn_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int, c_int,
                              c_int, c_int, c_int, c_float, c_float, c_uint64, c_uint64, c_void_p, c_void_p,
                              c_void_p, c_int64, c_void_p]),
    "ste_xattn_bwd_bf16": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int,
                                   c_int, c_int, c_int, c_int, c_float, c_float, c_uint64, c_uint64, c_void_p,
                                   c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "ste_align_attn_fwd": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                   c_float, c_uint64, c_void_p, c_void_p, c_int64, c_void_p]),
    "ste_align_attn_bwd": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int, c_int,
                                   c_int, c_int, c_int, c_float, c_uint64, c_void_p, c_void_p, c_int64, c_void_p,
                                   c_int64, c_void_p]),
    "ste_rank1_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                              c_void_p]),
    "ste_l2norm_fwd": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "ste_l2norm_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "ste_similarity": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "ste_pair_loss_fwd": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_int, c_int, c_float, c_float, c_float,
                                  c_void_p, c_void_p, c_void_p, c_void_p]),
    "ste_pair_loss_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_float, c_float, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_void_p]),
    "ste_pair_sim_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                 c_void_p, c_void_p]),
    "ste_pair_metrics": (c_int, [c_void_p, c_int64, c_int, c_int, c_float, c_void_p, c_int, c_float, c_void_p,
                                 c_void_p]),
    "ste_inbatch_ce": (c_int, [c_void_p, c_int64, c_int, c_int, c_int, c_float, c_float, c_void_p, c_void_p, c_void_p,
                               c_int64, c_void_p]),
    "ste_rowmat_f32": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "ste_text_embed_fwd": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p]),
    "ste_text_embed_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_int64, c_void_p]),
    "ste_text_embed_bwd_ws_floats": (c_int64, [c_int, c_int, c_int]),
    "ste_sumsq": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "ste_adamw": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float, c_float,
                          c_float, c_float, c_int, c_void_p, c_float, c_void_p]),
    "ste_cast_f32_bf16": (c_int, [c_void_p, c_void_p, c_int64, c_void_p]),
    "ste_colsum": (c_int, [c_void_p, c_int, c_int64, c_int, c_int64, c_void_p, c_void_p, c_int64, c_void_p]),
    "ste_colsum_ws_floats": (c_int64, [c_int64, c_int]),
    "ste_rowsum_ordered": (c_int, [c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p]),
    "ste_axpby2d": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int, c_float, c_float, c_void_p]),
    "ste_copy2d": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int, c_int, c_void_p]),
    "ste_transpose16": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int, c_void_p]),
    "ste_spec_mask_fwd": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p]),
    "ste_spec_mask_bwd": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p, c_int64,
                                  c_void_p]),
    "ste_spec_mask_bwd_ws_floats": (c_int64, [c_int64, c_int]),
    "ste_scale_rows": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_int64, c_void_p]),
    "ste_mask_i64_to_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p]),
    "ste_w2v_conv0_fwd": (c_int, [c_void_p, c_int64, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                  c_void_p]),
    "ste_w2v_gn_work": (c_int64, [c_int, c_int, c_int, c_int]),
    "ste_w2v_gn_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_int64, c_void_p]),
    "ste_w2v_gn_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int,
                               c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                               c_void_p]),
    "ste_w2v_slab_sum": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p]),
    "ste_w2v_conv_fold": (c_int, [c_void_p, c_int64, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                  c_int, c_void_p]),
    "ste_w2v_perm12": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "ste_w2v_pos_pack": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "ste_w2v_pos_elem": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                                 c_void_p]),
    "ste_w2v_wnorm_fwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "ste_w2v_wnorm_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                  c_void_p]),
    "ste_w2v_frame_mask": (c_int, [c_void_p, c_int, c_int, c_int, c_int, C.POINTER(c_int), C.POINTER(c_int), c_void_p,
                                   c_void_p, c_void_p]),
    "ste_w2v_wave_norm": (c_int, [c_void_p, c_int64, c_void_p, c_int, c_int, c_float, c_void_p, c_void_p]),
    "ste_w2v_drop_rows": (c_int, [c_void_p, c_int, c_int, c_float, c_uint64, c_void_p, c_void_p]),
    "ste_version": (C.c_char_p, []),
}

SYMBOLS = tuple(_SIGS)
_lib = None


class SteError(RuntimeError):
    pass


def load() -> C.CDLL:
    """Load libste.so (once).  Raises if it is missing: no fallback exists."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise SteError(f"{LIB_PATH} not found — build it with __graft_entry__.build() "
                           "(speech_transcript_embeddings_amd/_build.py); there is no fallback path")
        _lib = C.CDLL(str(LIB_PATH))
    return _lib


_fns: dict = {}


def fn(name: str):
    f = _fns.get(name)
    if f is None:
        f = getattr(load(), name)
        f.restype, f.argtypes = _SIGS[name]
        _fns[name] = f
    return f


def call(name: str, *args) -> None:
    rc = fn(name)(*args)
    if rc != 0:
        raise SteError(f"{name} failed with status {rc}")


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int | None:
    """Device pointer of a tensor (None for None)."""
    return None if t is None else t.data_ptr()

"""CPU checks of the C-ABI boundary (include/ste.h <-> libste.so <-> _lib.py).

No kernel is launched: the library is loaded (its HIP runtime dependency resolves to the
one torch ships), every declared symbol must be exported, the ctypes signature table must
cover exactly the header, and the host-only entry points (version string, GEMM kernel
selection, argument validation that returns before any launch) are exercised."""
import ctypes as C
import re

import pytest

from conftest import ROOT

HEADER = ROOT / "include" / "ste.h"


def _declared():
    txt = HEADER.read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(ste_\w+)\s*\(", txt, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    from speech_transcript_embeddings_amd import _lib
    if not _lib.LIB_PATH.exists():
        pytest.fail("libste.so not built — run __graft_entry__.build()")
    return _lib


def test_header_declares_the_path():
    names = _declared()
    for must in ["ste_gemm", "ste_layernorm_fwd", "ste_layernorm_bwd", "ste_attention_fwd", "ste_attention_bwd",
                 "ste_glu_dwconv_fwd", "ste_fbank", "ste_pair_loss_fwd", "ste_adamw", "ste_align_attn_fwd"]:
        assert must in names, must


def test_library_exports_every_declared_symbol(lib):
    so = lib.load()
    missing = [n for n in _declared() if not hasattr(so, n)]
    assert not missing, missing


def test_ctypes_table_matches_header(lib):
    assert sorted(lib.SYMBOLS) == _declared()


def test_version(lib):
    assert lib.fn("ste_version")().decode().endswith("gfx950")


def test_gemm_kernel_selection(lib):
    a = lib.GemmArgs()
    # encoder FFN GEMM at c2: M = 64*499 tokens -> the 256x256 8-phase global_load_lds kernel
    a.M, a.N, a.K, a.batch, a.a_kc, a.b_kc = 31936, 4096, 1024, 1, 1, 1
    assert lib.fn("ste_gemm_kernel")(C.byref(a)) == 8
    a.b_kc = 0
    assert lib.fn("ste_gemm_kernel")(C.byref(a)) == 9
    # weight-gradient reduction (A = dYᵀ) and small head GEMMs stay on the 128x128 kernel
    a.a_kc, a.b_kc = 0, 0
    assert lib.fn("ste_gemm_kernel")(C.byref(a)) == 3
    a.a_kc, a.b_kc, a.M, a.N = 1, 1, 64, 768
    assert lib.fn("ste_gemm_kernel")(C.byref(a)) == 0
    a.K = 1000  # K % 64 != 0 -> small kernel
    a.M, a.N = 31936, 4096
    assert lib.fn("ste_gemm_kernel")(C.byref(a)) == 0


@pytest.mark.parametrize("num_m,num_n", [(125, 16), (125, 12), (125, 4), (32, 9), (1, 16), (7, 8), (3, 3), (125, 8)])
def test_gemm_tile_raster(lib, num_m, num_n):
    """The GEMM kernels' tile order (ste_gemm_tile_map, the same function the device code calls) is
    a bijection onto the tile grid that walks groups of 8 m-tiles, m fastest: 32 consecutive ids
    (one XCD's CUs at a time) at N = 1,024 (4 tiles wide) are 8 A row panels x 4 W column panels."""
    f = lib.fn("ste_gemm_tile_map")
    tm, tn = C.c_int(), C.c_int()
    seen = []
    for t in range(num_m * num_n):
        assert f(t, num_m, num_n, C.byref(tm), C.byref(tn)) == 0
        assert 0 <= tm.value < num_m and 0 <= tn.value < num_n
        seen.append((tm.value, tn.value))
    assert len(set(seen)) == num_m * num_n
    assert f(num_m * num_n, num_m, num_n, C.byref(tm), C.byref(tn)) != 0
    for t, (m, n) in enumerate(seen):
        g0 = (t // (8 * num_n)) * 8
        gsize = min(8, num_m - g0)
        j = t % (8 * num_n)
        assert (m, n) == (g0 + j % gsize, j // gsize)
    if num_n == 4 and num_m >= 8:
        w = seen[:32]
        assert len({m for m, _ in w}) == 8 and len({n for _, n in w}) == 4


def test_gemm_split_policies(lib):
    """Host-side plan choice (no launch): the few-tile split-K of narrow outputs and the batched
    k-major weight gradients on the 8-phase kernel (kernel ids: include/ste.h)."""
    k = lib.fn("ste_gemm_kernel")
    a = lib.GemmArgs()
    # text FFN-out at c2, split-bf16 forward: 96 tiles, 96 K-tiles, workspace given -> 2 K-slabs
    a.M, a.N, a.K, a.batch, a.a_kc, a.b_kc = 8192, 768, 6144, 1, 1, 1
    a.ws, a.ws_bytes = 1, 80 << 20
    assert k(C.byref(a)) == 12
    a.ws, a.ws_bytes = None, 0                      # no workspace: the 128x128 kernel
    assert k(C.byref(a)) == 0
    a.ws, a.ws_bytes = 1, 2 * 8192 * 768 * 4 - 4    # workspace one float short of 2 slabs
    assert k(C.byref(a)) == 0
    a.ws_bytes = 80 << 20
    a.K = 2304                                      # 36 K-tiles: below the plan's 40
    assert k(C.byref(a)) == 0
    a.K, a.colsum = 6144, 1                         # column sums are never split
    assert k(C.byref(a)) == 0
    a.colsum = None
    a.M = 31936                                     # 375 tiles fill the chip: unsplit 8-phase
    assert k(C.byref(a)) == 8
    # wav2vec2 conv1 dW at b = 64: per-clip slabs, both operands k-major, ragged K -> 8-phase
    b = lib.GemmArgs()
    b.M, b.N, b.K, b.batch, b.a_kc, b.b_kc = 512, 1536, 15999, 64, 0, 0
    assert k(C.byref(b)) == 11
    buf = C.create_string_buffer(128)
    lib.fn("ste_gemm_kernel_name")(C.byref(b), buf, 128)
    assert buf.value == b"gemm_8ph_kernel<false, false, 0, 0>"
    b.batch = 4                                     # 48 tiles: stays on the small kernel
    assert k(C.byref(b)) == 3
    b.batch, b.bias = 64, 1                         # any epilogue beyond alpha/beta: small kernel
    assert k(C.byref(b)) == 3


def test_gemm_mx8_plan(lib):
    """ste_gemm_mx8's kernel choice (no launch): the 8-phase MX kernel addresses its operands by
    32-bit byte offsets, so an operand of 4 GiB or more must take the single-stage kernel
    (ADVICE r3)."""
    k = lib.fn("ste_gemm_mx8_kernel")
    a = lib.GemmArgs()
    # c5 FFN-out: M = 64 x 1499 frames, bias + fp32 residual
    a.M, a.N, a.K, a.batch, a.a_kc, a.b_kc, a.lda, a.ldb = 95936, 1024, 4096, 1, 1, 1, 4096, 4096
    a.C, a.bias, a.R = 1, 1, 1
    assert k(C.byref(a), 0) == 1
    a.M = (1 << 32) // 4096 + 256                   # M·lda crosses 4 GiB of fp8 bytes
    assert k(C.byref(a), 0) == 0
    a.M = (1 << 32) // 4096 - 256                   # just below
    assert k(C.byref(a), 0) == 1
    a.M, a.N, a.ldb = 95936, 1024, (1 << 32) // 1024   # B operand over the limit
    assert k(C.byref(a), 0) == 0
    a.ldb = 4096
    a.R = None                                      # bias + fp32 out: no compile-time MX epilogue
    assert k(C.byref(a), 0) == 0
    a.R, a.M = 1, 512                               # 8 tiles: single-stage
    assert k(C.byref(a), 0) == 0


def test_gemm_plan_min_tiles(lib):
    """ste_gemm_plan_min_tiles (host-only): the tile counts from which the persistent 8-phase bf16 /
    MX-fp8 kernels are planned (240 by default); the parity tests lower them to 1 (ops.bench_gemm_plan)
    so that a B <= 4 instance runs the compile-time epilogue instantiations of the b = 64 step, then
    restore them."""
    f = lib.fn("ste_gemm_plan_min_tiles")
    pb, pm = C.c_int(), C.c_int()
    assert f(0, 0, C.byref(pb), C.byref(pm)) == 0
    assert (pb.value, pm.value) == (240, 240)
    k, km = lib.fn("ste_gemm_kernel"), lib.fn("ste_gemm_mx8_kernel")
    a = lib.GemmArgs()   # FFN-in of a B = 2 c2 instance: 998 rows, 4 x 16 tiles, bias + swish + C2, bf16 out
    a.M, a.N, a.K, a.batch, a.a_kc, a.b_kc, a.lda, a.ldb = 998, 4096, 1024, 1, 1, 1, 1024, 1024
    a.C, a.c_bf16, a.bias, a.C2, a.act = 1, 1, 1, 1, 1
    b = lib.GemmArgs()   # MX-fp8 FFN-out of a B = 1 c5 instance: 1,499 rows, 6 x 4 tiles, bias + residual
    b.M, b.N, b.K, b.batch, b.a_kc, b.b_kc, b.lda, b.ldb = 1499, 1024, 4096, 1, 1, 1, 4096, 4096
    b.C, b.bias, b.R = 1, 1, 1
    assert k(C.byref(a)) == 0 and km(C.byref(b), 0) == 0
    f(1, 1, None, None)
    try:
        assert k(C.byref(a)) == 8 and km(C.byref(b), 0) == 1
        buf = C.create_string_buffer(128)
        lib.fn("ste_gemm_kernel_name")(C.byref(a), buf, 128)
        assert buf.value == b"gemm_8ph_kernel<true, true, 515, 1>"
    finally:
        f(pb.value, pm.value, None, None)
    assert k(C.byref(a)) == 0 and km(C.byref(b), 0) == 0


def test_argument_errors_return_status_without_launch(lib):
    """Shape/alignment contract violations come back as non-zero status (-> SteError), never a launch."""
    a = lib.GemmArgs()
    a.M, a.N, a.K, a.a_kc, a.b_kc, a.lda, a.ldb = 64, 64, 100, 1, 1, 100, 100  # K % 8 != 0
    assert lib.fn("ste_gemm")(C.byref(a), None) != 0
    a.K = 0
    assert lib.fn("ste_gemm")(C.byref(a), None) != 0
    with pytest.raises(lib.SteError):
        lib.call("ste_copy2d", None, 1, None, 1, 4, 4, 3, None)  # elem_bytes must be 2 or 4
    assert lib.fn("ste_scale_rows")(None, None, 4, 0, 1, None) != 0


def test_attention_contract_errors(lib):
    """The attention entry points reject a relative window past the 80-bin table, unaligned row
    strides and a dropout rate outside [0, 1) with a status, before any launch."""
    ERR_ARG, ERR_SHAPE = 1001, 1002                       # include/ste.h STE_ERR_ARG / STE_ERR_SHAPE
    a = lib.AttnArgs()
    a.B, a.T, a.H = 2, 100, 2
    a.ldq = a.ldk = a.ldv = a.ldo = 384
    a.rel_E, a.rel_left, a.rel_right = 16, 72, 8          # 81 bins (pointer never dereferenced)
    assert lib.fn("ste_attention_fwd")(C.byref(a), None) == ERR_SHAPE
    assert lib.fn("ste_attention_bwd")(C.byref(a), None) == ERR_SHAPE
    a.rel_left = 71                                       # 80 bins, but no o / lse given
    assert lib.fn("ste_attention_fwd")(C.byref(a), None) == ERR_ARG
    a.ldk = 388                                           # row stride not a multiple of 8 elements
    assert lib.fn("ste_attention_fwd")(C.byref(a), None) == ERR_SHAPE
    a.ldk, a.drop_p = 384, 1.0
    assert lib.fn("ste_attention_fwd")(C.byref(a), None) == ERR_ARG

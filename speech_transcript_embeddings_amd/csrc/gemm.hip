// bf16 MFMA GEMM with fused epilogues — every nn.Linear / pointwise Conv1d of the
// hot path (forward Y = X·Wᵀ, backward dX = dY·W and dW = dYᵀ·X) runs through here.
//
// Replaces the aten::addmm / aten::mm calls behind nn.Linear in
//   transformers models/wav2vec2_bert/modeling_wav2vec2_bert.py:119-226,229-337 (FFN, QKVO, pointwise convs)
//   transformers models/xlm_roberta/modeling_xlm_roberta.py:186-398             (QKV, O, FFN)
//   /root/reference/training/trainer_unfreeze.py:66-310,436-491                 (heads)
//
// C[m,n] = Σ_k A[m,k]·B[k,n]; operand layouts are "KC" (k contiguous: A[m*lda+k],
// B[n*ldb+k] — the nn.Linear weight layout) or "KM" (k-major: A[k*lda+m], B[k*ldb+n]).
//   forward  Y  = X·Wᵀ : A=X  (KC), B=W  (KC)
//   backward dX = dY·W : A=dY (KC), B=W  (KM)
//   backward dW = dYᵀX : A=dY (KM), B=X  (KM)
// KM tiles are staged k-major in LDS and read with ds_read_b64_tr_b16 (hardware
// transpose), so no operand is ever transposed in HBM.
//
// Two kernels, chosen per shape:
//  * gemm_big: 256x256x64 tile, 512 threads (8 waves as 2(M)x4(N), 128x64 per wave,
//    8x4 v_mfma_f32_16x16x32_bf16), operands streamed global->LDS with global_load_lds
//    (16 B/lane, no VGPR staging) into a 2-deep LDS ring whose XOR swizzle is realised
//    through the per-lane SOURCE address (the LDS image is lane-linear).  Used when the
//    grid has >= ~1 wave of 256 CUs and K % 64 == 0 (all big encoder GEMMs).
//  * gemm_bf16_kernel: 128x128x64 tile, 256 threads, register-staged (zero-filled
//    tails in every dimension): small / ragged GEMMs and the dW reductions.
// Both: XCD-aware bijective block remap + grouped tile order for L2 reuse, and an
// LDS-staged epilogue with row-contiguous (16 B/lane) loads and stores.
#include <cstdio>
#include <utility>
#include "common.h"
#include "../../include/ste.h"

namespace {


STE_DEV int km_chunk_xor(int k) { return ((k & 3) | ((k >> 1) & 4)) << 1; }

STE_DEV float apply_act(float v, int act) {
  switch (act) {
    case STE_ACT_SWISH: return swish_f(v);
    case STE_ACT_GELU: return gelu_f(v);
    case STE_ACT_TANH: return tanhf(v);
    case STE_ACT_RELU: return fmaxf(v, 0.0f);
    default: return v;
  }
}
STE_DEV float act_grad(float z, int act) {
  switch (act) {
    case STE_ACT_SWISH_BWD: return swish_d(z);
    case STE_ACT_GELU_BWD: return gelu_d(z);
    case STE_ACT_TANH_BWD_OUT: return 1.0f - z * z;   // z holds tanh output
    case STE_ACT_RELU_BWD: return z > 0.0f ? 1.0f : 0.0f;
    default: return 1.0f;
  }
}

// ------------------------------------------------------------------ epilogue
// The calling wave has staged a [nrows x 64] fp32 tile (row stride EPI_LD) at `epi`;
// rows map to output rows row0.., staged columns 0..31 to col0.., 32..63 to col1..
// (col1 = col0 + 32 for a contiguous 64-column slab).  8 lanes per row, 8 columns per
// lane: bf16 outputs leave as one 16-B store per lane (the epilogue is store-ISSUE-bound,
// so instruction count, not bytes, sets its length).
constexpr int EPI_LD = 68;

struct Csum {
  f32x4 lo, hi;
};

STE_DEV f32x8 load_bf16x8(const bf16* p) {
  const bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
  f32x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = (float)v[e];
  return r;
}
STE_DEV void store_bf16x8(bf16* p, f32x8 v) {
  bf16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
  *reinterpret_cast<bf16x8*>(p) = o;
}
STE_DEV f32x8 load_f32x8(const float* p) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
  return f32x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
STE_DEV void store_f32x8(float* p, f32x8 v) {
  *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
  *reinterpret_cast<f32x4*>(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
}
// partial loads/stores for the last columns of a ragged N (e < nval only)
STE_DEV f32x8 load_part(const void* p, bool is_bf16, int nval) {
  f32x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = e < nval ? (is_bf16 ? (float)((const bf16*)p)[e] : ((const float*)p)[e]) : 0.f;
  return r;
}
STE_DEV void store_part(void* p, bool is_bf16, f32x8 v, int nval) {
#pragma unroll
  for (int e = 0; e < 8; ++e)
    if (e < nval) {
      if (is_bf16) ((bf16*)p)[e] = (bf16)v[e];
      else ((float*)p)[e] = v[e];
    }
}
// the low half v - bf16(v) of 8 values (the C3 copy of a [hi | lo] split output, c3_lo)
STE_DEV f32x8 lo8(f32x8 v) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] -= (float)(bf16)v[e];
  return v;
}
STE_DEV f32x8 ld8(const void* p, bool is_bf16, bool full, int nval) {
  if (!full) return load_part(p, is_bf16, nval);
  return is_bf16 ? load_bf16x8((const bf16*)p) : load_f32x8((const float*)p);
}
STE_DEV void st8(void* p, bool is_bf16, f32x8 v, bool full, int nval) {
  if (!full) store_part(p, is_bf16, v, nval);
  else if (is_bf16) store_bf16x8((bf16*)p, v);
  else store_f32x8((float*)p, v);
}

// MX-fp8 block quantisation of 8 values held by each of 4 consecutive lanes (one 32-element
// block): scale 2^e with e = ceil(log2(amax/448)) (no saturation; zero blocks 2^-127), OCP e4m3
// values to q[0..7], the E8M0 byte to *s from the block's first lane.  Used by ste_mx8_quant and
// by the GEMM epilogue's fp8 output (the FFN intermediate feeding the next MX-fp8 GEMM).
STE_DEV void mx8_block_store(f32x8 v, uint8_t* q, uint8_t* s, int lane) {
  float amax = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[e]));
  amax = fmaxf(amax, __shfl_xor(amax, 1));
  amax = fmaxf(amax, __shfl_xor(amax, 2));
  const int ex = mx8_exp(amax);
  const float inv = ldexpf(1.0f, -ex);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = fminf(fmaxf(v[e] * inv, -448.f), 448.f);
  uint32_t lo = 0, hi = 0;
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], lo, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], lo, true);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4], v[5], hi, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6], v[7], hi, true);
  *reinterpret_cast<uint2*>(q) = make_uint2(lo, hi);
  if ((lane & 3) == 0) *s = (uint8_t)(ex + 127);
}

struct Q8Out {  // optional MX-fp8 copy of a GEMM output: q [M][ldq] e4m3, s [M][ldq/32] E8M0
  uint8_t* q;
  uint8_t* s;
  int64_t ldq;
};

// MX-fp8 operands of gemm_8ph_kernel<…, MX = true>: the E8M0 block scales (one per 32 k of a row,
// [rows][K/32] bytes) of A and B, and the optional MX-fp8 copy of the output (generic epilogue)
struct Mx8Args {
  const uint8_t* sa;
  const uint8_t* sb;
  int64_t lsa, lsb;
  Q8Out q8;
};

// The generic epilogue of one lane's 8 columns of one row (run-time feature switches): used by
// the fp32-staged tile epilogue and by the split-K reduction below.
STE_DEV void epi_apply8(const ste_gemm_args& p, f32x8 v, int row, int col, bool full, int nval, f32x8 bias,
                        uint32_t thresh, float inv_keep, int64_t offC, int64_t offR, Csum& csum, const Q8Out* q8,
                        int lane) {
  v = (v + bias) * p.alpha;
  if (p.act >= STE_ACT_SWISH && p.act <= STE_ACT_RELU) {
    if (p.C2) st8((bf16*)p.C2 + offC + (int64_t)row * p.ldc2 + col, true, v, full, nval);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = apply_act(v[e], p.act);
  } else if (p.act >= STE_ACT_SWISH_BWD) {
    const f32x8 z = ld8((const bf16*)p.Z + offC + (int64_t)row * p.ldz + col, true, full, nval);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= act_grad(z[e], p.act);
  }
  if (p.drop_p > 0.f) {
    const uint64_t base = (uint64_t)row * (uint64_t)p.drop_ld + (uint64_t)col;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= drop_scale(p.seed, base + e, thresh, inv_keep);
  }
  if (p.row_scale) v = v * p.row_scale[row];
  if (!full) {
#pragma unroll
    for (int e = 0; e < 8; ++e) if (e >= nval) v[e] = 0.f;
  }
  if (p.colsum) {
    csum.lo += f32x4{v[0], v[1], v[2], v[3]};
    csum.hi += f32x4{v[4], v[5], v[6], v[7]};
  }
  if (p.R) {
    const char* rp = (const char*)p.R + (offR + (int64_t)row * p.ldr + col) * (p.r_bf16 ? 2 : 4);
    v += ld8(rp, p.r_bf16, full, nval);
  }
  char* cp = (char*)p.C + (offC + (int64_t)row * p.ldc + col) * (p.c_bf16 ? 2 : 4);
  if (p.beta != 0.f) v += ld8(cp, p.c_bf16, full, nval) * p.beta;
  if (q8) mx8_block_store(v, q8->q + (int64_t)row * q8->ldq + col, q8->s + (int64_t)row * (q8->ldq >> 5) + (col >> 5),
                          lane);
  if (p.C) st8(cp, p.c_bf16, v, full, nval);
  if (p.C3) st8((bf16*)p.C3 + offC + (int64_t)row * p.ldc3 + col, true, p.c3_lo ? lo8(v) : v, full, nval);
}

STE_DEV void epilogue_tile(const ste_gemm_args& p, const float* epi, int nrows, int row0, int col0, int col1,
                           int batch, int lane, Csum& csum, int ld = EPI_LD, bool swz16 = false,
                           const Q8Out* q8 = nullptr) {
  const int cl = (lane & 7) * 8;  // staged column of this lane's 8
  const int col = cl < 32 ? col0 + cl : col1 + (cl - 32);
  const int nval = p.N - col;     // valid columns from `col`
  if (nval <= 0) return;
  const bool full = nval >= 8;
  const f32x8 bias = p.bias ? ld8(p.bias + col, false, full, nval) : f32x8{};
  const uint32_t thresh = (uint32_t)(p.drop_p * 4294967296.0);
  const float inv_keep = p.drop_p > 0.f ? 1.0f / (1.0f - p.drop_p) : 1.0f;
  const int64_t offC = (int64_t)batch * p.strideC;
  const int64_t offR = (int64_t)batch * p.strideR;
  for (int lr = lane >> 3; lr < nrows; lr += 8) {
    const int row = row0 + lr;
    if (row >= p.M) break;
    const float* src = epi + lr * ld + cl;
    f32x4 s0 = *reinterpret_cast<const f32x4*>(src), s1 = *reinterpret_cast<const f32x4*>(src + 4);
    if (swz16 && ((lr >> 1) & 1)) {  // the 8-phase slot's chunk swizzle (see epi_store16)
      const f32x4 t = s0;
      s0 = s1;
      s1 = t;
    }
    epi_apply8(p, f32x8{s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]}, row, col, full, nval, bias, thresh,
               inv_keep, offC, offR, csum, q8, lane);
  }
}

// the wave's column sums: with a workspace (p.ws, ordered mode, see cs_plan) into partial row prow
// = (batch·num_m + tile_m)·2 + wave row (the ordered second pass sums the rows in order: run-to-run
// deterministic bias gradients), else one fp32 atomic per column
STE_DEV void colsum_flush(const ste_gemm_args& p, Csum csum, int col0, int col1, int batch, int lane,
                          int64_t prow) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
#pragma unroll
    for (int sh = 8; sh < 64; sh <<= 1) {
      csum.lo[e] += __shfl_xor(csum.lo[e], sh, 64);
      csum.hi[e] += __shfl_xor(csum.hi[e], sh, 64);
    }
  }
  const int cl = (lane & 7) * 8;
  const int col = cl < 32 ? col0 + cl : col1 + (cl - 32);
  if (lane < 8) {
    if (p.ws) {
      float* out = p.ws + prow * p.N + col;
      if (col + 8 <= p.N && !(p.N & 3)) {
        *reinterpret_cast<f32x4*>(out) = csum.lo;
        *reinterpret_cast<f32x4*>(out + 4) = csum.hi;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (col + e < p.N) out[e] = csum.lo[e];
          if (col + 4 + e < p.N) out[4 + e] = csum.hi[e];
        }
      }
      return;
    }
    float* out = p.colsum + (int64_t)batch * p.N + col;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (col + e < p.N) atomicAdd(out + e, csum.lo[e]);
      if (col + 4 + e < p.N) atomicAdd(out + 4 + e, csum.hi[e]);
    }
  }
}

// ---------------------------------------------------- specialised epilogue (8-phase)
// The feature set of a launch is a compile-time bitmask for the hot configurations, so a
// pass carries no per-element runtime switches, and every global load of a pass (Z, R,
// beta*C) is issued before any of its stores: the compiler's waits then never serialise
// a row behind the previous row's stores.  EF_GENERIC keeps every feature runtime.
enum : int {
  EF_BIAS = 1, EF_C2 = 2, EF_Z = 4, EF_DROP = 8, EF_RS = 16, EF_COLSUM = 32, EF_R = 64, EF_RBF16 = 128,
  EF_BETA = 256, EF_CBF16 = 512, EF_C3 = 1024,
  EF_Q8 = 2048,   // + MX-fp8 copy of the output (8-phase MX kernel: the FFN intermediate for the next MX GEMM)
  EF_NOC = 4096,  // no C output (with EF_Q8: a frozen layer's FFN intermediate exists only in fp8)
  EF_GENERIC = -1
};

int epi_flags(const ste_gemm_args& a) {
  int f = 0;
  const bool fwd_act = a.act >= STE_ACT_SWISH && a.act <= STE_ACT_RELU;
  const bool bwd_act = a.act >= STE_ACT_SWISH_BWD;
  if (a.bias) f |= EF_BIAS;
  if (a.C2 && fwd_act) f |= EF_C2;
  if (bwd_act) f |= EF_Z;
  if (a.drop_p > 0.f) f |= EF_DROP;
  if (a.row_scale) f |= EF_RS;
  if (a.colsum) f |= EF_COLSUM;
  if (a.R) f |= EF_R | (a.r_bf16 ? EF_RBF16 : 0);
  if (a.beta != 0.f) f |= EF_BETA;
  if (a.c_bf16) f |= EF_CBF16;
  if (a.C3) f |= EF_C3;
  return f;
}

STE_DEV f32x8 act8(f32x8 v, int act) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float x = v[e];
    if (act == STE_ACT_SWISH) v[e] = x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));
    else if (act == STE_ACT_GELU) v[e] = gelu_f(x);
    else if (act == STE_ACT_TANH) v[e] = tanhf(x);
    else if (act == STE_ACT_RELU) v[e] = fmaxf(x, 0.f);
  }
  return v;
}
STE_DEV f32x8 actd8(f32x8 z, int act) {
  f32x8 g;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float x = z[e];
    if (act == STE_ACT_SWISH_BWD) {
      const float sg = __builtin_amdgcn_rcpf(1.0f + __expf(-x));
      g[e] = sg * (1.0f + x * (1.0f - sg));
    } else if (act == STE_ACT_GELU_BWD) g[e] = gelu_d(x);
    else if (act == STE_ACT_TANH_BWD_OUT) g[e] = 1.0f - x * x;
    else if (act == STE_ACT_RELU_BWD) g[e] = x > 0.f ? 1.f : 0.f;
    else g[e] = 1.f;
  }
  return g;
}

// One 16-row pass of a wave's 128 x 64 accumulator block, staged fp32 in the wave's
// private [16][64] LDS slot with 16-B chunks XOR-swizzled by bit 1 of the row
// (chunk ^ ((row >> 1) & 1): conflict-free ds_read_b128, 2-way ds_write_b32 which is free).
// Staged columns 0..31 -> col0.., 32..63 -> col1...  Lane: 8 columns of rows lr and lr + 8.
// FULL: every row < M and every column < N: straight-line code, so the pass issues exactly
// epi_stores<EF>()/8 global stores (the next tile's first vmcnt waits count them).
// epi_load16 issues a pass's global loads (Z, R, beta*C) one pass AHEAD, before the
// previous pass's stores, so waiting for them never waits for in-flight stores.
struct EpiFlags {
  int act;
  bool fwd_act, f_c2, f_z, f_drop, f_rs, f_cs, f_r, r_bf, f_beta, c_bf, f_c3;
};
template <int EF, int ACT>
STE_DEV EpiFlags epi_flags_dev(const ste_gemm_args& p) {
  EpiFlags f;
  if constexpr (EF < 0) {  // generic: every feature at run time
    f.act = p.act;
    f.fwd_act = p.act >= STE_ACT_SWISH && p.act <= STE_ACT_RELU;
    f.f_c2 = p.C2 != nullptr && f.fwd_act;
    f.f_z = p.act >= STE_ACT_SWISH_BWD;
    f.f_drop = p.drop_p > 0.f;
    f.f_rs = p.row_scale != nullptr;
    f.f_cs = p.colsum != nullptr;
    f.f_r = p.R != nullptr;
    f.r_bf = p.r_bf16 != 0;
    f.f_beta = p.beta != 0.f;
    f.c_bf = p.c_bf16 != 0;
    f.f_c3 = p.C3 != nullptr;
  } else {
    f.act = ACT;
    f.fwd_act = ACT >= STE_ACT_SWISH && ACT <= STE_ACT_RELU;
    f.f_c2 = (EF & EF_C2) != 0;
    f.f_z = (EF & EF_Z) != 0;
    f.f_drop = (EF & EF_DROP) != 0;
    f.f_rs = (EF & EF_RS) != 0;
    f.f_cs = (EF & EF_COLSUM) != 0;
    f.f_r = (EF & EF_R) != 0;
    f.r_bf = (EF & EF_RBF16) != 0;
    f.f_beta = (EF & EF_BETA) != 0;
    f.c_bf = (EF & EF_CBF16) != 0;
    f.f_c3 = (EF & EF_C3) != 0;
  }
  return f;
}
// global stores one lane issues over a tile's 8 passes on the FULL path (0 = unknown)
template <int EF>
constexpr int epi_stores() {
  if (EF < 0) return 0;
  return 16 * (((EF & EF_NOC) ? 0 : ((EF & EF_CBF16) ? 1 : 2)) + ((EF & EF_C2) ? 1 : 0) + ((EF & EF_C3) ? 1 : 0) +
               ((EF & EF_Q8) ? 2 : 0));
}
struct EpiLoads {
  f32x8 z[2], r[2], c[2];
};
constexpr int EPI16_FLOATS = 16 * 64;  // one wave's staging slot

template <int EF, int ACT, bool FULL>
STE_DEV void epi_load16(const ste_gemm_args& p, int row0, int col0, int col1, int batch, int lane, EpiLoads& L) {
  const EpiFlags f = epi_flags_dev<EF, ACT>(p);
  const int cl = (lane & 7) * 8;
  const int col = cl < 32 ? col0 + cl : col1 + (cl - 32);
  const int nval = FULL ? 8 : p.N - col;
  const bool full = FULL || nval >= 8;
  const int lr = lane >> 3;
  const int64_t offC = (int64_t)batch * p.strideC;
  const int64_t offR = (int64_t)batch * p.strideR;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int64_t row = row0 + lr + 8 * k;
    L.z[k] = f32x8{};
    L.r[k] = f32x8{};
    L.c[k] = f32x8{};
    if (!FULL && (nval <= 0 || row >= p.M)) continue;
    if (f.f_z) L.z[k] = ld8((const bf16*)p.Z + offC + row * p.ldz + col, true, full, nval);
    if (f.f_r) L.r[k] = ld8((const char*)p.R + (offR + row * p.ldr + col) * (f.r_bf ? 2 : 4), f.r_bf, full, nval);
    if (f.f_beta)
      L.c[k] = ld8((const char*)p.C + (offC + row * p.ldc + col) * (f.c_bf ? 2 : 4), f.c_bf, full, nval);
  }
}

template <int EF, int ACT, bool FULL>
STE_DEV void epi_store16(const ste_gemm_args& p, const float* epi, int row0, int col0, int col1, int batch,
                         int lane, f32x8 bias, const EpiLoads& L, Csum& csum, const Q8Out* q8 = nullptr) {
  const EpiFlags f = epi_flags_dev<EF, ACT>(p);
  const int cg = lane & 7, cl = cg * 8;
  const int col = cl < 32 ? col0 + cl : col1 + (cl - 32);
  const int nval = FULL ? 8 : p.N - col;
  if (!FULL && nval <= 0) return;
  const bool full = FULL || nval >= 8;
  const int lr = lane >> 3;
  const int64_t offC = (int64_t)batch * p.strideC;
  f32x8 v[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int row = lr + 8 * k;
    const int sw = (row >> 1) & 1;  // chunks 2cg, 2cg+1 sit swapped when set
    const float* src = epi + row * 64 + cl;
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(src), s1 = *reinterpret_cast<const f32x4*>(src + 4);
    const f32x4 lo = sw ? s1 : s0, hi = sw ? s0 : s1;
    v[k] = f32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
  const uint32_t thresh = (uint32_t)(p.drop_p * 4294967296.0);
  const float inv_keep = f.f_drop ? 1.0f / (1.0f - p.drop_p) : 1.0f;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int64_t row = row0 + lr + 8 * k;
    if (!FULL && row >= p.M) continue;
    f32x8 x = (v[k] + bias) * p.alpha;
    if (f.f_c2) st8((bf16*)p.C2 + offC + row * p.ldc2 + col, true, x, full, nval);
    if (f.fwd_act) x = act8(x, f.act);
    if (f.f_z) x = x * actd8(L.z[k], f.act);
    if (f.f_drop) {
      const uint64_t base = (uint64_t)row * (uint64_t)p.drop_ld + (uint64_t)col;
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] *= drop_scale(p.seed, base + e, thresh, inv_keep);
    }
    if (f.f_rs) x = x * p.row_scale[row];
    if (!full) {
#pragma unroll
      for (int e = 0; e < 8; ++e) if (e >= nval) x[e] = 0.f;
    }
    if (f.f_cs) {
      csum.lo += f32x4{x[0], x[1], x[2], x[3]};
      csum.hi += f32x4{x[4], x[5], x[6], x[7]};
    }
    if (f.f_r) x += L.r[k];
    if (f.f_beta) x += L.c[k] * p.beta;
    if constexpr (EF >= 0 && (EF & EF_Q8) != 0)   // 4 lanes = one 32-column block (FULL tiles: N % 128 == 0)
      mx8_block_store(x, q8->q + row * q8->ldq + col, q8->s + row * (q8->ldq >> 5) + (col >> 5), lane);
    if (EF < 0 || (EF & EF_NOC) == 0) st8((char*)p.C + (offC + row * p.ldc + col) * (f.c_bf ? 2 : 4), f.c_bf, x, full, nval);
    if (f.f_c3) st8((bf16*)p.C3 + offC + row * p.ldc3 + col, true, p.c3_lo ? lo8(x) : x, full, nval);
  }
}

// ------------------------------------- bf16-staged epilogue (8-phase, bf16 outputs)
// For epilogues with a single bf16 output and no operand loads (plain, bias, bias +
// activation: the dominant bf16 dX GEMM, QKV, pointwise conv 1, FFN-in at inference), the
// kernel issues its MFMAs with the operands swapped (the B fragment as the
// MFMA's A): each 16x16 accumulator block then holds, in lane l, 4 CONSECUTIVE columns
// 4*(l >> 4)..+3 of output row (l & 15).  Bias, activation, Z, column sums are applied in
// that layout; the results are packed to bf16 (one 8-B ds_write_b64 per block) into the
// wave's 4 KiB slot as [32 rows][64 columns] with 16-B chunks XOR-swizzled by (row & 7),
// and read back row-contiguous (16 B = 8 columns per lane) for 16-B global stores: half the
// LDS bytes of fp32 staging, a quarter of its LDS writes, 4 round trips per tile instead of 8.
// Measured (A/B, M 31,936, uniform data): plain bf16 K=1024 +4.8 %, K=4096 +1.1 %, QKV with bias
// +1.4 %.  With a second output (C2) or Z loads / column sums the extra register pressure
// (spills) or the extra image pass lost up to 10 %, so those keep the fp32-staged epilogue.
constexpr int DJ[4] = {0, 16, 128, 144};  // column of accumulator block j from the lane's first column

template <int EF>
constexpr bool epi_bf16s() {
  return EF >= 0 && (EF & EF_CBF16) != 0 &&
         (EF & (EF_R | EF_BETA | EF_C3 | EF_RS | EF_DROP | EF_C2 | EF_COLSUM | EF_Z | EF_Q8 | EF_NOC)) == 0;
}
STE_DEV f32x4 act4(f32x4 v, int act) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float x = v[e];
    if (act == STE_ACT_SWISH) v[e] = x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));
    else if (act == STE_ACT_GELU) v[e] = gelu_f(x);
    else if (act == STE_ACT_TANH) v[e] = tanhf(x);
    else if (act == STE_ACT_RELU) v[e] = fmaxf(x, 0.f);
  }
  return v;
}
// bias of the lane's 4 columns of each accumulator block (zeros past N)
STE_DEV void swap_bias(const ste_gemm_args& p, int n0, int wn, int lane, f32x4 (&bias)[4]) {
  const int col = n0 + wn * 32 + 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = col + DJ[j], nval = p.N - c;
    f32x4 b = {0.f, 0.f, 0.f, 0.f};
    if (nval >= 4) b = *reinterpret_cast<const f32x4*>(p.bias + c);
    else
#pragma unroll
      for (int e = 0; e < 4; ++e) if (e < nval) b[e] = p.bias[c + e];
    bias[j] = b;
  }
}
STE_DEV uint32_t pk2_bf16(float a, float b) {
  const bf16 x = (bf16)a, y = (bf16)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// one 32-row bf16 image in the slot: value(ii, j) of every accumulator block of the pass is
// written as soon as it is computed (no pass-sized register array), then read back as
// 8 columns x 4 rows per lane and stored (rows r, r+8, r+16, r+24 of the pass; chunk c < 4 ->
// columns c0 + 8c, c >= 4 -> c1 + 8(c - 4))
template <bool FULL, typename ValueFn>
STE_DEV void bf16s_pass(char* slot, ValueFn value, bf16* dst, int64_t ld, int row0, int M, int N, int c0, int c1,
                        int lane) {
  const int r16 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int ii = 0; ii < 2; ++ii)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 v = value(ii, j);
      const int r = ii * 16 + r16;
      const int c16 = 2 * j + (g >> 1);  // 16-B chunk of the 128-B row (8 columns)
      const int off = r * 128 + ((c16 ^ (r & 7)) << 4) + 8 * (g & 1);
      *reinterpret_cast<u32x2*>(slot + off) = u32x2{pk2_bf16(v[0], v[1]), pk2_bf16(v[2], v[3])};
    }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  const int c = lane & 7;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = (lane >> 3) + 8 * k;
    const u32x4 w = *reinterpret_cast<const u32x4*>(slot + r * 128 + ((c ^ (r & 7)) << 4));
    const int row = row0 + r;
    const int col = c < 4 ? c0 + 8 * c : c1 + 8 * (c - 4);
    bf16* q = dst + (int64_t)row * ld + col;
    if (FULL) {
      *reinterpret_cast<u32x4*>(q) = w;
    } else if (row < M) {
      const int nval = N - col;
      if (nval >= 8) *reinterpret_cast<u32x4*>(q) = w;
      else
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (e < nval) q[e] = __builtin_bit_cast(bf16, (uint16_t)(w[e >> 1] >> (16 * (e & 1))));
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
}

// acc[i][j]: row m0 + wm*128 + i*16 + (lane & 15), columns n0 + wn*32 + 4*(lane >> 4) + DJ[j] .. +3
// (epi_bf16s<EF>: C = act(alpha * (acc + bias)) in bf16, nothing read)
template <int EF, int ACT, bool FULL>
STE_DEV void epilogue_bf16s(const ste_gemm_args& p, const f32x4 (&acc)[8][4], char* slot, int m0, int n0, int batch,
                            int wm, int wn, int lane_in, const f32x4 (&bias)[4]) {
  static_assert(epi_bf16s<EF>(), "single bf16 output, no operand loads");
  int lane = lane_in;
  asm volatile("" : "+v"(lane));  // keep the lane-derived slot / store addressing out of the main loop
  constexpr bool FWD = ACT >= STE_ACT_SWISH && ACT <= STE_ACT_RELU;
  const int64_t offC = (int64_t)batch * p.strideC;
  const int c0 = n0 + wn * 32, c1 = n0 + 128 + wn * 32;
  const int rbase = m0 + wm * 128;
  const float alpha = p.alpha;
#pragma unroll
  for (int ps = 0; ps < 4; ++ps) {
    auto value = [&](int ii, int j) {
      f32x4 x = acc[2 * ps + ii][j];
      if constexpr ((EF & EF_BIAS) != 0) x += bias[j];
      x *= alpha;
      if (FWD) x = act4(x, ACT);
      return x;
    };
    bf16s_pass<FULL>(slot, value, (bf16*)p.C + offC, p.ldc, rbase + 2 * ps * 16, p.M, p.N, c0, c1, lane);
  }
}

// tile id (after the XCD remap, which hands each XCD's CUs 32 consecutive ids at a time) ->
// (tile_m, tile_n): groups of 8 m-tiles, m fastest within the group, so the 32 concurrent tiles
// of an XCD at N = 1,024 (4 tiles wide) are 8 A row panels x 4 W column panels.  (Round 4 tried
// 4 m-tiles x 8-wide n-blocks for outputs >= 8 tiles wide, fewer A panels per XCD wave: the
// N = 4,096 GEMMs ran 3-8 % slower, profiles/r4n_raster_ab.txt.)  Bijective on [0, num_m * num_n).
#ifndef STE_TILE_GROUP
#define STE_TILE_GROUP 8   // A/B builds: -DSTE_TILE_GROUP=16
#endif
STE_HD void tile_of(int t, int num_m, int num_n, int& tm, int& tn) {
  constexpr int GROUP = STE_TILE_GROUP;
  const int group = t / (GROUP * num_n);
  const int first_m = group * GROUP;
  const int gsize = num_m - first_m < GROUP ? num_m - first_m : GROUP;
  tm = first_m + (t % (GROUP * num_n)) % gsize;
  tn = (t % (GROUP * num_n)) / gsize;
}
// block id -> (batch, tile_m, tile_n)
STE_DEV void map_tile_bid(int bid, int num_m, int num_n, int& batch, int& tm, int& tn) {
  const int tiles = num_m * num_n;
  batch = bid / tiles;
  tile_of(bid - batch * tiles, num_m, num_n, tm, tn);
}
STE_DEV void map_tile(int nwg, int num_m, int num_n, int& batch, int& tm, int& tn) {
  map_tile_bid(xcd_remap(blockIdx.x, nwg), num_m, num_n, batch, tm, tn);
}

// =========================================================== small/ragged kernel
namespace small {
constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_BYTES = BM * BK * 2;
constexpr int EPI_BYTES = 4 * 64 * EPI_LD * 4;
constexpr int LDS_BYTES = (4 * TILE_BYTES > EPI_BYTES) ? 4 * TILE_BYTES : EPI_BYTES;

struct Stage {
  bf16x8 v[4];
};

template <bool KC>
STE_DEV void stage_load(Stage& st, const bf16* __restrict__ base, int64_t ld, int row0, int rows, int k0, int K,
                        int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int c = tid + NT * i;
    int r, kk;
    bool ok;
    const bf16* p;
    if (KC) {
      r = c >> 3; kk = (c & 7) * 8;
      ok = (row0 + r < rows) && (k0 + kk < K);
      p = base + (int64_t)(row0 + r) * ld + (k0 + kk);
    } else {
      kk = c >> 4; r = (c & 15) * 8;
      ok = (k0 + kk < K) && (row0 + r < rows);
      p = base + (int64_t)(k0 + kk) * ld + (row0 + r);
    }
    if (ok) st.v[i] = *reinterpret_cast<const bf16x8*>(p);
    else st.v[i] = bf16x8{};
  }
}

template <bool KC>
STE_DEV void stage_store(const Stage& st, char* tile, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int c = tid + NT * i;
    int off;
    if (KC) {
      int r = c >> 3, ch = c & 7;
      off = r * 128 + ((ch ^ (r & 7)) << 4);
    } else {
      int k = c >> 4, ch = c & 15;
      off = k * 256 + ((ch ^ km_chunk_xor(k)) << 4);
    }
    *reinterpret_cast<bf16x8*>(tile + off) = st.v[i];
  }
}
}  // namespace small

// fragment for mfma_f32_16x16x32_bf16: lane l holds X[row=rb+(l&15)][k=32s+8(l>>4)+j], j=0..7.
// KC image: [rows][64 k] (128 B rows, chunk ^ (row&7));  KM image: [64 k][ROWB bytes] (chunk ^ km_xor(k)).
template <bool KC, int KM_ROW_BYTES>
STE_DEV bf16x8 frag_load(const char* tile, int rb, int s, int lane) {
  if (KC) {
    int r = rb + (lane & 15);
    int ch = s * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(tile + r * 128 + ((ch ^ (r & 7)) << 4));
  } else {
    int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    int k = s * 32 + 8 * g + q;
    int quad = (rb >> 2) + p;
    int a0 = k * KM_ROW_BYTES + ((quad ^ (km_chunk_xor(k) << 1)) << 3);
    int k1 = k + 4;
    int a1 = k1 * KM_ROW_BYTES + ((quad ^ (km_chunk_xor(k1) << 1)) << 3);
    s16x4 lo = ds_read_tr16(tile + a0);
    s16x4 hi = ds_read_tr16(tile + a1);
    return join_tr(lo, hi);
  }
}

template <bool A_KC, bool B_KC>
__global__ __launch_bounds__(small::NT, 2) void gemm_bf16_kernel(ste_gemm_args p) {
  using namespace small;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // LDS_BYTES dynamic
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int num_m = (p.M + BM - 1) / BM, num_n = (p.N + BN - 1) / BN;
  int batch, tm, tn;
  map_tile(gridDim.x, num_m, num_n, batch, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const bf16* A = (const bf16*)p.A + (int64_t)batch * p.strideA;
  const bf16* B = (const bf16*)p.B + (int64_t)batch * p.strideB;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  Stage sa, sb;
  stage_load<A_KC>(sa, A, p.lda, m0, p.M, 0, p.K, tid);
  stage_load<B_KC>(sb, B, p.ldb, n0, p.N, 0, p.K, tid);
  stage_store<A_KC>(sa, smem, tid);
  stage_store<B_KC>(sb, smem + TILE_BYTES, tid);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      stage_load<A_KC>(sa, A, p.lda, m0, p.M, (kt + 1) * BK, p.K, tid);
      stage_load<B_KC>(sb, B, p.ldb, n0, p.N, (kt + 1) * BK, p.K, tid);
    }
    const char* ta = smem + cur * 2 * TILE_BYTES;
    const char* tb = ta + TILE_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag_load<A_KC, 256>(ta, wm * 64 + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag_load<B_KC, 256>(tb, wn * 64 + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(fa[i], fb[j], acc[i][j]);
    }
    if (more) {
      char* na = smem + (cur ^ 1) * 2 * TILE_BYTES;
      stage_store<A_KC>(sa, na, tid);
      stage_store<B_KC>(sb, na + TILE_BYTES, tid);
    }
    __syncthreads();
  }

  float* epi = reinterpret_cast<float*>(smem) + wave * 64 * EPI_LD;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        epi[(i * 16 + (lane >> 4) * 4 + r) * EPI_LD + j * 16 + (lane & 15)] = acc[i][j][r];
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  Csum csum = {};
  epilogue_tile(p, epi, 64, m0 + wm * 64, n0 + wn * 64, n0 + wn * 64 + 32, batch, lane, csum);
  if (p.colsum)
    colsum_flush(p, csum, n0 + wn * 64, n0 + wn * 64 + 32, batch, lane, ((int64_t)batch * num_m + tm) * 2 + wm);
}

// ================================================================= big kernel
namespace big {
constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
constexpr int TILE_BYTES = BM * BK * 2;        // 32 KiB per operand per stage
constexpr int STAGE_BYTES = 2 * TILE_BYTES;
constexpr int LDS_BYTES = 2 * STAGE_BYTES;     // 128 KiB: 2-deep ring
constexpr int EPI_ROWS = 32;                   // rows staged per epilogue pass per wave

// issue this wave's 4 global_load_lds pieces (1 KiB each) of one operand tile.
// KC tile [256 rows][64 k]: piece p = rows 8p..8p+7; lane L -> row 8p+L/8, chunk (L%8)^(L/8).
// KM tile [64 k][256 rows] (512 B k-rows): piece p = k-rows 2p,2p+1; lane L -> k-row 2p+L/32,
//   logical chunk (L%32) ^ km_xor(k-row).  Row indices past the operand are clamped (their
//   products only reach discarded outputs); K % 64 == 0 is required.
template <bool KC>
STE_DEV void issue_tile(const bf16* base, int64_t ld, int row0, int rows, int k0, char* tile, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = wave * 4 + i;
    const bf16* src;
    if (KC) {
      const int r = piece * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ (lane >> 3);
      const int gr = min(row0 + r, rows - 1);
      src = base + (int64_t)gr * ld + k0 + ch * 8;
    } else {
      const int kk = piece * 2 + (lane >> 5);
      const int ch = (lane & 31) ^ km_chunk_xor(kk);
      const int gc = min(row0 + ch * 8, rows - 8);
      src = base + (int64_t)(k0 + kk) * ld + gc;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(tile + piece * 1024), 16, 0, 0);
  }
}
}  // namespace big

template <bool A_KC, bool B_KC>
__global__ __launch_bounds__(big::NT, 2) void gemm_big_kernel(ste_gemm_args p) {
  using namespace big;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int num_m = (p.M + BM - 1) / BM, num_n = (p.N + BN - 1) / BN;
  int batch, tm, tn;
  map_tile(gridDim.x, num_m, num_n, batch, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const bf16* A = (const bf16*)p.A + (int64_t)batch * p.strideA;
  const bf16* B = (const bf16*)p.B + (int64_t)batch * p.strideB;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / BK;
  issue_tile<A_KC>(A, p.lda, m0, p.M, 0, smem, wave, lane);
  issue_tile<B_KC>(B, p.ldb, n0, p.N, 0, smem + TILE_BYTES, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      char* nxt = smem + (cur ^ 1) * STAGE_BYTES;
      issue_tile<A_KC>(A, p.lda, m0, p.M, (kt + 1) * BK, nxt, wave, lane);
      issue_tile<B_KC>(B, p.ldb, n0, p.N, (kt + 1) * BK, nxt + TILE_BYTES, wave, lane);
    }
    const char* ta = smem + cur * STAGE_BYTES;
    const char* tb = ta + TILE_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 fb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag_load<B_KC, 512>(tb, wn * 64 + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const bf16x8 fa = frag_load<A_KC, 512>(ta, wm * 128 + i * 16, s, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(fa, fb[j], acc[i][j]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: 4 passes of 32 rows x 64 cols per wave through LDS
  float* epi = reinterpret_cast<float*>(smem) + wave * EPI_ROWS * EPI_LD;
  Csum csum = {};
  // (explicit passes: a rolled pass loop would index acc dynamically and demote it to scratch)
#define STE_EPI_PASS(PS)                                                                                     \
  {                                                                                                          \
    for (int ii = 0; ii < 2; ++ii) {                                                                         \
      _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                                        \
        _Pragma("unroll") for (int r = 0; r < 4; ++r) {                                                      \
          epi[(ii * 16 + (lane >> 4) * 4 + r) * EPI_LD + j * 16 + (lane & 15)] = acc[2 * (PS) + ii][j][r];   \
        }                                                                                                    \
      }                                                                                                      \
    }                                                                                                        \
    __builtin_amdgcn_s_waitcnt(0xc07f);                                                                      \
    __builtin_amdgcn_wave_barrier();                                                                         \
    for (int hh = 0; hh < big::EPI_ROWS; hh += 16) {                                                         \
      if (!EPI_SKIP) epilogue_tile(p, epi + hh * EPI_LD, 16, m0 + wm * 128 + (PS) * big::EPI_ROWS + hh,     \
                                   EPI_COL0, EPI_COL1, batch, lane, csum);                                   \
    }                                                                                                        \
    __builtin_amdgcn_s_waitcnt(0xc07f);                                                                      \
    __builtin_amdgcn_wave_barrier();                                                                         \
  }
  constexpr bool EPI_SKIP = false;
#define EPI_COL0 (n0 + wn * 64)
#define EPI_COL1 (n0 + wn * 64 + 32)
  STE_EPI_PASS(0) STE_EPI_PASS(1) STE_EPI_PASS(2) STE_EPI_PASS(3)
#undef EPI_COL0
#undef EPI_COL1
  if (p.colsum)
    colsum_flush(p, csum, n0 + wn * 64, n0 + wn * 64 + 32, batch, lane, ((int64_t)batch * num_m + tm) * 2 + wm);
}

// ============================================================ 8-phase kernel
// Same 256x256x64 tile and 2(M)x4(N) waves as gemm_big, but each K-tile is split into
// four half-tiles (A rows / B cols that one C-quadrant of every wave needs) and the
// K-loop runs 4 phases per K-tile:
//   phase 0: read B-half0 + A-half0 -> MFMA quadrant (A0,B0)     stage B-half1 of tile t+1
//   phase 1: read B-half1           -> MFMA (A0,B1)              stage A-half1 of tile t+1
//   phase 2: read A-half1           -> MFMA (A1,B1)              stage A-half0 of tile t+2
//   phase 3: (registers)            -> MFMA (A1,B0)              stage B-half0 of tile t+2
// Every phase issues one half-tile of global_load_lds (2 per lane) and waits with a COUNTED
// vmcnt(8) (4 half-tiles stay in flight across the barriers, never drained in steady state),
// so HBM/L2 latency hides behind ~4 phases of MFMA.  Buffer safety (2 LDS buffers of 4
// half-tiles): a half-tile is restaged >= 2 phases after its last ds_read (its data then
// lives in registers), and read >= 1 phase after the wait+barrier that retires it.
namespace ph8 {
constexpr int NT = 512;
constexpr int HALF = 16384;                   // 128 rows x 64 k bf16
constexpr int BUF = 4 * HALF;                 // A0 | A1 | B0 | B1 of one K-tile
constexpr int RING_BYTES = 2 * BUF;           // 128 KiB operand ring
constexpr int EPI_OFF = RING_BYTES;            // 8 waves x [16][64] fp32 epilogue slots
constexpr int LDS_BYTES = EPI_OFF + 8 * 16 * 64 * 4;   // 160 KiB

// physical row pr (0..127) of half-tile h -> row of the 256-row tile.  A (G = 64): each
// 64-row group (one per wave row wm) holds that wave's h-th 64 rows.  B (G = 128): half h
// is the contiguous column range h*128.. (whole 256-B k-rows for the KM image); wave wn
// owns columns wn*32..+31 of each half.
template <int G>
STE_DEV int half_row(int pr, int h) {
  if (G == 128) return h * 128 + pr;
  return (pr / G) * (2 * G) + h * G + (pr % G);
}

// O32: the source as a 32-bit byte offset from the (wave-uniform) base, which the DMA takes as
// saddr + voffset: one VGPR per piece instead of a 64-bit pointer (operands < 4 GiB; the MX kernel,
// whose scale staging needs the registers)
template <bool KC, int G, bool O32 = false>
STE_DEV void stage_half(const bf16* base, int64_t ld, int row0, int rows, int k0, int h, char* dst, int wave,
                        int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int piece = wave * 2 + i;  // 1 KiB each, 16 per half-tile
    const bf16* src;
    if (KC) {  // image [128 rows][64 k], 128-B rows, chunk ^ (row & 7)
      const int pr = piece * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ (lane >> 3);
      const int gr = min(row0 + half_row<G>(pr, h), rows - 1);
      if (O32) src = (const bf16*)((const char*)base + (uint32_t)(((uint32_t)gr * (uint32_t)ld + k0 + ch * 8) * 2u));
      else src = base + (int64_t)gr * ld + k0 + ch * 8;
    } else {   // image [64 k][128 cols], 256-B k-rows, chunk ^ km_xor(k)
      const int kk = piece * 4 + (lane >> 4);
      const int lc = (lane & 15) ^ km_chunk_xor(kk);
      const int gc = min(row0 + half_row<G>(lc * 8, h), rows - 8);
      src = base + (int64_t)(k0 + kk) * ld + gc;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + piece * 1024), 16, 0, 0);
  }
}
// MX (e4m3 operands, K-tile = 128 fp8 = the same 128-B LDS rows as 64 bf16): the K-tile's scales,
// 4 bytes (k-blocks 0..3) per row, A then B, 2 KiB per stage in the epilogue-slot region (the MX
// kernel stages its epilogue in the ring's free K-tile-1 halves instead); one 4-B LDS-DMA piece per
// wave: waves 0-3 the A rows, 4-7 the B rows
constexpr int SC_OFF = EPI_OFF;
constexpr int SC_STAGE = 2048;
STE_DEV void stage_scales(const Mx8Args& mx, int m0, int M, int n0, int N, int t, char* smem, int wave, int lane) {
  const bool isb = wave >= 4;
  const int r = (wave & 3) * 64 + lane;
  const uint8_t* src = isb ? mx.sb + (uint32_t)(min(n0 + r, N - 1) * (uint32_t)mx.lsb + 4 * t)
                           : mx.sa + (uint32_t)(min(m0 + r, M - 1) * (uint32_t)mx.lsa + 4 * t);
  char* dst = smem + SC_OFF + (t & 1) * SC_STAGE + (isb ? 1024 : 0) + (wave & 3) * 256;
  __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)dst, 4, 0, 0);
}
// the scale bytes lane l feeds the MFMAs (its row l & 15 of each 16-row group, k-block l >> 4),
// two per register: ds_read_u8_d16 into bits 0-7, ds_read_u8_d16_hi into bits 16-23 (the MFMA's
// scale op_sel then picks byte 0 or 2).  asm reads: the caller waits lgkmcnt before the MFMAs.
template <int OFF>
STE_DEV void ds_u8_lo(int& r, uint32_t addr) {
  asm volatile("ds_read_u8_d16 %0, %1 offset:%2" : "+v"(r) : "v"(addr), "i"(OFF) : "memory");
}
template <int OFF>
STE_DEV void ds_u8_hi(int& r, uint32_t addr) {
  asm volatile("ds_read_u8_d16_hi %0, %1 offset:%2" : "+v"(r) : "v"(addr), "i"(OFF) : "memory");
}
template <int OFF>
STE_DEV void ds_u8(int& r, uint32_t addr) {
  asm volatile("ds_read_u8 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF) : "memory");
}
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4m __attribute__((ext_vector_type(4)));
// the MX operand of row rb + (l & 15): bytes k 16g..16g+15 and 64+16g.. of its swizzled 128-B row
// (g = l >> 4), straight into one 8-register tuple
STE_DEV i32x8 frag_mx(const char* tile, int rb, int lane) {
  const int r = rb + (lane & 15), g = lane >> 4;
  const i32x4m lo = *reinterpret_cast<const i32x4m*>(tile + r * 128 + ((g ^ (r & 7)) << 4));
  const i32x4m hi = *reinterpret_cast<const i32x4m*>(tile + r * 128 + (((g + 4) ^ (r & 7)) << 4));
  return i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
// f(integral_constant<int, I>) for I = 0..N-1 (compile-time indices for the MFMA's op_sel)
template <typename F, int... I>
STE_DEV void static_for_impl(F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
STE_DEV void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}
// scales: each in byte 0 of its own register (ds_read_u8), read with scale-select 0 — the form the
// single-stage kernel (and the lane/scale probe) uses.  Round 5: the first form packed two scales
// per register (ds_read_u8_d16 / _d16_hi) and picked byte 2 with the builtin's scale-select
// argument, which read a zero byte (a 2^-127 scale) for every odd row / column group: 3/4 of
// every tile came out ~0 since the kernel was added (profiles/r5q_mx8_bisect.txt, r5_mx8_diag.py).
// The six extra registers cost 9-26 spilled VGPRs in the MX instantiations; the kernel still runs
// the c5 fp8 step 2.7 % faster than the single-stage one (profiles/r5t_*)
template <int X, int Y>
STE_DEV f32x4 mfma_mx(const i32x8& x, const i32x8& y, f32x4 c, int sx, int sy) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(x, y, c, 0, 0, 0, sx, 0, sy);
}
}  // namespace ph8

#define STE_BARRIER() asm volatile("s_barrier" ::: "memory")
// MFMA-cluster priority: default raises it around every cluster; STE_PRIO_STATIC (experiment
// builds) instead gives the second-dispatched wave group (waves 4-7) a static priority of 1
#ifdef STE_PRIO_STATIC
#define STE_PRIO_HI()
#define STE_PRIO_LO()
#else
#define STE_PRIO_HI() __builtin_amdgcn_s_setprio(1)
#define STE_PRIO_LO() __builtin_amdgcn_s_setprio(0)
#endif
#define STE_VMCNT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

// KM fragment through inline-asm ds_read_b64_tr_b16.  The builtin form makes hipcc's
// waitcnt pass treat the read as aliasing every in-flight global_load_lds and emit
// vmcnt(0) before it, which drains the 8-phase pipeline; the asm form is invisible to that
// pass, so the kernel orders these reads itself (lgkmcnt(0) + sched_barrier before the
// MFMAs that consume them).
STE_DEV bf16x8 frag_load_km_asm(const char* tile, int rb, int s, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  const int k = s * 32 + 8 * g + q;
  const int quad = (rb >> 2) + pp;
  const int k1 = k + 4;
  const s16x4 lo = ds_read_tr16_asm(tile + k * 256 + ((quad ^ (km_chunk_xor(k) << 1)) << 3));
  const s16x4 hi = ds_read_tr16_asm(tile + k1 * 256 + ((quad ^ (km_chunk_xor(k1) << 1)) << 3));
  return join_tr(lo, hi);
}
template <bool B_KC>
STE_DEV bf16x8 frag_b_8ph(const char* tile, int rb, int s, int lane) {
  if (B_KC) return frag_load<true, 256>(tile, rb, s, lane);
  return frag_load_km_asm(tile, rb, s, lane);
}
template <bool A_KC>
STE_DEV bf16x8 frag_a_8ph(const char* tile, int rb, int s, int lane) {
  if (A_KC) return frag_load<true, 256>(tile, rb, s, lane);
  return frag_load_km_asm(tile, rb, s, lane);
}
// wait for this wave's LDS reads (incl. the asm ones) before the MFMA cluster
#define STE_LDS_SYNC(ASM)                               \
  do {                                                  \
    if (ASM) {                                          \
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
      __builtin_amdgcn_sched_barrier(0);                \
    }                                                   \
  } while (0)

// A_KC=false (A k-major, the weight-gradient dYᵀ operand) stages A like a KM B operand and
// reads it through ds_read_b64_tr_b16; everything else is shared.
//
// Persistent: a grid of min(tiles, CUs) workgroups loops over virtual tiles
// vb = blockIdx.x, +gridDim.x, ... (same XCD-aware order as one tile per workgroup).
// Tile hand-over: the next tile's prologue (K-tile 0 + half of K-tile 1, into the operand
// ring) is issued right after the main loop, BEFORE this tile's epilogue, which stages
// through its own 32 KiB LDS slots.  The next tile's first vmcnt waits then allow for the
// epilogue's global stores still in flight (exactly epi_stores<EF>() of them on a FULL
// tile; 0 = drain everything otherwise), so those stores drain under the next tile's MFMAs
// instead of stalling its first operand wait.  EF/ACT: compile-time epilogue.
// bias of this lane's 8 epilogue columns (fp32; zeros past N)
STE_DEV f32x8 tile_bias(const ste_gemm_args& p, int n0, int wn, int lane) {
  const int cl = (lane & 7) * 8;
  const int col = cl < 32 ? n0 + wn * 32 + cl : n0 + 128 + wn * 32 + (cl - 32);
  const int nval = p.N - col;
  return nval > 0 ? ld8(p.bias + col, false, nval >= 8, nval) : f32x8{};
}

// acc[i][j] = rows wm*128 + i*16, cols (j >> 1)*128 + wn*32 + (j & 1)*16: 8 passes of
// 16 rows x 64 columns through the wave's own LDS slot; straight-line code per FULL value.
template <int EF, int ACT, bool FULL>
STE_DEV void epilogue_8ph(const ste_gemm_args& p, const f32x4 (&acc)[8][4], float* epi, int m0, int n0, int batch,
                          int wm, int wn, int lane, f32x8 bias, const Q8Out* q8 = nullptr) {
  Csum csum = {};
  const int c0 = n0 + wn * 32, c1 = n0 + 128 + wn * 32;
#define STE_EPI_STAGE(PS)                                                                       \
  {                                                                                             \
    _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                             \
      _Pragma("unroll") for (int r = 0; r < 4; ++r) {                                           \
        const int row = (lane >> 4) * 4 + r, chunk = (4 * j + ((lane & 15) >> 2)) ^ ((r >> 1) & 1); \
        epi[row * 64 + chunk * 4 + (lane & 3)] = acc[PS][j][r];                                 \
      }                                                                                         \
    }                                                                                           \
    __builtin_amdgcn_s_waitcnt(0xc07f);                                                         \
    __builtin_amdgcn_wave_barrier();                                                            \
  }
#define STE_EPI_ROW0(PS) (m0 + wm * 128 + (PS) * 16)
#define STE_EPI_LOAD(PS, L) epi_load16<EF, ACT, FULL>(p, STE_EPI_ROW0(PS), c0, c1, batch, lane, L);
#define STE_EPI_STORE(PS, L)                                                                    \
  epi_store16<EF, ACT, FULL>(p, epi, STE_EPI_ROW0(PS), c0, c1, batch, lane, bias, L, csum, q8); \
  __builtin_amdgcn_s_waitcnt(0xc07f);                                                           \
  __builtin_amdgcn_wave_barrier();
  if constexpr (EF < 0) {
#define STE_EPI_G(PS)                                                                           \
    STE_EPI_STAGE(PS)                                                                           \
    epilogue_tile(p, epi, 16, STE_EPI_ROW0(PS), c0, c1, batch, lane, csum, 64, true, q8);       \
    __builtin_amdgcn_s_waitcnt(0xc07f);                                                         \
    __builtin_amdgcn_wave_barrier();
    STE_EPI_G(0) STE_EPI_G(1) STE_EPI_G(2) STE_EPI_G(3) STE_EPI_G(4) STE_EPI_G(5) STE_EPI_G(6) STE_EPI_G(7)
#undef STE_EPI_G
  } else {
    EpiLoads L0, L1;
    STE_EPI_LOAD(0, L0)
    STE_EPI_STAGE(0) STE_EPI_LOAD(1, L1) STE_EPI_STORE(0, L0)
    STE_EPI_STAGE(1) STE_EPI_LOAD(2, L0) STE_EPI_STORE(1, L1)
    STE_EPI_STAGE(2) STE_EPI_LOAD(3, L1) STE_EPI_STORE(2, L0)
    STE_EPI_STAGE(3) STE_EPI_LOAD(4, L0) STE_EPI_STORE(3, L1)
    STE_EPI_STAGE(4) STE_EPI_LOAD(5, L1) STE_EPI_STORE(4, L0)
    STE_EPI_STAGE(5) STE_EPI_LOAD(6, L0) STE_EPI_STORE(5, L1)
    STE_EPI_STAGE(6) STE_EPI_LOAD(7, L1) STE_EPI_STORE(6, L0)
    STE_EPI_STAGE(7) STE_EPI_STORE(7, L1)
  }
#undef STE_EPI_STAGE
#undef STE_EPI_ROW0
#undef STE_EPI_LOAD
#undef STE_EPI_STORE
  if (EF < 0 ? p.colsum != nullptr : (EF & EF_COLSUM) != 0)
    colsum_flush(p, csum, c0, c1, batch, lane, ((int64_t)batch * ((p.M + 255) >> 8) + (m0 >> 8)) * 2 + wm);
}

// The epilogue of an operand-loading (Z or R) compile-time epilogue on a full tile, with the next
// tile's prologue DMA issued after the first two passes' loads: those loads are older than the DMA
// (vmcnt counts in issue order), so they land without waiting for it, and every later pass's loads
// are issued two passes ahead, after the DMA.  All of this tile's stores then follow the
// prologue, so the next tile's first waits may leave them in flight (epi_stores<EF>(), as the
// load-free EPI_OVL epilogues do) and they drain under its first K-tiles; the DMA latency hides
// under the epilogue instead of following it.
#ifndef STE_EPI_PRE
#define STE_EPI_PRE 1
#endif
template <int EF, int ACT, class Pro>
STE_DEV void epilogue_8ph_pre(const ste_gemm_args& p, const f32x4 (&acc)[8][4], float* epi, int m0, int n0, int batch,
                              int wm, int wn, int lane, f32x8 bias, Pro&& prologue) {
  static_assert(EF >= 0 && (EF & (EF_COLSUM | EF_BETA | EF_RS | EF_Q8)) == 0, "EPI_PRE epilogues");
  Csum csum = {};
  const int c0 = n0 + wn * 32, c1 = n0 + 128 + wn * 32;
#define STE_EPI_STAGE(PS)                                                                       \
  {                                                                                             \
    _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                             \
      _Pragma("unroll") for (int r = 0; r < 4; ++r) {                                           \
        const int row = (lane >> 4) * 4 + r, chunk = (4 * j + ((lane & 15) >> 2)) ^ ((r >> 1) & 1); \
        epi[row * 64 + chunk * 4 + (lane & 3)] = acc[PS][j][r];                                 \
      }                                                                                         \
    }                                                                                           \
    __builtin_amdgcn_s_waitcnt(0xc07f);                                                         \
    __builtin_amdgcn_wave_barrier();                                                            \
  }
#define STE_EPI_ROW0(PS) (m0 + wm * 128 + (PS) * 16)
#define STE_EPI_LOAD(PS, L) epi_load16<EF, ACT, true>(p, STE_EPI_ROW0(PS), c0, c1, batch, lane, L);
#define STE_EPI_STORE(PS, L)                                                                    \
  epi_store16<EF, ACT, true>(p, epi, STE_EPI_ROW0(PS), c0, c1, batch, lane, bias, L, csum);     \
  __builtin_amdgcn_s_waitcnt(0xc07f);                                                           \
  __builtin_amdgcn_wave_barrier();
  EpiLoads L0, L1;
  STE_EPI_LOAD(0, L0) STE_EPI_LOAD(1, L1)
  prologue();
  STE_EPI_STAGE(0) STE_EPI_STORE(0, L0) STE_EPI_LOAD(2, L0)
  STE_EPI_STAGE(1) STE_EPI_STORE(1, L1) STE_EPI_LOAD(3, L1)
  STE_EPI_STAGE(2) STE_EPI_STORE(2, L0) STE_EPI_LOAD(4, L0)
  STE_EPI_STAGE(3) STE_EPI_STORE(3, L1) STE_EPI_LOAD(5, L1)
  STE_EPI_STAGE(4) STE_EPI_STORE(4, L0) STE_EPI_LOAD(6, L0)
  STE_EPI_STAGE(5) STE_EPI_STORE(5, L1) STE_EPI_LOAD(7, L1)
  STE_EPI_STAGE(6) STE_EPI_STORE(6, L0)
  STE_EPI_STAGE(7) STE_EPI_STORE(7, L1)
#undef STE_EPI_STAGE
#undef STE_EPI_ROW0
#undef STE_EPI_LOAD
#undef STE_EPI_STORE
}

// steady-state operand wait: W pieces stay in flight (4 half-tiles = 8; MX adds the K-tile's scale
// piece, issued with A-half 0, so 9), plus the previous tile's epilogue stores still draining
// (capped at the 6-bit vmcnt field: waiting for a few more of those stores is merely early)
template <int W, int E>
STE_DEV void vm_wait8(int extra) {
  constexpr int WE = W + E < 63 ? W + E : 63;
  if (E > 0 && extra) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WE) : "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W) : "memory");
}

// Operands of batch entry `batch` and its K-tile count.  Split-K slab launches (ste_gemm's
// weight-gradient plan, A_KC = B_KC = false, and the few-tile epilogue plan, k-contiguous; batch = slab) mark themselves with ws_bytes =
// -(rem + 1), a field the kernel never reads otherwise: the K/64 - S·Kc K-tiles that do not
// divide over the S slabs go one each to slabs 0..rem-1 (slab s starts at K-tile
// s·Kc + min(s, rem)), so no remainder launch is needed.
template <bool A_KC, bool B_KC>
STE_DEV void operand_bases(const ste_gemm_args& p, int batch, const bf16*& A, const bf16*& B, int& nk) {
  if (p.ws_bytes < 0) {
    const int kc = p.K / 64, rem = (int)(-p.ws_bytes - 1);
    const int64_t k0 = ((int64_t)batch * kc + (batch < rem ? batch : rem)) * 64;
    A = (const bf16*)p.A + k0 * (A_KC ? 1 : p.lda);
    B = (const bf16*)p.B + k0 * (B_KC ? 1 : p.ldb);
    nk = kc + (batch < rem ? 1 : 0);
    return;
  }
  A = (const bf16*)p.A + (int64_t)batch * p.strideA;
  B = (const bf16*)p.B + (int64_t)batch * p.strideB;
  nk = p.K / 64;
}

// MX: e4m3 operands (A_KC = B_KC = true), the kernel arguments in bf16 units (K, lda, ldb halved:
// two fp8 per bf16 slot), scales and the optional fp8 output copy in mx.
template <bool A_KC, bool B_KC, int EF, int ACT, bool MX = false>
__global__ __launch_bounds__(ph8::NT, 1) void gemm_8ph_kernel(ste_gemm_args p, Mx8Args mx) {
  using namespace ph8;
  constexpr int E_ST = epi_stores<EF>();
  constexpr bool SW = epi_bf16s<EF>();  // swapped MFMA operands + bf16-staged epilogue
  constexpr int VW = MX ? 9 : 8;
  static_assert(!MX || (A_KC && B_KC), "MX operands are k-contiguous");
  static_assert(VW <= 63, "vmcnt immediate");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int num_m = (p.M + 255) / 256, num_n = (p.N + 255) / 256;
  const int total = num_m * num_n * p.batch;
  int nk = p.K / 64;
  int vb = blockIdx.x;
  if (vb >= total) return;
  int batch, tm, tn;
  map_tile_bid(xcd_remap(vb, total), num_m, num_n, batch, tm, tn);
  int m0 = tm * 256, n0 = tn * 256;
  const bf16* A;
  const bf16* B;
  operand_bases<A_KC, B_KC>(p, batch, A, B, nk);
#define STAGE_A(t, h) \
  stage_half<A_KC, 64, MX>(A, p.lda, m0, p.M, (t) * 64, h, smem + ((t) & 1) * BUF + (h) * HALF, wave, lane)
#define STAGE_B(t, h) \
  stage_half<B_KC, 128, MX>(B, p.ldb, n0, p.N, (t) * 64, h, smem + ((t) & 1) * BUF + (2 + (h)) * HALF, wave, lane)
#define STAGE_S(t) \
  if constexpr (MX) stage_scales(mx, m0, p.M, n0, p.N, (t), smem, wave, lane)
#define STAGE_PROLOGUE()                                                    \
  {                                                                         \
    STAGE_A(0, 0); STAGE_S(0); STAGE_B(0, 0); STAGE_B(0, 1); STAGE_A(0, 1); \
    if (nk > 1) { STAGE_A(1, 0); STAGE_S(1); STAGE_B(1, 0); }               \
  }
  // prologue of the first tile: tile 0 complete, tile 1's A0/B0 (phases (-1,*) of the steady state)
  STAGE_PROLOGUE();
  int extra = 0;  // stores of the previous tile's epilogue issued after this prologue (FULL tiles)
  // MX: the epilogue-slot region holds the scale stages; the epilogue stages through ring buffer 1's
  // A1 / B1 halves instead, which no DMA touches between the main loop and the next tile's phase 0
  char* const epi_base = MX ? smem + BUF + (wave < 4 ? HALF : 3 * HALF) + (wave & 3) * EPI16_FLOATS * 4
                            : smem + EPI_OFF + wave * EPI16_FLOATS * 4;
  float* epi = reinterpret_cast<float*>(epi_base);
  constexpr bool EPI_OVL = EF >= 0 && (EF & (EF_Z | EF_R | EF_BETA | EF_COLSUM | EF_RS)) == 0;
  // operand-loading epilogues (residual adds, activation backward x Z): the prologue DMA goes out
  // behind the first two passes' loads (epilogue_8ph_pre); A/B builds: -DSTE_EPI_PRE=0
  constexpr bool EPI_PRE_OK = EF >= 0 && !EPI_OVL && !MX && !SW && (EF & (EF_Z | EF_R)) != 0 &&
                              (EF & (EF_BETA | EF_COLSUM | EF_RS | EF_Q8 | EF_DROP)) == 0;   // DROP: spills
  constexpr bool epi_pre = EPI_PRE_OK && STE_EPI_PRE;
  f32x8 bias = f32x8{};
  f32x4 sbias[4] = {};
  // the tile's bias preloaded across the main loop — except MX, whose main loop needs the registers
  // (loaded at the epilogue instead)
  if constexpr (EF >= 0 && (EF & EF_BIAS) != 0 && !MX) {
    if constexpr (SW) swap_bias(p, n0, wn, lane, sbias);
    else bias = tile_bias(p, n0, wn, lane);
  }

  for (;;) {
    if (nk > 1) vm_wait8<VW, E_ST>(extra);
    else STE_VMCNT(0);
    STE_BARRIER();

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    bf16x8 a0[4][2], a1[4][2], b0[2][2], b1[2][2];
    i32x8 ma0[MX ? 4 : 1], ma1[MX ? 4 : 1], mb0[MX ? 2 : 1], mb1[MX ? 2 : 1];
    // Ping-pong: waves 4-7 run one barrier behind waves 0-3, so on every SIMD (one wave of
    // each group) one wave's MFMA cluster overlaps the other's ds_reads + staging.  Buffer
    // safety holds with the extra barrier of skew (reads stay >= 1 phase after the retiring
    // wait+barrier of every producer, restaging >= 2 phases after the last read).
    if (wm == 1) STE_BARRIER();
#ifdef STE_PRIO_STATIC
    if (wm == 1) __builtin_amdgcn_s_setprio(1);
#endif
    for (int t = 0; t < nk; ++t) {
      const char* buf = smem + (t & 1) * BUF;
      const bool tail = t + 2 >= nk;  // fewer stages in flight: drain fully instead of counting
      const int ex = t == 0 ? extra : 0;
      // MX: the K-tile's 12 scale bytes of this lane in 6 registers, read with phase 0's fragments
      // (S(t) is staged with A-half 0 of K-tile t and retired by the same waits): sca[i >> 1] holds
      // A row group i (rows wm*128 + 16i..), scb[j >> 1] B column group j
      int sca[8] = {0, 0, 0, 0, 0, 0, 0, 0}, scb[4] = {0, 0, 0, 0};
      if constexpr (MX) {
        typedef __attribute__((address_space(3))) char lds_char_t;
        // the lane id regenerated (mbcnt) behind an opaque copy each K-tile: the addresses are rebuilt
        // (a few VALU) instead of being hoisted out of the loop and spilled (a scratch reload inside
        // the loop makes hipcc drain the counted DMA pipeline with vmcnt(0))
        int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        asm volatile("" : "+v"(ln));
        const uint32_t sbase = (uint32_t)(uintptr_t)(lds_char_t*)smem + SC_OFF + (t & 1) * SC_STAGE + (ln >> 4) +
                               (ln & 15) * 4;
        const uint32_t aa = sbase + wm * 512, ab = sbase + 1024 + wn * 128;
        ds_u8<0>(sca[0], aa);    ds_u8<64>(sca[1], aa);
        ds_u8<128>(sca[2], aa);  ds_u8<192>(sca[3], aa);
        ds_u8<256>(sca[4], aa);  ds_u8<320>(sca[5], aa);
        ds_u8<384>(sca[6], aa);  ds_u8<448>(sca[7], aa);
        ds_u8<0>(scb[0], ab);    ds_u8<64>(scb[1], ab);
        ds_u8<512>(scb[2], ab);  ds_u8<576>(scb[3], ab);
      }
      // ---- phase 0
      if constexpr (MX) {
#pragma unroll
        for (int j = 0; j < 2; ++j) mb0[j] = frag_mx(buf + 2 * HALF, wn * 32 + j * 16, lane);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 4; ++i) ma0[i] = frag_mx(buf, wm * 64 + i * 16, lane);
      } else {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) b0[j][s] = frag_b_8ph<B_KC>(buf + 2 * HALF, wn * 32 + j * 16, s, lane);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int s = 0; s < 2; ++s) a0[i][s] = frag_a_8ph<A_KC>(buf, wm * 64 + i * 16, s, lane);
      }
      if (t + 1 < nk) STAGE_B(t + 1, 1);
      if (tail) STE_VMCNT(0); else vm_wait8<VW, E_ST>(ex);
      STE_BARRIER();
      STE_LDS_SYNC(!A_KC || !B_KC || MX);   // MX: the asm scale reads
      STE_PRIO_HI();
      if constexpr (MX) {
        static_for<4>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          static_for<2>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            acc[i][j] = SW ? mfma_mx<j, i>(mb0[j], ma0[i], acc[i][j], scb[j], sca[i])
                           : mfma_mx<i, j>(ma0[i], mb0[j], acc[i][j], sca[i], scb[j]);
          });
        });
      } else {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = SW ? mfma16(b0[j][s], a0[i][s], acc[i][j]) : mfma16(a0[i][s], b0[j][s], acc[i][j]);
      }
      STE_PRIO_LO();
      STE_BARRIER();
      // ---- phase 1
      if constexpr (MX) {
#pragma unroll
        for (int j = 0; j < 2; ++j) mb1[j] = frag_mx(buf + 3 * HALF, wn * 32 + j * 16, lane);
      } else {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) b1[j][s] = frag_b_8ph<B_KC>(buf + 3 * HALF, wn * 32 + j * 16, s, lane);
      }
      if (t + 1 < nk) STAGE_A(t + 1, 1);
      if (tail) STE_VMCNT(0); else vm_wait8<VW, E_ST>(ex);
      STE_BARRIER();
      STE_LDS_SYNC(!B_KC);
      STE_PRIO_HI();
      if constexpr (MX) {
        static_for<4>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          static_for<2>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            acc[i][2 + j] = SW ? mfma_mx<j, i>(mb1[j], ma0[i], acc[i][2 + j], scb[2 + j], sca[i])
                               : mfma_mx<i, j>(ma0[i], mb1[j], acc[i][2 + j], sca[i], scb[2 + j]);
          });
        });
      } else {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][2 + j] = SW ? mfma16(b1[j][s], a0[i][s], acc[i][2 + j]) : mfma16(a0[i][s], b1[j][s], acc[i][2 + j]);
      }
      STE_PRIO_LO();
      STE_BARRIER();
      // ---- phase 2
      if constexpr (MX) {
#pragma unroll
        for (int i = 0; i < 4; ++i) ma1[i] = frag_mx(buf + HALF, wm * 64 + i * 16, lane);
      } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int s = 0; s < 2; ++s) a1[i][s] = frag_a_8ph<A_KC>(buf + HALF, wm * 64 + i * 16, s, lane);
      }
      if (t + 2 < nk) {
        STAGE_A(t + 2, 0);
        STAGE_S(t + 2);
      }
      STE_BARRIER();
      STE_LDS_SYNC(!A_KC);
      STE_PRIO_HI();
      if constexpr (MX) {
        static_for<4>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          static_for<2>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            acc[4 + i][2 + j] = SW ? mfma_mx<j, i>(mb1[j], ma1[i], acc[4 + i][2 + j], scb[2 + j], sca[4 + i])
                                   : mfma_mx<i, j>(ma1[i], mb1[j], acc[4 + i][2 + j], sca[4 + i], scb[2 + j]);
          });
        });
      } else {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[4 + i][2 + j] = SW ? mfma16(b1[j][s], a1[i][s], acc[4 + i][2 + j]) : mfma16(a1[i][s], b1[j][s], acc[4 + i][2 + j]);
      }
      STE_PRIO_LO();
      STE_BARRIER();
      // ---- phase 3
      if (t + 2 < nk) STAGE_B(t + 2, 0);
      if (tail) STE_VMCNT(0); else vm_wait8<VW, E_ST>(ex);
      STE_BARRIER();
      STE_PRIO_HI();
      if constexpr (MX) {
        static_for<4>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          static_for<2>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            acc[4 + i][j] = SW ? mfma_mx<j, i>(mb0[j], ma1[i], acc[4 + i][j], scb[j], sca[4 + i])
                               : mfma_mx<i, j>(ma1[i], mb0[j], acc[4 + i][j], sca[4 + i], scb[j]);
          });
        });
      } else {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[4 + i][j] = SW ? mfma16(b0[j][s], a1[i][s], acc[4 + i][j]) : mfma16(a1[i][s], b0[j][s], acc[4 + i][j]);
      }
      STE_PRIO_LO();
      STE_BARRIER();
    }
    if (wm == 0) STE_BARRIER();  // re-align the groups (equal barrier counts): every ring read is done

    // ---- hand-over to the next tile.  Load-free epilogues (EPI_OVL) issue the next tile's
    // prologue first and let their stores drain under its first K-tile; epilogues that read
    // Z / R / beta*C run first (their loads must not queue behind the prologue's DMA).
    const int em0 = m0, en0 = n0, ebatch = batch;
    const int vb_next = vb + gridDim.x;
    const bool more = vb_next < total;
    const bool full_tile = em0 + 256 <= p.M && en0 + 256 <= p.N;
    if constexpr (EF >= 0 && (EF & EF_BIAS) != 0 && MX) {
      // this tile's bias, issued before the next prologue's DMA (the compiler counts that DMA in the
      // wait it places before the bias's first use)
      if constexpr (SW) swap_bias(p, en0, wn, lane, sbias);
      else bias = tile_bias(p, en0, wn, lane);
    } else {
      asm volatile("" : "+v"(bias));  // bias landed long ago (the main loop drained vmcnt): no waits below
    }
    if constexpr (SW && (EF & EF_BIAS) != 0 && !MX) {
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(sbias[j]));
    }
    auto next_prologue = [&]() {
      if (more) {
        map_tile_bid(xcd_remap(vb_next, total), num_m, num_n, batch, tm, tn);
        m0 = tm * 256;
        n0 = tn * 256;
        operand_bases<A_KC, B_KC>(p, batch, A, B, nk);
        STAGE_PROLOGUE();
      }
    };
    if (EPI_OVL) next_prologue();
    bool pro_done = EPI_OVL;
    if constexpr (SW) {
      char* slot = epi_base;
      if (full_tile) epilogue_bf16s<EF, ACT, true>(p, acc, slot, em0, en0, ebatch, wm, wn, lane, sbias);
      else epilogue_bf16s<EF, ACT, false>(p, acc, slot, em0, en0, ebatch, wm, wn, lane, sbias);
    } else {
      const Q8Out* q8 = MX && mx.q8.q ? &mx.q8 : nullptr;
      if constexpr (EPI_PRE_OK) {
        if (full_tile && epi_pre) {
          epilogue_8ph_pre<EF, ACT>(p, acc, epi, em0, en0, ebatch, wm, wn, lane, bias, next_prologue);
          pro_done = true;
        } else if (full_tile) {
          epilogue_8ph<EF, ACT, true>(p, acc, epi, em0, en0, ebatch, wm, wn, lane, bias, q8);
        } else {
          epilogue_8ph<EF, ACT, false>(p, acc, epi, em0, en0, ebatch, wm, wn, lane, bias, q8);
        }
      } else {
        if (full_tile) epilogue_8ph<EF, ACT, true>(p, acc, epi, em0, en0, ebatch, wm, wn, lane, bias, q8);
        else epilogue_8ph<EF, ACT, false>(p, acc, epi, em0, en0, ebatch, wm, wn, lane, bias, q8);
      }
    }
    if (!pro_done) next_prologue();
    if (!more) break;
    vb = vb_next;
    extra = ((EPI_OVL || (EPI_PRE_OK && epi_pre)) && full_tile) ? 1 : 0;
    if constexpr (EF >= 0 && (EF & EF_BIAS) != 0 && !MX) {
      if constexpr (SW) swap_bias(p, n0, wn, lane, sbias);
      else bias = tile_bias(p, n0, wn, lane);
    }
  }
#undef STAGE_A
#undef STAGE_B
#undef STAGE_S
#undef STAGE_PROLOGUE
#undef STE_LDS_SYNC
}
#undef STE_EPI_PASS

// CUs of the current device (one persistent workgroup each)
int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0, v = 0;
    n = (hipGetDevice(&dev) == hipSuccess &&
         hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
  }
  return n;
}

// (A_KC, B_KC, epilogue flags, activation) instantiated with a compile-time epilogue; every
// other combination runs the EF_GENERIC instantiation of the same kernel.
#define STE_EPI_SPECS(X)                                                              \
  X(true, true, EF_BIAS | EF_C2 | EF_CBF16, STE_ACT_SWISH)   /* FFN intermediate   */ \
  X(true, true, EF_BIAS | EF_C2 | EF_CBF16, STE_ACT_GELU)    /* XLM-R intermediate */ \
  X(true, true, EF_BIAS | EF_CBF16, STE_ACT_SWISH)           /* FFN in, no backward */ \
  X(true, true, EF_C2 | EF_CBF16, STE_ACT_GELU)              /* wav2vec2 conv layer */ \
  X(true, true, EF_C2, STE_ACT_GELU)                         /* wav2vec2 last conv  */ \
  X(true, true, EF_BIAS | EF_R | EF_DROP, STE_ACT_NONE)      /* post-LN O-proj / FFN out + dropout */ \
  X(true, true, EF_BIAS | EF_C2 | EF_DROP | EF_CBF16, STE_ACT_GELU) /* wav2vec2 FFN in + act dropout */ \
  X(true, true, EF_BIAS | EF_CBF16, STE_ACT_GELU)                                     \
  X(true, true, EF_BIAS | EF_C3, STE_ACT_NONE)               /* precise text QKV: fp32 + bf16 copy */ \
  X(true, true, EF_BIAS | EF_C2 | EF_C3 | EF_CBF16, STE_ACT_GELU) /* precise text FFN in: h, h_lo, z */ \
  X(true, true, EF_BIAS | EF_R, STE_ACT_NONE)                /* FFN out, O-proj    */ \
  X(true, true, EF_BIAS | EF_CBF16, STE_ACT_NONE)            /* QKV                */ \
  X(true, true, EF_CBF16, STE_ACT_NONE)                      /* pointwise conv 1   */ \
  X(true, true, EF_R | EF_DROP, STE_ACT_NONE)                /* pointwise conv 2   */ \
  X(true, true, EF_R, STE_ACT_NONE)                                                   \
  X(true, false, EF_CBF16, STE_ACT_NONE)                     /* dX, bf16 out       */ \
  X(true, false, 0, STE_ACT_NONE)                            /* dX, fp32 out       */ \
  X(true, true, EF_Z | EF_COLSUM | EF_CBF16, STE_ACT_SWISH_BWD) /* dz = dh·W ⊙ act'(z), Wᵀ copy */ \
  X(true, true, EF_Z | EF_COLSUM | EF_CBF16, STE_ACT_GELU_BWD)                        \
  X(true, true, EF_Z | EF_COLSUM | EF_C3 | EF_CBF16, STE_ACT_GELU_BWD) /* precise text dz: dz, dz_lo */ \
  X(true, true, EF_Z | EF_C3 | EF_CBF16, STE_ACT_GELU_BWD)            /* ... frozen layer        */ \
  X(true, true, EF_Z | EF_CBF16, STE_ACT_SWISH_BWD)          /* frozen layer: no db */ \
  X(true, true, EF_Z | EF_CBF16, STE_ACT_GELU_BWD)                                    \
  X(true, true, EF_Z | EF_COLSUM | EF_DROP | EF_CBF16, STE_ACT_GELU_BWD) /* wav2vec2 act dropout */ \
  X(true, true, EF_Z | EF_DROP | EF_CBF16, STE_ACT_GELU_BWD) /* frozen wav2vec2 layer, act dropout */ \
  X(true, true, 0, STE_ACT_NONE)                             /* few-tile split-K slabs */ \
  X(false, false, 0, STE_ACT_NONE)                           /* dW split-K slabs   */

template <bool A_KC, bool B_KC>
int launch_8ph(const ste_gemm_args& a, hipStream_t s) {
  const int nb = ((a.M + 255) / 256) * ((a.N + 255) / 256) * a.batch;
  const int grid = nb < num_cus() ? nb : num_cus();
  const int ef = epi_flags(a);
#define STE_TRY(AK, BK, E, ACT)                                                                       \
  if constexpr (AK == A_KC && BK == B_KC) {                                                           \
    if (ef == (E) && a.act == (ACT)) {                                                                \
      hipLaunchKernelGGL((gemm_8ph_kernel<A_KC, B_KC, (E), (ACT)>), dim3(grid), dim3(ph8::NT),        \
                         ph8::LDS_BYTES, s, a, Mx8Args{});                                            \
      STE_CHECK_LAUNCH();                                                                             \
      return 0;                                                                                       \
    }                                                                                                 \
  }
  STE_EPI_SPECS(STE_TRY)
#undef STE_TRY
  hipLaunchKernelGGL((gemm_8ph_kernel<A_KC, B_KC, EF_GENERIC, 0>), dim3(grid), dim3(ph8::NT), ph8::LDS_BYTES, s, a,
                     Mx8Args{});
  STE_CHECK_LAUNCH();
  return 0;
}

// C = beta*C + alpha*sum_s ws[s]  (fp32 [M,N] slabs): one thread per 4 columns over the whole
// output, its MAXS slab loads (clamped to the last slab past S) issued together with C's, then
// summed in slab order (run-to-run identical); S > MAXS (MAXS = 16) continues in a loop.
template <int MAXS>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(float* __restrict__ C, int64_t ldc,
                                                            const float* __restrict__ ws, int M, int N, int S,
                                                            float alpha, float beta) {
  const int n4 = N >> 2;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)M * n4) return;
  const int64_t slab = (int64_t)M * N;
  const int m = (int)(i / n4), c = (int)(i - (int64_t)m * n4) * 4;
  const float* w = ws + (int64_t)m * N + c;
  float* cp = C + (int64_t)m * ldc + c;
  f32x4 v[MAXS];
#pragma unroll
  for (int k = 0; k < MAXS; ++k) v[k] = *reinterpret_cast<const f32x4*>(w + (k < S ? k : S - 1) * slab);
  const f32x4 cv = beta != 0.f ? *reinterpret_cast<const f32x4*>(cp) : f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc = v[0];
#pragma unroll
  for (int k = 1; k < MAXS; ++k)
    if (k < S) acc += v[k];
  for (int k = MAXS; k < S; ++k) acc += *reinterpret_cast<const f32x4*>(w + k * slab);
  f32x4 out = acc * alpha;
  if (beta != 0.f) out += cv * beta;
  *reinterpret_cast<f32x4*>(cp) = out;
}

// Few-tile split-K: C = epilogue(sum_s ws[s]) for the forward / input-gradient GEMMs whose
// output is too narrow to fill the CUs with 256x256 tiles (the text encoder's N = 768 outputs
// at M = 8,192: 96 tiles).  The slabs are summed in slab order (run-to-run identical) and the
// generic epilogue (bias, activation, Z, dropout, row scale, residual, beta, C2 / C3) applied
// per 8 columns, exactly as the tile epilogue would.  No column sums (plan excludes them).
__global__ __launch_bounds__(256) void splitk_epi_kernel(ste_gemm_args p, const float* __restrict__ ws, int S) {
  const int n8 = p.N >> 3;
  const int64_t total = (int64_t)p.M * n8;
  const int64_t slab = (int64_t)p.M * p.N;
  const uint32_t thresh = (uint32_t)(p.drop_p * 4294967296.0);
  const float inv_keep = p.drop_p > 0.f ? 1.0f / (1.0f - p.drop_p) : 1.0f;
  Csum csum = {};   // unused: the plan excludes column sums
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int row = (int)(i / n8), col = (int)(i - (int64_t)row * n8) * 8;
    const float* w = ws + (int64_t)row * p.N + col;
    f32x4 lo = *reinterpret_cast<const f32x4*>(w), hi = *reinterpret_cast<const f32x4*>(w + 4);
    for (int k = 1; k < S; ++k) {
      lo += *reinterpret_cast<const f32x4*>(w + k * slab);
      hi += *reinterpret_cast<const f32x4*>(w + k * slab + 4);
    }
    const f32x8 bias = p.bias ? ld8(p.bias + col, false, true, 8) : f32x8{};
    epi_apply8(p, f32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]}, row, col, true, 8, bias, thresh,
               inv_keep, 0, 0, csum, nullptr, 0);
  }
}

// Few-tile plan: k-contiguous operands, one output image, no column sums, N % 8 == 0, K a
// multiple of 64 with >= 40 K-tiles (at 36 — the text QKV input gradient — the split only broke
// even in isolation and its 2 x 25 MB of slabs still cost HBM time beside the audio stream), fewer 256x256 tiles than CUs / 2: S = 2
// slabs (2 x tiles workgroups).  STE_GEMM_FEW_SPLIT=0 disables it (A/B).
int few_split(const ste_gemm_args& a) {
  static int on = -1;
  if (on < 0) {
    const char* e = STE_AB_ENV("STE_GEMM_FEW_SPLIT");
    on = (e && e[0] == '0') ? 0 : 1;
  }
  if (!on || !a.a_kc || !a.b_kc || !a.ws || a.batch != 1 || a.colsum) return 0;
  if ((a.N & 7) || (a.K & 63) || a.K / 64 < 40 || a.M < 2048) return 0;
  const int tiles = ((a.M + 255) / 256) * ((a.N + 255) / 256);
  if (tiles * 2 > num_cus()) return 0;
  if (2 * (int64_t)a.M * a.N * 4 > a.ws_bytes) return 0;
  return 2;
}

// Batched weight gradients (both operands k-major, batch > 1: the wav2vec2 conv stack's per-clip
// dW slabs over strided views, K = frames of one clip, usually ragged): the 8-phase kernel over
// the whole-64 part of K (the batch fills the chip), the K % 64 tail accumulated by the small
// kernel.  Plain alpha/beta epilogue only.
bool batched_dw_ok(const ste_gemm_args& a) {
  static int on = -1;   // STE_GEMM_BATCHED_DW=0: the small kernel (A/B)
  if (on < 0) {
    const char* e = STE_AB_ENV("STE_GEMM_BATCHED_DW");
    on = (e && e[0] == '0') ? 0 : 1;
  }
  if (!on || a.a_kc || a.b_kc || a.batch < 2) return false;
  if (a.bias || a.C2 || a.C3 || a.R || a.Z || a.colsum || a.row_scale || a.act || a.drop_p > 0.f) return false;
  if ((a.M & 7) || (a.N & 7) || a.M < 256 || a.N < 256 || a.K < 1024) return false;
  const long tiles = (long)((a.M + 255) / 256) * ((a.N + 255) / 256) * a.batch;
  return tiles >= 240;
}

// Weight-gradient plan: S K-slabs of Kc (or Kc + 1: the K/64 - S·Kc leftover tiles, one each
// to the first slabs) 64-deep tiles on the 8-phase kernel with both operands k-major; only a
// ragged K % 64 tail goes to the small kernel.
struct SplitPlan {
  int S, Kc;  // S == 0: not applicable
};
SplitPlan splitk_plan(const ste_gemm_args& a) {
  SplitPlan pl{0, 0};
  if (a.a_kc || a.b_kc || !a.ws || a.batch != 1) return pl;
  if (a.bias || a.C2 || a.C3 || a.R || a.Z || a.colsum || a.row_scale || a.act || a.drop_p > 0.f || a.c_bf16) return pl;
  if ((a.M & 7) || (a.N & 7)) return pl;
  const int nk = a.K / 64;
  const int tiles = ((a.M + 255) / 256) * ((a.N + 255) / 256);
  if (nk < 16 || tiles > 256) return pl;
  int S = 256 / tiles;
  if (S > nk / 8) S = nk / 8;
  const int64_t slab = (int64_t)a.M * a.N * 4;
  while (S > 1 && S * slab > a.ws_bytes) --S;
  if (S < 1 || S * slab > a.ws_bytes) return pl;
  pl.S = S;
  pl.Kc = nk / S;
  return pl;
}

template <bool A_KC, bool B_KC>
int launch_small(const ste_gemm_args& a, hipStream_t s) {
  using namespace small;
  const int num_m = (a.M + BM - 1) / BM, num_n = (a.N + BN - 1) / BN;
  const int nb = num_m * num_n * a.batch;
  hipLaunchKernelGGL((gemm_bf16_kernel<A_KC, B_KC>), dim3(nb), dim3(NT), LDS_BYTES, s, a);
  STE_CHECK_LAUNCH();
  return 0;
}

template <bool A_KC, bool B_KC>
int launch_big(const ste_gemm_args& a, hipStream_t s) {
  using namespace big;
  const int num_m = (a.M + BM - 1) / BM, num_n = (a.N + BN - 1) / BN;
  const int nb = num_m * num_n * a.batch;
  hipLaunchKernelGGL((gemm_big_kernel<A_KC, B_KC>), dim3(nb), dim3(NT), LDS_BYTES, s, a);
  STE_CHECK_LAUNCH();
  return 0;
}

bool big_ok_shape(const ste_gemm_args& a) {
  if (a.K % big::BK) return false;
  if (!a.a_kc || a.M < 8) return false;                 // dW reductions stay on the small kernel
  if (!a.b_kc && (a.N % 8)) return false;
  return true;
}
// plan thresholds (ste_gemm_plan_min_tiles; the A/B build also reads STE_GEMM_MIN_TILES)
int g_min_tiles_bf16 = -1, g_min_tiles_mx8 = 240;
int min_tiles_bf16() {
  if (g_min_tiles_bf16 < 0) {
    const char* e = STE_AB_ENV("STE_GEMM_MIN_TILES");
    g_min_tiles_bf16 = e ? atoi(e) : 240;
  }
  return g_min_tiles_bf16;
}
bool big_ok(const ste_gemm_args& a) {
  if (!big_ok_shape(a)) return false;
  const long tiles = (long)((a.M + 255) / 256) * ((a.N + 255) / 256) * a.batch;
  return tiles >= min_tiles_bf16();
}

}  // namespace

static int env_flag(const char* name) {
  const char* e = STE_AB_ENV(name);
  return (e && e[0] == '1') ? 1 : 0;
}
// STE_GEMM_SMALL_ONLY=1: every shape on the 128x128 kernel; STE_GEMM_2PH=1: the 2-buffer
// gemm_big schedule instead of the 8-phase one (A/B comparisons in one process).
static int gemm_mode() {
  static int mode = -1;
  if (mode < 0) mode = env_flag("STE_GEMM_SMALL_ONLY") ? 0 : (env_flag("STE_GEMM_2PH") ? 1 : 2);
  return mode;
}

extern "C" int ste_gemm_kernel(const ste_gemm_args* args) {
  if (!args) return STE_ERR_ARG;
  ste_gemm_args a = *args;
  if (a.batch <= 0) a.batch = 1;
  const int variant = (a.a_kc ? 0 : 2) + (a.b_kc ? 0 : 1);
  if (gemm_mode() == 2 && splitk_plan(a).S > 0) return STE_GEMM_KERNEL_SPLITK + variant;
  if (gemm_mode() == 2 && few_split(a) && big_ok_shape(a)) return STE_GEMM_KERNEL_SPLITK + variant;
  if (gemm_mode() == 2 && batched_dw_ok(a)) return STE_GEMM_KERNEL_8PH + variant;
  if (gemm_mode() > 0 && big_ok(a)) return (gemm_mode() == 2 ? STE_GEMM_KERNEL_8PH : STE_GEMM_KERNEL_BIG) + variant;
  return STE_GEMM_KERNEL_SMALL + variant;
}

// rocprofv3's (demangled, namespace-stripped) name of the kernel ste_gemm would launch
extern "C" int ste_gemm_kernel_name(const ste_gemm_args* args, char* buf, int len) {
  if (!args || !buf || len <= 0) return STE_ERR_ARG;
  const int k = ste_gemm_kernel(args);
  const int v = k & 3;
  const char* ak = (v & 2) ? "false" : "true";
  const char* bk = (v & 1) ? "false" : "true";
  if (k >= STE_GEMM_KERNEL_8PH) {
    ste_gemm_args a = *args;
    int ef = -1, act = 0;
    if (k >= STE_GEMM_KERNEL_SPLITK) {
      ef = 0;
    } else {
      const int f = epi_flags(a);
#define STE_MATCH(AK, BK, E, ACT) \
  if (AK == (bool)a.a_kc && BK == (bool)a.b_kc && f == (E) && a.act == (ACT)) { ef = (E); act = (ACT); }
      STE_EPI_SPECS(STE_MATCH)
#undef STE_MATCH
    }
    snprintf(buf, len, "gemm_8ph_kernel<%s, %s, %d, %d>", ak, bk, ef, act);
  } else {
    snprintf(buf, len, "%s<%s, %s>", k >= STE_GEMM_KERNEL_BIG ? "gemm_big_kernel" : "gemm_bf16_kernel", ak, bk);
  }
  return 0;
}

extern "C" int ste_gemm(const ste_gemm_args* args, void* stream) {
  if (!args) return STE_ERR_ARG;
  ste_gemm_args a = *args;
  if (a.batch <= 0) a.batch = 1;
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) return STE_ERR_ARG;
  // alignment contract (16-B operand chunks)
  if (a.a_kc ? (a.K & 7) || (a.lda & 7) : (a.M & 7) || (a.lda & 7)) return STE_ERR_SHAPE;
  if (a.b_kc ? (a.K & 7) || (a.ldb & 7) : (a.N & 7) || (a.ldb & 7)) return STE_ERR_SHAPE;
  if (a.drop_ld == 0) a.drop_ld = a.N;
  // epilogue contract: 16-B aligned rows for every output / epilogue operand (8 columns per lane)
  // (N < 8: every column goes through the element-wise tail path, any alignment works)
  auto misaligned = [&a](const void* ptr, int64_t ld, int esz) {
    return a.N >= 8 && ptr && ((((uintptr_t)ptr) & 15) || ((ld * esz) & 15));
  };
  if (misaligned(a.C, a.ldc, a.c_bf16 ? 2 : 4) || misaligned(a.C2, a.ldc2, 2) || misaligned(a.C3, a.ldc3, 2) ||
      misaligned(a.R, a.ldr, a.r_bf16 ? 2 : 4) || misaligned(a.Z, a.ldz, 2) || misaligned(a.bias, 0, 4))
    return STE_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  const int mode = gemm_mode();
  if (mode == 2) {
    const SplitPlan pl = splitk_plan(a);
    if (pl.S > 0) {
      ste_gemm_args g = a;
      const int64_t kc = (int64_t)pl.Kc * 64;
      const int nk_all = a.K / 64;
      const int rem = nk_all - pl.S * pl.Kc;   // whole K-tiles past S·Kc: one each to slabs 0..rem-1
      g.K = (int)kc;
      g.batch = pl.S;
      g.strideA = kc * a.lda;
      g.strideB = kc * a.ldb;
      g.ws = nullptr;
      g.ws_bytes = -(int64_t)(rem + 1);
      g.C = a.ws; g.ldc = a.N; g.strideC = (int64_t)a.M * a.N; g.c_bf16 = 0;
      g.alpha = 1.f; g.beta = 0.f;
      if (int e = launch_8ph<false, false>(g, s)) return e;
      const int64_t work = (int64_t)a.M * (a.N / 4);
      const dim3 rgrid((unsigned)((work + 255) / 256));
      if (pl.S <= 4)
        hipLaunchKernelGGL(splitk_reduce_kernel<4>, rgrid, dim3(256), 0, s, (float*)a.C, a.ldc, a.ws, a.M, a.N, pl.S,
                           a.alpha, a.beta);
      else if (pl.S <= 8)
        hipLaunchKernelGGL(splitk_reduce_kernel<8>, rgrid, dim3(256), 0, s, (float*)a.C, a.ldc, a.ws, a.M, a.N, pl.S,
                           a.alpha, a.beta);
      else
        hipLaunchKernelGGL(splitk_reduce_kernel<16>, rgrid, dim3(256), 0, s, (float*)a.C, a.ldc, a.ws, a.M, a.N, pl.S,
                           a.alpha, a.beta);
      STE_CHECK_LAUNCH();
      const int64_t kdone = (int64_t)nk_all * 64;
      if (kdone < a.K) {  // the ragged K % 64 tail: accumulate on the small kernel
        ste_gemm_args r = a;
        r.K = (int)(a.K - kdone);
        r.A = (const bf16*)a.A + kdone * a.lda;
        r.B = (const bf16*)a.B + kdone * a.ldb;
        r.beta = 1.f;
        r.ws = nullptr;
        return launch_small<false, false>(r, s);
      }
      return 0;
    }
  }
  if (mode == 2 && batched_dw_ok(a)) {
    ste_gemm_args g = a;
    const int64_t kdone = (int64_t)(a.K / 64) * 64;
    g.K = (int)kdone;
    if (int e = launch_8ph<false, false>(g, s)) return e;
    if (kdone < a.K) {  // ragged tail: += on the small kernel, per batch entry
      ste_gemm_args r = a;
      r.K = (int)(a.K - kdone);
      r.A = (const bf16*)a.A + kdone * a.lda;
      r.B = (const bf16*)a.B + kdone * a.ldb;
      r.beta = 1.f;
      return launch_small<false, false>(r, s);
    }
    return 0;
  }
  if (mode == 2 && few_split(a) && big_ok_shape(a)) {
    const int S = few_split(a);
    ste_gemm_args g = a;
    const int nk_all = a.K / 64;
    g.K = (nk_all / S) * 64;
    g.batch = S;
    g.ws = nullptr;
    g.ws_bytes = -(int64_t)(nk_all - S * (nk_all / S) + 1);
    g.bias = nullptr; g.C2 = nullptr; g.C3 = nullptr; g.R = nullptr; g.Z = nullptr; g.colsum = nullptr;
    g.row_scale = nullptr; g.act = 0; g.drop_p = 0.f;
    g.C = a.ws; g.ldc = a.N; g.strideC = (int64_t)a.M * a.N; g.c_bf16 = 0;
    g.alpha = 1.f; g.beta = 0.f;
    if (int e = launch_8ph<true, true>(g, s)) return e;
    const int64_t work = (int64_t)a.M * (a.N / 8);
    const int blocks = (int)((work + 255) / 256 < 4096 ? (work + 255) / 256 : 4096);
    hipLaunchKernelGGL(splitk_epi_kernel, dim3(blocks), dim3(256), 0, s, a, (const float*)a.ws, S);
    STE_CHECK_LAUNCH();
    return 0;
  }
  // column sums (bias gradients): with a large enough workspace every tile row writes its two waves'
  // partial rows there and one ordered pass adds them up (run-to-run deterministic); without one,
  // fp32 atomics.  The plans above never take a colsum launch, so ws is free for the partials.
  const bool use_big = mode > 0 && big_ok(a);
  int64_t cs_rows = 0;
  if (a.colsum) {
    const int bm = use_big ? 256 : small::BM;
    const int64_t rows = 2 * (int64_t)((a.M + bm - 1) / bm);
    if (a.ws && a.ws_bytes >= rows * a.batch * a.N * 4) cs_rows = rows;
  }
  if (!cs_rows) a.ws = nullptr;
  int e;
  if (use_big) {
    if (mode == 2) e = a.b_kc ? launch_8ph<true, true>(a, s) : launch_8ph<true, false>(a, s);
    else e = a.b_kc ? launch_big<true, true>(a, s) : launch_big<true, false>(a, s);
  } else if (a.a_kc && a.b_kc) {
    e = launch_small<true, true>(a, s);
  } else if (a.a_kc && !a.b_kc) {
    e = launch_small<true, false>(a, s);
  } else if (!a.a_kc && !a.b_kc) {
    e = launch_small<false, false>(a, s);
  } else {
    e = launch_small<false, true>(a, s);
  }
  if (e == 0 && cs_rows) e = ste_rowsum_ordered(a.ws, cs_rows, a.N, a.batch, a.colsum, stream);
  return e;
}

extern "C" int ste_gemm_tile_map(int t, int num_m, int num_n, int* tm, int* tn) {
  if (!tm || !tn || num_m <= 0 || num_n <= 0 || t < 0 || t >= num_m * num_n) return STE_ERR_ARG;
  tile_of(t, num_m, num_n, *tm, *tn);
  return 0;
}

extern "C" int64_t ste_gemm_colsum_ws_floats(const ste_gemm_args* args) {
  if (!args || !args->colsum) return 0;
  const int bm = 64;   // the smallest row tile of any GEMM kernel (ste_gemm_f32): an upper bound
  return 2 * (int64_t)((args->M + bm - 1) / bm) * (args->batch > 0 ? args->batch : 1) * args->N;
}

// ============================================================ MX-fp8 GEMM (config 5)
// Y = X·Wᵀ with both operands OCP e4m3 (KC, k contiguous) and E8M0 block scales, one per 32
// consecutive k of a row ([rows][K/32] bytes): v_mfma_scale_f32_16x16x128_f8f6f4, which runs at
// twice the bf16 MFMA rate (MI355X_MICROARCH.md, matrix cores).  Same 256x256 tile, 8 waves
// (2(M) x 4(N), 128x64 each), 2-deep global_load_lds ring and general epilogue as gemm_big;
// a K-tile is 128 fp8 = 128 B per row, so the LDS image and its swizzle are gemm_big's.
// Operand lane map of the 16x16x128 form (probed on the box with exact integer data,
// scratch/mx8_probe.hip): lane l holds row l&15, bytes 0-15 = k 16g..16g+15 and bytes 16-31 =
// k 64+16g..+15 (g = l>>4); the scale of row r's k-block kb is read from lane r + 16·kb.  So
// lane l supplies the scale of its own row and k-block g.
namespace mx8 {
constexpr int BM = 256, BN = 256, BK = 128, NT = 512;
constexpr int TILE_BYTES = BM * BK;             // 32 KiB per operand per stage
constexpr int SC_BYTES = BM * 4;                // 4 scale bytes per row per K-tile
constexpr int STAGE_BYTES = 2 * TILE_BYTES + 2 * SC_BYTES;
constexpr int LDS_BYTES = 2 * STAGE_BYTES;      // 132 KiB
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4v __attribute__((ext_vector_type(4)));

STE_DEV void issue_tile(const uint8_t* base, int64_t ld, int row0, int rows, int k0, char* tile, int wave,
                        int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = wave * 4 + i;
    const int r = piece * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ (lane >> 3);
    const int gr = min(row0 + r, rows - 1);
    const uint8_t* src = base + (int64_t)gr * ld + k0 + ch * 16;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(tile + piece * 1024), 16, 0, 0);
  }
}
// waves 0-3: A scales of rows 64w..64w+63; waves 4-7: B scales.  One dword (4 k-blocks) per row.
STE_DEV void issue_scales(const uint8_t* sa, const uint8_t* sb, int64_t lds_a, int64_t lds_b, int m0, int M, int n0,
                          int N, int k0, char* stage, int wave, int lane) {
  const bool isb = wave >= 4;
  const int r = (wave & 3) * 64 + lane;
  const uint8_t* src = isb ? sb + (int64_t)min(n0 + r, N - 1) * lds_b + (k0 >> 5)
                           : sa + (int64_t)min(m0 + r, M - 1) * lds_a + (k0 >> 5);
  char* dst = stage + 2 * TILE_BYTES + (isb ? SC_BYTES : 0) + (wave & 3) * 256;
  __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)dst, 4, 0, 0);
}
STE_DEV i32x8 frag(const char* tile, int rb, int lane) {
  const int r = rb + (lane & 15), g = lane >> 4;
  const i32x4v lo = *reinterpret_cast<const i32x4v*>(tile + r * 128 + ((g ^ (r & 7)) << 4));
  const i32x4v hi = *reinterpret_cast<const i32x4v*>(tile + r * 128 + (((g + 4) ^ (r & 7)) << 4));
  return i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
STE_DEV int scale(const char* sc, int rb, int lane) {
  return *reinterpret_cast<const int*>(sc + (rb + (lane & 15)) * 4) >> (8 * (lane >> 4));
}
}  // namespace mx8

__global__ __launch_bounds__(mx8::NT, 1) void gemm_mx8_kernel(ste_gemm_args p, const uint8_t* sa, const uint8_t* sb,
                                                              Q8Out q8o) {
  using namespace mx8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int num_m = (p.M + BM - 1) / BM, num_n = (p.N + BN - 1) / BN;
  int batch, tm, tn;
  map_tile(gridDim.x, num_m, num_n, batch, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const uint8_t* A = (const uint8_t*)p.A;
  const uint8_t* B = (const uint8_t*)p.B;
  const int64_t lsa = p.K >> 5, lsb = p.K >> 5;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / BK;
  issue_tile(A, p.lda, m0, p.M, 0, smem, wave, lane);
  issue_tile(B, p.ldb, n0, p.N, 0, smem + TILE_BYTES, wave, lane);
  issue_scales(sa, sb, lsa, lsb, m0, p.M, n0, p.N, 0, smem, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      char* nxt = smem + (cur ^ 1) * STAGE_BYTES;
      issue_tile(A, p.lda, m0, p.M, (kt + 1) * BK, nxt, wave, lane);
      issue_tile(B, p.ldb, n0, p.N, (kt + 1) * BK, nxt + TILE_BYTES, wave, lane);
      issue_scales(sa, sb, lsa, lsb, m0, p.M, n0, p.N, (kt + 1) * BK, nxt, wave, lane);
    }
    const char* ta = smem + cur * STAGE_BYTES;
    const char* tb = ta + TILE_BYTES;
    const char* sca = ta + 2 * TILE_BYTES;
    const char* scb = sca + SC_BYTES;
    i32x8 fb[4];
    int sbv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      fb[j] = frag(tb, wn * 64 + j * 16, lane);
      sbv[j] = scale(scb, wn * 64 + j * 16, lane);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const i32x8 fa = frag(ta, wm * 128 + i * 16, lane);
      const int sav = scale(sca, wm * 128 + i * 16, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fa, fb[j], acc[i][j], 0, 0, 0, sav, 0, sbv[j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  float* epi = reinterpret_cast<float*>(smem) + wave * big::EPI_ROWS * EPI_LD;
  Csum csum = {};
  constexpr bool EPI_SKIP = false;
#define EPI_COL0 (n0 + wn * 64)
#define EPI_COL1 (n0 + wn * 64 + 32)
#define STE_EPI_PASS(PS)                                                                                     \
  {                                                                                                          \
    for (int ii = 0; ii < 2; ++ii) {                                                                         \
      _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                                        \
        _Pragma("unroll") for (int r = 0; r < 4; ++r) {                                                      \
          epi[(ii * 16 + (lane >> 4) * 4 + r) * EPI_LD + j * 16 + (lane & 15)] = acc[2 * (PS) + ii][j][r];   \
        }                                                                                                    \
      }                                                                                                      \
    }                                                                                                        \
    __builtin_amdgcn_s_waitcnt(0xc07f);                                                                      \
    __builtin_amdgcn_wave_barrier();                                                                         \
    for (int hh = 0; hh < big::EPI_ROWS; hh += 16) {                                                         \
      if (!EPI_SKIP) epilogue_tile(p, epi + hh * EPI_LD, 16, m0 + wm * 128 + (PS) * big::EPI_ROWS + hh,     \
                                   EPI_COL0, EPI_COL1, batch, lane, csum, EPI_LD, false, q8o.q ? &q8o : nullptr);                                   \
    }                                                                                                        \
    __builtin_amdgcn_s_waitcnt(0xc07f);                                                                      \
    __builtin_amdgcn_wave_barrier();                                                                         \
  }
  STE_EPI_PASS(0) STE_EPI_PASS(1) STE_EPI_PASS(2) STE_EPI_PASS(3)
#undef STE_EPI_PASS
#undef EPI_COL0
#undef EPI_COL1
  if (p.colsum)
    colsum_flush(p, csum, n0 + wn * 64, n0 + wn * 64 + 32, batch, lane, ((int64_t)batch * num_m + tm) * 2 + wm);
}

// bf16 [rows][K] (row stride ld) -> e4m3 [rows][K] + E8M0 [rows][K/32].  Block scale 2^e with
// e = ceil(log2(amax/448)): the largest element maps to <= 448 (no saturation), zero blocks
// get 2^-127.  4 lanes (8 elements each) per 32-element block.
__global__ __launch_bounds__(256) void mx8_quant_kernel(const bf16* x, int64_t ld, int rows, int K, uint8_t* q,
                                                        uint8_t* sc) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int per_row = K >> 3;
  const int64_t r = t / per_row;  // K % 128 == 0: a 4-lane block never straddles rows
  const int c = (int)(t - r * per_row) * 8;
  if (r >= rows) return;
  mx8_block_store(load_bf16x8(x + r * ld + c), q + r * K + c, sc + r * (K >> 5) + (c >> 5), threadIdx.x);
}

extern "C" int ste_mx8_quant(const void* x, int64_t ldx, int rows, int K, void* q, void* scales, void* stream) {
  if (rows <= 0 || K <= 0 || (K & 127) || ldx < K || (ldx & 7)) return STE_ERR_SHAPE;
  const int64_t threads = (int64_t)rows * (K >> 3);
  hipLaunchKernelGGL(mx8_quant_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)x, ldx, rows, K, (uint8_t*)q, (uint8_t*)scales);
  STE_CHECK_LAUNCH();
  return 0;
}

namespace {
// STE_MX8_8PH=0: the single-stage gemm_mx8_kernel for every shape (A/B runs)
// Round 5: until the scale-select fix (mfma_mx) the persistent 8-phase MX kernel returned wrong
// products at every shape it was planned for (>= 240 tiles), in every tree since round 3
// (profiles/r5q_mx8_bisect.txt); tests/test_kernels_gpu.py::test_gemm_mx8_8ph_specs now checks
// each of its compile-time epilogues there.  libste_ab.so with STE_MX8_8PH=0: the single-stage
// gemm_mx8_kernel for every MX GEMM (A/B)
bool mx8_8ph_on() {
  static int v = -1;
  if (v < 0) {
    const char* e = STE_AB_ENV("STE_MX8_8PH");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}
// MX-fp8 on the persistent 8-phase kernel: the e4m3 operands passed as bf16 pairs (K, lda, ldb
// halved), compile-time epilogues for the Conformer forward GEMMs (and, for the opt-in MX-fp8
// input gradients, the activation-backward dz), the run-time epilogue (which also writes the fp8
// copy) otherwise
#define STE_MX8_SPECS(X)                                                      \
  X(EF_BIAS | EF_CBF16, STE_ACT_NONE)                            /* QKV */         \
  X(EF_CBF16, STE_ACT_NONE)                                      /* pw conv 1 */   \
  X(EF_BIAS | EF_R, STE_ACT_NONE)                                /* O, FFN out */  \
  X(EF_BIAS | EF_C2 | EF_CBF16 | EF_Q8, STE_ACT_SWISH)           /* FFN in */      \
  X(EF_BIAS | EF_C2 | EF_CBF16 | EF_Q8 | EF_NOC, STE_ACT_SWISH)  /* FFN in, frozen: fp8 copy only */ \
  X(EF_Z | EF_CBF16, STE_ACT_SWISH_BWD)                          /* dz (fp8_bwd A/B) */

int mx8_ef(const ste_gemm_args& a, bool q_out) { return epi_flags(a) | (q_out ? EF_Q8 : 0) | (a.C ? 0 : EF_NOC); }

// Host-side plan: the persistent 8-phase MX kernel, or the single-stage gemm_mx8_kernel.  The
// 8-phase kernel's operand and scale DMA sources are 32-bit byte offsets from the operand base
// (stage_half<.., O32>, stage_scales), so each operand (fp8 bytes, M·lda / N·ldb) must stay
// below 4 GiB; larger operands, other epilogues and shapes under 240 tiles take the single-stage
// kernel (64-bit addressing)
bool mx8_8ph_plan(const ste_gemm_args& a, bool q_out) {
  if (!mx8_8ph_on() || gemm_mode() != 2) return false;
  const int64_t nb = (int64_t)((a.M + 255) / 256) * ((a.N + 255) / 256);
  if (nb < g_min_tiles_mx8 || (q_out && (a.N % 256) != 0)) return false;   // fp8 copy per FULL 256-column tile
  const uint64_t lim = 1ull << 32;
  if ((uint64_t)a.M * (uint64_t)a.lda >= lim || (uint64_t)a.N * (uint64_t)a.ldb >= lim) return false;
  const int ef = mx8_ef(a, q_out);
#define STE_MX_MATCH(E, ACT) if (ef == (E) && a.act == (ACT)) return true;
  STE_MX8_SPECS(STE_MX_MATCH)
#undef STE_MX_MATCH
  return false;
}

int launch_mx8_8ph(const ste_gemm_args& a8, const Mx8Args& mx, hipStream_t s) {
  ste_gemm_args a = a8;
  a.K = a8.K / 2;
  a.lda = a8.lda / 2;
  a.ldb = a8.ldb / 2;
  const int nb = ((a.M + 255) / 256) * ((a.N + 255) / 256);
  const int grid = nb < num_cus() ? nb : num_cus();
  const int ef = mx8_ef(a, mx.q8.q != nullptr);
#define STE_MX(E, ACT)                                                                                          \
  if (ef == (E) && a.act == (ACT)) {                                                                            \
    hipLaunchKernelGGL((gemm_8ph_kernel<true, true, (E), (ACT), true>), dim3(grid), dim3(ph8::NT), ph8::LDS_BYTES, \
                       s, a, mx);                                                                               \
    STE_CHECK_LAUNCH();                                                                                         \
    return 0;                                                                                                   \
  }
  STE_MX8_SPECS(STE_MX)
#undef STE_MX
  return -1;   // other epilogues: the single-stage kernel
}
}  // namespace

extern "C" int ste_gemm_plan_min_tiles(int bf16_tiles, int mx8_tiles, int* prev_bf16, int* prev_mx8) {
  if (prev_bf16) *prev_bf16 = min_tiles_bf16();
  if (prev_mx8) *prev_mx8 = g_min_tiles_mx8;
  if (bf16_tiles > 0) g_min_tiles_bf16 = bf16_tiles;
  if (mx8_tiles > 0) g_min_tiles_mx8 = mx8_tiles;
  return 0;
}

extern "C" int ste_gemm_mx8_kernel(const ste_gemm_args* args, int q_out) {
  if (!args) return STE_ERR_ARG;
  return mx8_8ph_plan(*args, q_out != 0) ? 1 : 0;
}

extern "C" int ste_gemm_mx8(const ste_gemm_args* args, const void* a_scales, const void* b_scales, void* q_out,
                            void* q_scales, void* stream) {
  if (!args || !a_scales || !b_scales || (!args->C && !q_out) || (!q_out != !q_scales)) return STE_ERR_ARG;
  if (q_out && ((args->N & 127) || (((uintptr_t)q_out) & 7) || args->colsum)) return STE_ERR_SHAPE;
  ste_gemm_args a = *args;
  a.batch = 1;
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) return STE_ERR_ARG;
  if (!a.a_kc || !a.b_kc || (a.K & 127) || (a.lda & 15) || (a.ldb & 15) || a.lda < a.K || a.ldb < a.K || a.ws)
    return STE_ERR_SHAPE;
  if (a.drop_ld == 0) a.drop_ld = a.N;
  auto misaligned = [&a](const void* ptr, int64_t ld, int esz) {
    return a.N >= 8 && ptr && ((((uintptr_t)ptr) & 15) || ((ld * esz) & 15));
  };
  if (misaligned(a.C, a.ldc, a.c_bf16 ? 2 : 4) || misaligned(a.C2, a.ldc2, 2) || misaligned(a.C3, a.ldc3, 2) ||
      misaligned(a.R, a.ldr, a.r_bf16 ? 2 : 4) || misaligned(a.Z, a.ldz, 2) || misaligned(a.bias, 0, 4) ||
      (((uintptr_t)a.A) & 15) || (((uintptr_t)a.B) & 15) || (((uintptr_t)a_scales) & 3) ||
      (((uintptr_t)b_scales) & 3))
    return STE_ERR_SHAPE;
  const int nb = ((a.M + 255) / 256) * ((a.N + 255) / 256);
  const Q8Out q8o = {(uint8_t*)q_out, (uint8_t*)q_scales, a.N};
  if (mx8_8ph_plan(a, q_out != nullptr)) {
    const Mx8Args mx = {(const uint8_t*)a_scales, (const uint8_t*)b_scales, a.K / 32, a.K / 32, q8o};
    if (launch_mx8_8ph(a, mx, (hipStream_t)stream) == 0) return 0;
  }
  hipLaunchKernelGGL(gemm_mx8_kernel, dim3(nb), dim3(mx8::NT), mx8::LDS_BYTES, (hipStream_t)stream, a,
                     (const uint8_t*)a_scales, (const uint8_t*)b_scales, q8o);
  STE_CHECK_LAUNCH();
  return 0;
}

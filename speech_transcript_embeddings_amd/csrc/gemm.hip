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
// Tile 128x128x64, 256 threads (4 waves in 2x2, 64x64 per wave, 4x4 v_mfma_f32_16x16x32_bf16),
// register-staged double-buffered LDS (issue next tile's global loads before the MFMAs,
// write them after), XOR-swizzled LDS images (conflict-free ds_read_b128 / tr reads),
// XCD-aware bijective block remap, LDS-staged epilogue with row-contiguous stores.
#include "common.h"
#include "../../include/ste.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_BYTES = BM * BK * 2;            // 16 KiB per operand tile
constexpr int EPI_LD = 68;                          // fp32 row stride of the epilogue staging
constexpr int EPI_BYTES = 4 * 64 * EPI_LD * 4;      // 4 waves x 64 rows
constexpr int LDS_BYTES = (4 * TILE_BYTES > EPI_BYTES) ? 4 * TILE_BYTES : EPI_BYTES;

struct Stage {
  bf16x8 v[4];
};

// ---- KC tile: [128 rows][64 k], 128 B per row, 16-B chunk c stored at (c ^ (row&7)).
template <bool KC>
STE_DEV void stage_load(Stage& st, const bf16* __restrict__ base, int64_t ld, int row0, int rows, int k0,
                        int K, int tid) {
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

STE_DEV int km_chunk_xor(int k) { return ((k & 3) | ((k >> 1) & 4)) << 1; }

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

// fragment for mfma_f32_16x16x32_bf16: lane l holds X[row=rb+(l&15)][k=32s+8(l>>4)+j], j=0..7
template <bool KC>
STE_DEV bf16x8 frag_load(const char* tile, int rb, int s, int lane) {
  if (KC) {
    int r = rb + (lane & 15);
    int ch = s * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(tile + r * 128 + ((ch ^ (r & 7)) << 4));
  } else {
    int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    int k = s * 32 + 8 * g + q;
    int quad = (rb >> 2) + p;
    int a0 = k * 256 + ((quad ^ (km_chunk_xor(k) << 1)) << 3);
    int k1 = k + 4;
    int a1 = k1 * 256 + ((quad ^ (km_chunk_xor(k1) << 1)) << 3);
    s16x4 lo = ds_read_tr16(tile + a0);
    s16x4 hi = ds_read_tr16(tile + a1);
    return join_tr(lo, hi);
  }
}

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

template <bool A_KC, bool B_KC>
__global__ __launch_bounds__(NT, 2) void gemm_bf16_kernel(ste_gemm_args p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // LDS_BYTES dynamic
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // ---- block -> tile (bijective XCD remap, then grouped ordering for L2 reuse)
  const int num_m = (p.M + BM - 1) / BM, num_n = (p.N + BN - 1) / BN;
  const int tiles = num_m * num_n;
  const int nwg = gridDim.x;
  int bid = blockIdx.x;
  {
    int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int batch = bid / tiles;
  int t = bid - batch * tiles;
  constexpr int GROUP = 8;
  int group = t / (GROUP * num_n);
  int first_m = group * GROUP;
  int gsize = min(num_m - first_m, GROUP);
  int tm = first_m + (t % (GROUP * num_n)) % gsize;
  int tn = (t % (GROUP * num_n)) / gsize;
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
      for (int i = 0; i < 4; ++i) fa[i] = frag_load<A_KC>(ta, wm * 64 + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag_load<B_KC>(tb, wn * 64 + j * 16, s, lane);
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

  // ---- epilogue: stage the wave's 64x64 fp32 tile through LDS, then row-contiguous I/O
  float* epi = reinterpret_cast<float*>(smem) + wave * 64 * EPI_LD;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        epi[(i * 16 + (lane >> 4) * 4 + r) * EPI_LD + j * 16 + (lane & 15)] = acc[i][j][r];
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): own-wave LDS writes done (wave-private region)
  __builtin_amdgcn_wave_barrier();

  const int col = n0 + wn * 64 + (lane & 15) * 4;
  const bool col_ok = col < p.N;
  f32x4 bias = {0.f, 0.f, 0.f, 0.f};
  if (p.bias && col_ok) bias = *reinterpret_cast<const f32x4*>(p.bias + col);
  const uint32_t thresh = (uint32_t)(p.drop_p * 4294967296.0);
  const float inv_keep = p.drop_p > 0.f ? 1.0f / (1.0f - p.drop_p) : 1.0f;
  f32x4 csum = {0.f, 0.f, 0.f, 0.f};
  const int64_t offC = (int64_t)batch * p.strideC;
  const int64_t offR = (int64_t)batch * p.strideR;

#pragma unroll 4
  for (int it = 0; it < 16; ++it) {
    const int lr = it * 4 + (lane >> 4);
    const int row = m0 + wm * 64 + lr;
    if (row >= p.M || !col_ok) continue;
    f32x4 v = *reinterpret_cast<const f32x4*>(epi + lr * EPI_LD + (lane & 15) * 4);
    v = (v + bias) * p.alpha;
    if (p.act >= STE_ACT_SWISH && p.act <= STE_ACT_RELU) {
      if (p.C2) store_bf16x4((bf16*)p.C2 + offC + (int64_t)row * p.ldc2 + col, v);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = apply_act(v[e], p.act);
    } else if (p.act >= STE_ACT_SWISH_BWD) {
      f32x4 z = load_bf16x4((const bf16*)p.Z + offC + (int64_t)row * p.ldz + col);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] *= act_grad(z[e], p.act);
    }
    if (p.drop_p > 0.f) {
      const uint64_t base = (uint64_t)row * (uint64_t)p.drop_ld + (uint64_t)col;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] *= drop_scale(p.seed, base + e, thresh, inv_keep);
    }
    if (p.row_scale) v = v * p.row_scale[row];
    if (p.colsum) csum += v;
    if (p.R) {
      if (p.r_bf16) v += load_bf16x4((const bf16*)p.R + offR + (int64_t)row * p.ldr + col);
      else v += *reinterpret_cast<const f32x4*>((const float*)p.R + offR + (int64_t)row * p.ldr + col);
    }
    if (p.c_bf16) {
      bf16* c = (bf16*)p.C + offC + (int64_t)row * p.ldc + col;
      if (p.beta != 0.f) v += load_bf16x4(c) * p.beta;
      store_bf16x4(c, v);
    } else {
      float* c = (float*)p.C + offC + (int64_t)row * p.ldc + col;
      if (p.beta != 0.f) v += *reinterpret_cast<const f32x4*>(c) * p.beta;
      *reinterpret_cast<f32x4*>(c) = v;
    }
    if (p.C3) store_bf16x4((bf16*)p.C3 + offC + (int64_t)row * p.ldc3 + col, v);
  }
  if (p.colsum) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      csum[e] += __shfl_xor(csum[e], 16, 64);
      csum[e] += __shfl_xor(csum[e], 32, 64);
    }
    if (lane < 16 && col_ok) {
#pragma unroll
      for (int e = 0; e < 4; ++e) atomicAdd(p.colsum + (int64_t)batch * p.N + col + e, csum[e]);
    }
  }
}

template <bool A_KC, bool B_KC>
int launch(const ste_gemm_args& a, hipStream_t s) {
  const int num_m = (a.M + BM - 1) / BM, num_n = (a.N + BN - 1) / BN;
  const int nb = num_m * num_n * (a.batch > 0 ? a.batch : 1);
  hipLaunchKernelGGL((gemm_bf16_kernel<A_KC, B_KC>), dim3(nb), dim3(NT), LDS_BYTES, s, a);
  STE_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int ste_gemm(const ste_gemm_args* args, void* stream) {
  if (!args) return STE_ERR_ARG;
  ste_gemm_args a = *args;
  if (a.batch <= 0) a.batch = 1;
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) return STE_ERR_ARG;
  // alignment contract (16-B operand chunks, 16-B epilogue vectors)
  if ((a.N & 3) != 0) return STE_ERR_SHAPE;
  if (a.a_kc ? (a.K & 7) || (a.lda & 7) : (a.M & 7) || (a.lda & 7)) return STE_ERR_SHAPE;
  if (a.b_kc ? (a.K & 7) || (a.ldb & 7) : (a.N & 7) || (a.ldb & 7)) return STE_ERR_SHAPE;
  if ((a.ldc & 3) || (a.C2 && (a.ldc2 & 3)) || (a.C3 && (a.ldc3 & 3)) || (a.R && (a.ldr & 3))) return STE_ERR_SHAPE;
  if (a.drop_ld == 0) a.drop_ld = a.N;
  hipStream_t s = (hipStream_t)stream;
  if (a.a_kc && a.b_kc) return launch<true, true>(a, s);
  if (a.a_kc && !a.b_kc) return launch<true, false>(a, s);
  if (!a.a_kc && !a.b_kc) return launch<false, false>(a, s);
  return launch<false, true>(a, s);
}

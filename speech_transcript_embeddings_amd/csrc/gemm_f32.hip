// fp32-operand GEMM on the exact-f32 matrix core (v_mfma_f32_16x16x4_f32: an fmaf chain,
// bit for bit) for the projection / cross-attention / fusion heads, whose gradients are
// differences of the positive and corrupted transcripts' nearly identical activations.
//
// Replaces the aten::addmm / aten::mm behind the heads' nn.Linear layers in
//   /root/reference/training/trainer_unfreeze.py:66-99   EnhancedProjection
//                                                   :125-168 CrossModalAttention q / out_proj
//                                                   :171-211 AttentivePooling scorer (text side)
//                                                   :470-477 text_fusion / audio_fusion
// The reference computes these in fp32 (run_embedding_trainer_unfreeze.sh:27 --no_fp16).  With
// bf16 operands the loss gradient ds·(t_neg - t_pos) — a difference of two embeddings that
// share 80 % of their tokens — turns 2^-9 operand rounding into 4-18 % gradient errors (DESIGN
// §4); these GEMMs are tiny (M = batch rows, or 2·b·L text rows for the pooling scorer), so
// they run in fp32 at the f32 matrix rate (1/16 of bf16, MI355X_MICROARCH.md matrix table).
//
// Same argument block and epilogue order as ste_gemm (include/ste.h), with A, B, C2 and Z fp32.
// Tile 64x64, 256 threads = 4 waves of 32x32 (2x2 16x16 accumulators); k staged through LDS in
// chunks of 16 as [k][m] images (row stride 80 floats: the four k rows a fragment read touches
// land on disjoint 16-bank groups).  Weight gradients (a_kc = b_kc = 0) with a long reduction
// and a workspace split K into S slabs written to ws and summed in slab order (deterministic).
#include "common.h"
#include "../../include/ste.h"

namespace {

constexpr int BM = 64, BN = 64, BKC = 16, NT = 256, LDSW = 80;

STE_DEV float act_fwd(float v, int act) {
  switch (act) {
    case STE_ACT_SWISH: return swish_f(v);
    case STE_ACT_GELU: return gelu_f(v);
    case STE_ACT_TANH: return tanhf(v);
    case STE_ACT_RELU: return fmaxf(v, 0.0f);
    default: return v;
  }
}
STE_DEV float act_bwd(float z, int act) {
  switch (act) {
    case STE_ACT_SWISH_BWD: return swish_d(z);
    case STE_ACT_GELU_BWD: return gelu_d(z);
    case STE_ACT_TANH_BWD_OUT: return 1.0f - z * z;
    case STE_ACT_RELU_BWD: return z > 0.0f ? 1.0f : 0.0f;
    default: return 1.0f;
  }
}

// Stage a [64 rows x 16 k] chunk of an operand into img[k][row] (zero outside the matrix).
// KC: X[r*ld + k] (one float4 of 4 consecutive k per thread); KM: X[k*ld + r] (4 consecutive rows).
template <bool KC>
STE_DEV void stage(const float* X, int64_t ld, int rows, int K, int r0, int k0, float* img, int tid) {
  if constexpr (KC) {
    const int r = tid >> 2, kq = (tid & 3) * 4;
    const int gr = r0 + r, gk = k0 + kq;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (gr < rows) {
      const float* src = X + (int64_t)gr * ld + gk;
      if (gk + 3 < K) v = *reinterpret_cast<const f32x4*>(src);
      else
        for (int e = 0; e < 4; ++e) v[e] = gk + e < K ? src[e] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) img[(kq + e) * LDSW + r] = v[e];
  } else {
    const int k = tid >> 4, rq = (tid & 15) * 4;
    const int gk = k0 + k, gr = r0 + rq;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (gk < K) {
      const float* src = X + (int64_t)gk * ld + gr;
      if (gr + 3 < rows) v = *reinterpret_cast<const f32x4*>(src);
      else
        for (int e = 0; e < 4; ++e) v[e] = gr + e < rows ? src[e] : 0.f;
    }
    *reinterpret_cast<f32x4*>(img + k * LDSW + rq) = v;
  }
}

// SPLIT: write the raw accumulators of K range [z*kc, (z+1)*kc) to ws[z][M][N] (no epilogue).
template <bool A_KC, bool B_KC, bool SPLIT>
__global__ __launch_bounds__(NT) void gemm_f32_kernel(ste_gemm_args p, int kc) {
  __shared__ __attribute__((aligned(16))) float sa[BKC * LDSW];
  __shared__ __attribute__((aligned(16))) float sb[BKC * LDSW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int wm = (w & 1) * 32, wn = (w >> 1) * 32;
  const int r = lane & 15, g = lane >> 4;
  const float* A = (const float*)p.A;
  const float* B = (const float*)p.B;
  const int kb = SPLIT ? blockIdx.z * kc : 0;
  const int ke = SPLIT ? min(p.K, kb + kc) : p.K;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = kb; k0 < ke; k0 += BKC) {
    // the K range end acts as the matrix edge for this slab
    stage<A_KC>(A, p.lda, p.M, ke, m0, k0, sa, tid);
    stage<B_KC>(B, p.ldb, p.N, ke, n0, k0, sb, tid);
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BKC; kk += 4) {
      const float a0 = sa[(kk + g) * LDSW + wm + r], a1 = sa[(kk + g) * LDSW + wm + 16 + r];
      const float b0 = sb[(kk + g) * LDSW + wn + r], b1 = sb[(kk + g) * LDSW + wn + 16 + r];
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    __syncthreads();
  }
  // accumulator (i, j) element e: row m0+wm+16i+4g+e, column n0+wn+16j+r
  if constexpr (SPLIT) {
    float* slab = p.ws + (int64_t)blockIdx.z * p.M * p.N;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = n0 + wn + 16 * j + r;
        if (col >= p.N) continue;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = m0 + wm + 16 * i + 4 * g + e;
          if (row < p.M) slab[(int64_t)row * p.N + col] = acc[i][j][e];
        }
      }
    return;
  }
  const uint32_t thresh = (uint32_t)(p.drop_p * 4294967296.0);
  const float inv_keep = p.drop_p > 0.f ? 1.0f / (1.0f - p.drop_p) : 1.0f;
  const bool fwd_act = p.act >= STE_ACT_SWISH && p.act <= STE_ACT_RELU;
  const bool bwd_act = p.act >= STE_ACT_SWISH_BWD;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn + 16 * j + r;
    const bool cv = col < p.N;
    const float bias = (p.bias && cv) ? p.bias[col] : 0.f;
    float cs = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + wm + 16 * i + 4 * g + e;
        if (!cv || row >= p.M) continue;
        float v = (acc[i][j][e] + bias) * p.alpha;
        if (fwd_act) {
          if (p.C2) ((float*)p.C2)[(int64_t)row * p.ldc2 + col] = v;
          v = act_fwd(v, p.act);
        } else if (bwd_act) {
          v *= act_bwd(((const float*)p.Z)[(int64_t)row * p.ldz + col], p.act);
        }
        if (p.drop_p > 0.f) v *= drop_scale(p.seed, (uint64_t)row * (uint64_t)p.drop_ld + (uint64_t)col, thresh, inv_keep);
        if (p.row_scale) v *= p.row_scale[row];
        cs += v;
        if (p.R) {
          const int64_t ro = (int64_t)row * p.ldr + col;
          v += p.r_bf16 ? (float)((const bf16*)p.R)[ro] : ((const float*)p.R)[ro];
        }
        const int64_t co = (int64_t)row * p.ldc + col;
        if (p.beta != 0.f) v += p.beta * (p.c_bf16 ? (float)((const bf16*)p.C)[co] : ((const float*)p.C)[co]);
        if (p.C) {
          if (p.c_bf16) ((bf16*)p.C)[co] = (bf16)v;
          else ((float*)p.C)[co] = v;
        }
        if (p.C3) ((bf16*)p.C3)[(int64_t)row * p.ldc3 + col] = (bf16)(p.c3_lo ? v - (float)(bf16)v : v);
      }
    if (p.colsum) {  // the column's 4 lane groups hold disjoint rows: sum them
      cs += __shfl_xor(cs, 16, 64);
      cs += __shfl_xor(cs, 32, 64);
      // ordered mode: this wave's partial row (tile row x wave row) in ws, summed in order by the
      // host's second pass; else one atomic per column
      if (g == 0 && cv) {
        if (p.ws) p.ws[((int64_t)blockIdx.x * 2 + (w & 1)) * p.N + col] = cs;
        else atomicAdd(p.colsum + col, cs);
      }
    }
  }
}

// C = beta·C + alpha·Σ_z ws[z] (slab order), 4 columns per thread
__global__ __launch_bounds__(256) void f32_slab_reduce_kernel(float* C, int64_t ldc, const float* ws, int M, int N,
                                                              int S, float alpha, float beta) {
  const int64_t per_row = (N + 3) / 4;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < (int64_t)M * per_row; t += (int64_t)gridDim.x * 256) {
    const int row = (int)(t / per_row), c = (int)(t - (int64_t)row * per_row) * 4;
    for (int e = 0; e < 4 && c + e < N; ++e) {
      float s = 0.f;
      for (int z = 0; z < S; ++z) s += ws[((int64_t)z * M + row) * N + c + e];
      float* o = C + (int64_t)row * ldc + c + e;
      *o = (beta != 0.f ? beta * *o : 0.f) + alpha * s;
    }
  }
}

template <bool A_KC, bool B_KC>
int launch(const ste_gemm_args& a, hipStream_t s) {
  const dim3 grid((a.M + BM - 1) / BM, (a.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_f32_kernel<A_KC, B_KC, false>), grid, dim3(NT), 0, s, a, 0);
  STE_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int ste_gemm_f32(const ste_gemm_args* args, void* stream) {
  if (!args) return STE_ERR_ARG;
  ste_gemm_args a = *args;
  if (a.batch > 1) return STE_ERR_SHAPE;
  if (a.M <= 0 || a.N <= 0 || a.K <= 0 || !a.A || !a.B) return STE_ERR_ARG;
  // 16-B operand loads: KC operands need K % 4 == 0 and ld % 4 == 0, KM operands rows % 4 == 0
  if (a.a_kc ? (a.K & 3) || (a.lda & 3) : (a.M & 3) || (a.lda & 3)) return STE_ERR_SHAPE;
  if (a.b_kc ? (a.K & 3) || (a.ldb & 3) : (a.N & 3) || (a.ldb & 3)) return STE_ERR_SHAPE;
  if ((((uintptr_t)a.A) & 15) || (((uintptr_t)a.B) & 15)) return STE_ERR_SHAPE;
  if (a.act >= STE_ACT_SWISH_BWD && !a.Z) return STE_ERR_ARG;
  if (!a.C && !a.C3) return STE_ERR_ARG;
  if (a.drop_ld == 0) a.drop_ld = a.N;
  hipStream_t s = (hipStream_t)stream;
  // weight gradient over a long reduction: split K into slabs when the tiles cannot fill the chip
  const bool plain = !a.bias && a.act == STE_ACT_NONE && a.drop_p == 0.f && !a.row_scale && !a.colsum && !a.R &&
                     !a.C2 && !a.C3 && a.C && !a.c_bf16;
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  if (plain && a.ws && tiles < 256 && a.K >= 1024) {
    int S = (512 + tiles - 1) / tiles;
    S = S < a.K / 256 ? S : a.K / 256;
    while (S > 1 && (int64_t)S * a.M * a.N * 4 > a.ws_bytes) --S;
    if (S > 1) {
      int kc = (a.K + S - 1) / S;
      kc = (kc + BKC - 1) / BKC * BKC;
      S = (a.K + kc - 1) / kc;
      const dim3 grid((a.M + BM - 1) / BM, (a.N + BN - 1) / BN, S);
      if (!a.a_kc && !a.b_kc)
        hipLaunchKernelGGL((gemm_f32_kernel<false, false, true>), grid, dim3(NT), 0, s, a, kc);
      else if (a.a_kc && a.b_kc)
        hipLaunchKernelGGL((gemm_f32_kernel<true, true, true>), grid, dim3(NT), 0, s, a, kc);
      else if (a.a_kc)
        hipLaunchKernelGGL((gemm_f32_kernel<true, false, true>), grid, dim3(NT), 0, s, a, kc);
      else
        hipLaunchKernelGGL((gemm_f32_kernel<false, true, true>), grid, dim3(NT), 0, s, a, kc);
      STE_CHECK_LAUNCH();
      const int64_t work = (int64_t)a.M * ((a.N + 3) / 4);
      const int blocks = (int)((work + 255) / 256 < 1024 ? (work + 255) / 256 : 1024);
      hipLaunchKernelGGL(f32_slab_reduce_kernel, dim3(blocks), dim3(256), 0, s, (float*)a.C, a.ldc, a.ws, a.M, a.N, S,
                         a.alpha, a.beta);
      STE_CHECK_LAUNCH();
      return 0;
    }
  }
  // column sums: ordered partial rows in ws when it is large enough (deterministic), else atomics
  int64_t cs_rows = 0;
  if (a.colsum) {
    const int64_t rows = 2 * (int64_t)((a.M + BM - 1) / BM);
    if (a.ws && a.ws_bytes >= rows * a.N * 4) cs_rows = rows;
  }
  if (!cs_rows) a.ws = nullptr;
  int e;
  if (a.a_kc && a.b_kc) e = launch<true, true>(a, s);
  else if (a.a_kc) e = launch<true, false>(a, s);
  else if (a.b_kc) e = launch<false, true>(a, s);
  else e = launch<false, false>(a, s);
  if (e == 0 && cs_rows) e = ste_rowsum_ordered(a.ws, cs_rows, a.N, 1, a.colsum, stream);
  return e;
}

// XLM-R embedding gather / scatter-add and the fused optimizer tail.
//   embeddings: tf:models/xlm_roberta/modeling_xlm_roberta.py:75-121 (+ position ids :142-155)
//   clip_grad_norm_ + AdamW: ref:training/trainer_unfreeze.py:1108-1110 with the param
//   groups of :1487-1511 (torch.optim.AdamW decoupled weight decay, amsgrad=False).
#include "common.h"
#include "../../include/ste.h"

namespace {

constexpr int NT = 256;

// one block per sequence: position ids = cumsum(ids != pad) * (ids != pad) + pad
__global__ __launch_bounds__(NT) void embed_fwd_kernel(const int64_t* ids, int L, int D, int pad, const float* word,
                                                     const float* pos, const float* type0, float* out,
                                                     int32_t* pos_ids) {
  __shared__ int spos[2048];
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) {
    int c = 0;
    for (int l = 0; l < L; ++l) {
      const int nz = ids[(int64_t)b * L + l] != pad;
      c += nz;
      spos[l] = nz ? c + pad : pad;
    }
  }
  __syncthreads();
  for (int l = tid; l < L; l += NT) pos_ids[(int64_t)b * L + l] = spos[l];
  for (int i = tid * 4; i < L * D; i += NT * 4) {
    const int l = i / D, c = i % D;
    const int64_t id = ids[(int64_t)b * L + l];
    f32x4 v = *reinterpret_cast<const f32x4*>(word + id * D + c);
    v += *reinterpret_cast<const f32x4*>(pos + (int64_t)spos[l] * D + c);
    v += *reinterpret_cast<const f32x4*>(type0 + c);
    *reinterpret_cast<f32x4*>(out + ((int64_t)b * L + l) * D + c) = v;
  }
}

// word / position table rows of the embedding backward, deterministically: one wave per token row
// r; the first row of each id sums the rows carrying that id in row order (ids cached in LDS as
// int32 when they fit) and adds the sum to its table row — one writer per row, no atomics, so the
// gradient is run-to-run identical (the rows of BOS / EOS and of each position repeat once per
// transcript).  pad ids get nothing (nn.Embedding(padding_idx)).  D % 4 == 0, D <= 1024.
constexpr int EMB_WAVES = 16;
constexpr int EMB_LDS_IDS = 16384;
template <typename IdT>
__global__ __launch_bounds__(EMB_WAVES * 64) void embed_rows_ordered_kernel(const IdT* __restrict__ ids, int rows,
                                                                          int D, int pad,
                                                                          const float* __restrict__ dout,
                                                                          float* __restrict__ table) {
  extern __shared__ int sids[];
  const bool in_lds = rows <= EMB_LDS_IDS;
  if (in_lds)
    for (int i = threadIdx.x; i < rows; i += EMB_WAVES * 64) sids[i] = (int)ids[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, r = blockIdx.x * EMB_WAVES + (threadIdx.x >> 6);
  if (r >= rows) return;
  auto id_at = [&](int j) { return in_lds ? sids[j] : (int)ids[j]; };
  const int id = id_at(r);
  if (id == pad || id < 0) return;
  for (int j0 = 0; j0 < r; j0 += 64) {   // an earlier row with this id owns the sum
    const int j = j0 + lane;
    if (__ballot(j < r && id_at(j) == id)) return;
  }
  f32x4 acc[4] = {};
  for (int j0 = r; j0 < rows; j0 += 64) {
    const int j = j0 + lane;
    uint64_t m = __ballot(j < rows && id_at(j) == id);
    while (m) {
      const int k = __builtin_ctzll(m);
      m &= m - 1;
      const float* src = dout + (int64_t)(j0 + k) * D;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = (lane + 64 * q) * 4;
        if (c < D) acc[q] += *reinterpret_cast<const f32x4*>(src + c);
      }
    }
  }
  float* dst = table + (int64_t)id * D;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = (lane + 64 * q) * 4;
    if (c < D) *reinterpret_cast<f32x4*>(dst + c) += acc[q];
  }
}

__global__ __launch_bounds__(NT) void sumsq_kernel(const float* g, int64_t n, double* acc, double* part) {
  __shared__ double red[NT / 64];
  double s = 0.0;
  float sf = 0.f;
  int cnt = 0;
  for (int64_t i = ((int64_t)blockIdx.x * NT + threadIdx.x) * 4; i < n; i += (int64_t)gridDim.x * NT * 4) {
    if (i + 3 < n) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(g + i);
      sf += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
    } else {
      for (int64_t j = i; j < n; ++j) sf += g[j] * g[j];
    }
    if (++cnt == 64) { s += sf; sf = 0.f; cnt = 0; }
  }
  s += sf;
  s = wave_sum_d(s);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) red[w] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < NT / 64; ++i) t += red[i];
    if (part) part[blockIdx.x] = t;   // summed in block order by sumsq_final_kernel
    else atomicAdd(acc, t);
  }
}

// acc += Σ_b part[b] (one wave: lane l sums blocks l, l+64, ... in order, then a fixed butterfly):
// the deterministic second pass of sumsq_kernel
__global__ __launch_bounds__(64) void sumsq_final_kernel(const double* part, int nb, double* acc) {
  double t = 0.0;
  for (int b = threadIdx.x; b < nb; b += 64) t += part[b];
  t = wave_sum_d(t);
  if (threadIdx.x == 0) acc[0] += t;
}

// One element of clip + AdamW.  Every path of adamw_kernel (two groups a stride apart, one group,
// scalar tail) goes through this, with the roundings spelled out (explicit fma, no contraction), so
// an element's result does not depend on which path it falls in: the update is then invariant to
// how the flat buffer is split into launches (TrainStep(overlap_optimizer=True) runs it per block).
__device__ __forceinline__ void adamw_elem(float& p, float g, float& m, float& v, float coef, float decay, float b1,
                                           float b2, float step, float bc2_sqrt, float eps) {
#pragma clang fp contract(off)
  const float gc = g * coef;
  m = __builtin_fmaf(b1, m, (1.f - b1) * gc);
  v = __builtin_fmaf(b2, v, ((1.f - b2) * gc) * gc);
  const float den = sqrtf(v) / bc2_sqrt + eps;
  p = __builtin_fmaf(-step, m / den, p * decay);
}

template <bool NTL>
__global__ __launch_bounds__(NT) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                 float* __restrict__ m, float* __restrict__ v, bf16* __restrict__ pb,
                                                 int64_t n, float lr, float b1, float b2, float eps, float wd,
                                                 float bc1, float bc2_sqrt, const double* sumsq, float max_norm) {
  float coef = 1.f;
  if (sumsq) {
    const float tn = (float)sqrt(*sumsq);
    coef = fminf(1.f, max_norm / (tn + 1e-6f));
  }
  const float step = lr / bc1;
  const float decay = 1.f - lr * wd;
  auto upd4 = [&](f32x4& pv, const f32x4& gv, f32x4& mv, f32x4& vv) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float pe = pv[e], me = mv[e], ve = vv[e];
      adamw_elem(pe, gv[e], me, ve, coef, decay, b1, b2, step, bc2_sqrt, eps);
      pv[e] = pe;
      mv[e] = me;
      vv[e] = ve;
    }
  };
  // NTL: non-temporal (streaming) loads and stores of the four fp32 arrays
  auto ld = [](const float* q) -> f32x4 {
    if constexpr (NTL) return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(q));
    else return *reinterpret_cast<const f32x4*>(q);
  };
  auto st = [](float* q, f32x4 x) {
    if constexpr (NTL) __builtin_nontemporal_store(x, reinterpret_cast<f32x4*>(q));
    else *reinterpret_cast<f32x4*>(q) = x;
  };
  // bulk: two 4-element groups a grid-stride apart per iteration, all eight 16-B loads issued before
  // the arithmetic (more bytes in flight per lane than the one-group loop)
  const int64_t stride = (int64_t)gridDim.x * NT * 4;
  int64_t i = ((int64_t)blockIdx.x * NT + threadIdx.x) * 4;
  for (; i + stride + 3 < n; i += 2 * stride) {
    f32x4 pv0 = ld(p + i), pv1 = ld(p + i + stride);
    const f32x4 gv0 = ld(g + i), gv1 = ld(g + i + stride);
    f32x4 mv0 = ld(m + i), mv1 = ld(m + i + stride);
    f32x4 vv0 = ld(v + i), vv1 = ld(v + i + stride);
    upd4(pv0, gv0, mv0, vv0);
    upd4(pv1, gv1, mv1, vv1);
    st(p + i, pv0);
    st(m + i, mv0);
    st(v + i, vv0);
    st(p + i + stride, pv1);
    st(m + i + stride, mv1);
    st(v + i + stride, vv1);
    if (pb) {
      store_bf16x4(pb + i, pv0);
      store_bf16x4(pb + i + stride, pv1);
    }
  }
  for (; i < n; i += stride) {
    if (i + 3 < n) {
      f32x4 pv = *reinterpret_cast<f32x4*>(p + i);
      const f32x4 gv = *reinterpret_cast<const f32x4*>(g + i);
      f32x4 mv = *reinterpret_cast<f32x4*>(m + i);
      f32x4 vv = *reinterpret_cast<f32x4*>(v + i);
      upd4(pv, gv, mv, vv);
      *reinterpret_cast<f32x4*>(p + i) = pv;
      *reinterpret_cast<f32x4*>(m + i) = mv;
      *reinterpret_cast<f32x4*>(v + i) = vv;
      if (pb) store_bf16x4(pb + i, pv);
    } else {
      for (int64_t j = i; j < n; ++j) {
        float pv = p[j], mv = m[j], vv = v[j];
        adamw_elem(pv, g[j], mv, vv, coef, decay, b1, b2, step, bc2_sqrt, eps);
        p[j] = pv;
        m[j] = mv;
        v[j] = vv;
        if (pb) pb[j] = (bf16)pv;
      }
    }
  }
}

inline unsigned grid_for(int64_t n) {
  int64_t b = (n / 4 + NT - 1) / NT;
  if (b > 8192) b = 8192;
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace

// ---------------------------------------------------------- row-sparse gradient exchange
// The word-embedding gradient of one rank is non-zero only in the rows of its token ids
// (SURVEY §8e).  Data-parallel ranks exchange (row id, row) lists instead of all-reducing
// the 250,002 x 768 table:  claim the rank's unique ids (first arrival wins a slot),
// extract those rows (zeroing them in place), all-gather the fixed-capacity lists, then
// add every rank's list in rank order (ids unique within a list, so no atomics and the
// same summation order on every rank).
namespace {
__global__ __launch_bounds__(NT) void rows_reset_kernel(int32_t* out_ids, int cap, int32_t* count) {
  const int i = blockIdx.x * NT + threadIdx.x;
  if (i < cap) out_ids[i] = -1;
  if (i == 0) *count = 0;
}
__global__ __launch_bounds__(NT) void rows_claim_kernel(const int64_t* ids, int n, int pad, int32_t* flags,
                                                       int32_t* out_ids, int cap, int32_t* count) {
  const int i = blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  const int64_t id = ids[i];
  if (id == pad || id < 0) return;
  if (atomicCAS(flags + id, 0, 1) == 0) {
    const int slot = atomicAdd(count, 1);
    if (slot < cap) out_ids[slot] = (int32_t)id;
  }
}
// one block per slot: rows[s] = grad[id] (then grad[id] = 0, flags[id] = 0); empty slot -> 0
__global__ __launch_bounds__(NT) void rows_extract_kernel(float* grad, int D, const int32_t* out_ids, int32_t* flags,
                                                         float* rows) {
  const int sidx = blockIdx.x;
  const int id = out_ids[sidx];
  float* dst = rows + (int64_t)sidx * D;
  if (id < 0) {
    for (int c = threadIdx.x * 4; c < D; c += NT * 4) *reinterpret_cast<f32x4*>(dst + c) = f32x4{0.f, 0.f, 0.f, 0.f};
    return;
  }
  float* src = grad + (int64_t)id * D;
  for (int c = threadIdx.x * 4; c < D; c += NT * 4) {
    *reinterpret_cast<f32x4*>(dst + c) = *reinterpret_cast<const f32x4*>(src + c);
    *reinterpret_cast<f32x4*>(src + c) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (threadIdx.x == 0) flags[id] = 0;
}
__global__ __launch_bounds__(NT) void rows_accumulate_kernel(float* grad, int D, const int32_t* ids, const float* rows,
                                                            float scale) {
  const int sidx = blockIdx.x;
  const int id = ids[sidx];
  if (id < 0) return;
  float* dst = grad + (int64_t)id * D;
  const float* src = rows + (int64_t)sidx * D;
  for (int c = threadIdx.x * 4; c < D; c += NT * 4)
    *reinterpret_cast<f32x4*>(dst + c) += *reinterpret_cast<const f32x4*>(src + c) * scale;
}
}  // namespace

extern "C" int ste_rows_extract(const int64_t* ids, int n, int pad_idx, float* grad, int D, int32_t* flags,
                                int32_t* out_ids, float* rows, int cap, int32_t* count, void* stream) {
  if (n < 0 || cap <= 0 || (D & 3) || !grad || !flags || !out_ids || !rows || !count) return STE_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(rows_reset_kernel, dim3((cap + NT - 1) / NT), dim3(NT), 0, s, out_ids, cap, count);
  STE_CHECK_LAUNCH();
  if (n > 0) {
    hipLaunchKernelGGL(rows_claim_kernel, dim3((n + NT - 1) / NT), dim3(NT), 0, s, ids, n, pad_idx, flags, out_ids,
                       cap, count);
    STE_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(rows_extract_kernel, dim3(cap), dim3(NT), 0, s, grad, D, out_ids, flags, rows);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_rows_accumulate(float* grad, int D, const int32_t* ids, const float* rows, int cap, float scale,
                                   void* stream) {
  if (cap <= 0 || (D & 3) || !grad || !ids || !rows) return STE_ERR_ARG;
  hipLaunchKernelGGL(rows_accumulate_kernel, dim3(cap), dim3(NT), 0, (hipStream_t)stream, grad, D, ids, rows, scale);
  STE_CHECK_LAUNCH();
  return 0;
}



extern "C" int ste_text_embed_fwd(const int64_t* ids, int B, int L, int D, int pad_idx, const float* word,
                                  const float* pos, const float* type0, float* out, int32_t* pos_ids, void* stream) {
  if (B <= 0 || L <= 0 || L > 2048 || (D & 3)) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(B), dim3(NT), 0, (hipStream_t)stream, ids, L, D, pad_idx, word, pos, type0,
                     out, pos_ids);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t ste_text_embed_bwd_ws_floats(int B, int L, int D) {
  return ste_colsum_ws_floats((int64_t)B * L, D);
}

extern "C" int ste_text_embed_bwd(const int64_t* ids, const int32_t* pos_ids, const float* dout, int B, int L, int D,
                                  int pad_idx, float* dword, float* dpos, float* dtype0, float* ws, int64_t ws_floats,
                                  void* stream) {
  const int rows = B * L;
  if (rows <= 0 || (D & 3) || D > 1024) return STE_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((rows + EMB_WAVES - 1) / EMB_WAVES);
  const size_t lds = rows <= EMB_LDS_IDS ? (size_t)rows * 4 : 0;
  if (dword) {
    hipLaunchKernelGGL(embed_rows_ordered_kernel<int64_t>, grid, dim3(EMB_WAVES * 64), lds, s, ids, rows, D, pad_idx,
                       dout, dword);
    STE_CHECK_LAUNCH();
  }
  if (dpos) {
    hipLaunchKernelGGL(embed_rows_ordered_kernel<int32_t>, grid, dim3(EMB_WAVES * 64), lds, s, pos_ids, rows, D,
                       pad_idx, dout, dpos);
    STE_CHECK_LAUNCH();
  }
  // token-type row 0: every row's gradient (ordered column sum with a workspace, else atomics)
  if (dtype0) return ste_colsum(dout, 0, rows, D, D, dtype0, ws, ws_floats, stream);
  return 0;
}

extern "C" int ste_sumsq(const float* g, int64_t n, double* acc, double* part, void* stream) {
  if (n <= 0) return 0;
  if (((uintptr_t)g) & 15) return STE_ERR_ARG;
  unsigned gr = grid_for(n);
  if (gr > 2048) gr = 2048;
  hipLaunchKernelGGL(sumsq_kernel, dim3(gr), dim3(NT), 0, (hipStream_t)stream, g, n, acc, part);
  STE_CHECK_LAUNCH();
  if (part) {
    hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, part, (int)gr, acc);
    STE_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int ste_adamw(float* p, const float* g, float* m, float* v, void* p_bf16, int64_t n, float lr, float beta1,
                         float beta2, float eps, float wd, int step, const double* sumsq, float max_norm,
                         void* stream) {
  if (n <= 0) return 0;
  if (step < 1) return STE_ERR_ARG;
  if ((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)m) | ((uintptr_t)v)) & 15) return STE_ERR_ARG;
  if (p_bf16 && (((uintptr_t)p_bf16) & 7)) return STE_ERR_ARG;
  const float bc1 = 1.f - powf(beta1, (float)step);
  const float bc2s = sqrtf(1.f - powf(beta2, (float)step));
  // the fp32 arrays stream through with non-temporal loads / stores (nothing re-reads them before
  // the next step; -3 % per launch, bitwise identical, profiles/r5a_adamw_nt.txt); A/B builds:
  // STE_ADAMW_NT=0 for plain accesses
  const char* ent = STE_AB_ENV("STE_ADAMW_NT");
  if (!(ent && ent[0] == '0'))
    hipLaunchKernelGGL(adamw_kernel<true>, dim3(grid_for(n)), dim3(NT), 0, (hipStream_t)stream, p, g, m, v,
                       (bf16*)p_bf16, n, lr, beta1, beta2, eps, wd, bc1, bc2s, sumsq, max_norm);
  else
  hipLaunchKernelGGL(adamw_kernel<false>, dim3(grid_for(n)), dim3(NT), 0, (hipStream_t)stream, p, g, m, v, (bf16*)p_bf16, n,
                     lr, beta1, beta2, eps, wd, bc1, bc2s, sumsq, max_norm);
  STE_CHECK_LAUNCH();
  return 0;
}

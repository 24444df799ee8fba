// Head-side kernels of EnhancedAudioTextModel (ref = /root/reference/training/trainer_unfreeze.py):
//   AttentivePooling core (ref:171-211) fwd/bwd; CLS / masked-mean pooling (ref:578-580, 621-636)
//   single-query CrossModalAttention core (ref:125-168, called with x.unsqueeze(1) at :653-667)
//   F.normalize (ref:561-563), batch similarity matrix on the fp32 MFMA (ref:1073-1074),
//   AlignmentAwareInfoNCE (ref:702-742) fwd/bwd.
// These are small (rows = batch), latency-bound kernels; the big sequence-length
// projections around them run through ste_gemm.
#include "common.h"
#include "../../include/ste.h"

namespace {

constexpr int NT = 256;

STE_DEV float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;
}
STE_DEV float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = -INFINITY;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s = fmaxf(s, red[i]);
  return s;
}

// 4 consecutive elements of a bf16 or fp32 row (the pooling kernels run on the bf16 audio states
// and on the fp32 text states, see ste_attn_pool_fwd_f32)
STE_DEV f32x4 ld4(const bf16* p) { return load_bf16x4(p); }
STE_DEV f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
STE_DEV void st4(bf16* p, f32x4 v) { store_bf16x4(p, v); }
STE_DEV void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

template <typename T>
STE_DEV float row_dot(const T* a, const float* b, int n, int lane) {
  float acc = 0.f;
  for (int c = lane * 4; c < n; c += 256) {
    f32x4 x = ld4(a + c);
    f32x4 y = *reinterpret_cast<const f32x4*>(b + c);
    acc += x[0] * y[0] + x[1] * y[1] + x[2] * y[2] + x[3] * y[3];
  }
  return wave_sum(acc);
}

// ------------------------------------------------------------ attentive pooling
// Forward, three launches so the [B*L, H] read is spread over the chip (one block per sample
// left 3/4 of the CUs idle and walked L rows serially):
//   pool_score_kernel   s_l = t_l·w2 + b2 (masked -> -1e9), one wave per row   grid (B, ceil(L/16))
//   pool_softmax_kernel w_l = softmax_l(s)                                     grid B
//   pool_wsum_kernel    pooled[c] = Σ_l w_l h_l[c]: 8 waves split the rows,    grid (B, ceil(H/256))
//                       partials summed in wave order (deterministic)
constexpr int POOL_SC_ROWS = 16;
constexpr int POOL_WS_NT = 512;

template <typename T>
__global__ __launch_bounds__(NT) void pool_score_kernel(const T* t, const float* w2, const float* b2,
                                                      const int32_t* mask, int L, int Hh, float* sc) {
  const int b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int l1 = min(L, (int)(blockIdx.y + 1) * POOL_SC_ROWS);
  for (int l = blockIdx.y * POOL_SC_ROWS + w; l < l1; l += NT / 64) {
    float s = row_dot(t + (int64_t)(b * L + l) * Hh, w2, Hh, lane) + b2[0];
    if (mask && mask[b * L + l] == 0) s = -1e9f;
    if (lane == 0) sc[b * L + l] = s;
  }
}

__global__ __launch_bounds__(NT) void pool_softmax_kernel(int L, float* sc) {
  __shared__ float red[8];
  float* r = sc + (int64_t)blockIdx.x * L;
  const int tid = threadIdx.x;
  float mx = -INFINITY;
  for (int l = tid; l < L; l += NT) mx = fmaxf(mx, r[l]);
  mx = block_max(mx, red);
  float sum = 0.f;
  for (int l = tid; l < L; l += NT) sum += __expf(r[l] - mx);
  sum = block_sum(sum, red);
  const float inv = 1.0f / sum;
  for (int l = tid; l < L; l += NT) r[l] = __expf(r[l] - mx) * inv;
}

template <typename T>
__global__ __launch_bounds__(POOL_WS_NT) void pool_wsum_kernel(const T* h, const float* weights, int L, int H,
                                                             float* pooled, bf16* pooled_bf16) {
  extern __shared__ float wl[];  // L weights
  __shared__ f32x4 part[POOL_WS_NT / 64][64];
  constexpr int NW = POOL_WS_NT / 64;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int l = tid; l < L; l += POOL_WS_NT) wl[l] = weights[b * L + l];
  __syncthreads();
  const int c = blockIdx.y * 256 + lane * 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (c < H) {
    const T* hp = h + (int64_t)b * L * H + c;
#pragma unroll 4
    for (int l = w; l < L; l += NW) acc += ld4(hp + (int64_t)l * H) * wl[l];
  }
  part[w][lane] = acc;
  __syncthreads();
  if (w == 0 && c < H) {
    f32x4 s = part[0][lane];
#pragma unroll
    for (int i = 1; i < NW; ++i) s += part[i][lane];
    *reinterpret_cast<f32x4*>(pooled + (int64_t)b * H + c) = s;
    if (pooled_bf16) store_bf16x4(pooled_bf16 + (int64_t)b * H + c, s);
  }
}

// Backward, four launches spread over (batch, row chunks) so the [B*L, H] reads fill the chip:
//   pool_dp_kernel     dP[l] = h_l·dpooled                               grid (B, ceil(L/16))
//   pool_dscore_kernel ds[l] = w_l (dP[l] - Σ_j w_j dP[j]), db2 += Σ ds   grid B
//   pool_dz_kernel     dh_l += w_l dpooled;  dz_l = ds_l w2 (1 - t_l²) (bf16 hi [+ lo]);
//                      per-chunk partials of Σ_l ds_l t_l, Σ_l dz_l      grid (B, ceil(L/64|16))
//   pool_dw_kernel     dw2 += Σ partials, db1 += Σ partials (chunk order) grid ceil(2Hh/64)
// Σ_l ds_l = 0 (softmax), so the scorer's bias gradient Σ_l dz_l is a small difference of large
// terms: it is summed from the fp32 dz here, never from the bf16-rounded copy, and the optional
// low half dz_lo = bf16(dz - bf16(dz)) lets the weight-gradient GEMM see dz to ~16 bits.  The
// column sums go through a partials buffer, not atomics: 2·Hh atomics per block onto the same
// 2·Hh addresses serialised in L2 and made the audio launch atomic-bound (~180 µs); the
// two-level sum is also run-to-run deterministic.
constexpr int POOL_DP_ROWS = 16;
// row chunk of pool_dz: 64 rows, or 16 when that leaves fewer than 512 blocks (text: 128 x 64 rows)
static int pool_dz_rows(int B, int L) { return (int64_t)B * ((L + 63) / 64) >= 512 ? 64 : 16; }
constexpr int POOL_DW_NT = 1024;

template <typename T>
__global__ __launch_bounds__(NT) void pool_dp_kernel(const T* h, const float* dpooled, int L, int H, float* dp_out) {
  const int b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* dp = dpooled + (int64_t)b * H;
  const int l1 = min(L, (int)(blockIdx.y + 1) * POOL_DP_ROWS);
  for (int l = blockIdx.y * POOL_DP_ROWS + w; l < l1; l += NT / 64) {
    const float s = row_dot(h + (int64_t)(b * L + l) * H, dp, H, lane);
    if (lane == 0) dp_out[b * L + l] = s;
  }
}

// masked positions get ds = 0 (the forward's masked_fill cuts their score gradient): that only
// matters for an all-masked sample, whose weights are uniform rather than 0 at those positions
__global__ __launch_bounds__(NT) void pool_dscore_kernel(const float* weights, const int32_t* mask, int L, float* dsc,
                                                       float* db2, float* db2_part) {
  __shared__ float red[8];
  const int b = blockIdx.x, tid = threadIdx.x;
  float acc = 0.f;
  for (int l = tid; l < L; l += NT) acc += weights[b * L + l] * dsc[b * L + l];
  const float tot = block_sum(acc, red);
  float dbs = 0.f;
  for (int l = tid; l < L; l += NT) {
    float ds = weights[b * L + l] * (dsc[b * L + l] - tot);
    if (mask && mask[b * L + l] == 0) ds = 0.f;
    dsc[b * L + l] = ds;
    dbs += ds;
  }
  dbs = block_sum(dbs, red);
  if (tid == 0 && db2) {   // the sample's term; summed over samples in order by the host's second pass
    if (db2_part) db2_part[b] = dbs;
    else atomicAdd(db2, dbs);
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void pool_dz_kernel(const T* t, const float* w2, const float* weights,
                                                   const float* dpooled, const float* dsc, int L, int Hh, int H,
                                                   float* dh, T* dz, bf16* dz_lo, float* part, int rows) {
  __shared__ f32x4 red[2 * NT];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int l0 = blockIdx.y * rows, l1 = min(L, l0 + rows);
  // dh[l][c] += w[l] * dpooled[c]
  const float* dp = dpooled + (int64_t)b * H;
  for (int c = tid * 4; c < H; c += NT * 4) {
    const f32x4 d = *reinterpret_cast<const f32x4*>(dp + c);
#pragma unroll 4
    for (int l = l0; l < l1; ++l) {
      f32x4* o = reinterpret_cast<f32x4*>(dh + (int64_t)(b * L + l) * H + c);
      *o = *o + d * weights[b * L + l];
    }
  }
  // dz rows: the block's threads are (groups x Hh/4 column quads); group g takes rows l0+g, +groups, ...
  const int cq = Hh >> 2, groups = NT / cq, g = tid / cq, k = (tid - g * cq) * 4;
  f32x4 g2 = {0.f, 0.f, 0.f, 0.f}, g1 = {0.f, 0.f, 0.f, 0.f};
  if (g < groups) {
    const f32x4 wv = *reinterpret_cast<const f32x4*>(w2 + k);
#pragma unroll 2
    for (int l = l0 + g; l < l1; l += groups) {
      const int64_t off = (int64_t)(b * L + l) * Hh + k;
      const f32x4 tv = ld4(t + off);
      const float ds = dsc[b * L + l];
      g2 += tv * ds;
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = ds * wv[e] * (1.f - tv[e] * tv[e]);
      g1 += o;
      if constexpr (sizeof(T) == 2) {
        if (dz_lo) store_bf16x4_split((bf16*)dz + off, dz_lo + off, o);
        else st4(dz + off, o);
      } else {
        st4(dz + off, o);
      }
    }
  }
  red[2 * tid] = g2;
  red[2 * tid + 1] = g1;
  __syncthreads();
  if (tid < cq) {
    f32x4 s2 = red[2 * tid], s1 = red[2 * tid + 1];
    for (int i = 1; i < groups; ++i) { s2 += red[2 * (i * cq + tid)]; s1 += red[2 * (i * cq + tid) + 1]; }
    float* pr = part + (int64_t)(b * gridDim.y + blockIdx.y) * 2 * Hh;
    *reinterpret_cast<f32x4*>(pr + k) = s2;
    *reinterpret_cast<f32x4*>(pr + Hh + k) = s1;
  }
}

// column sums of the [nrows, 2*Hh] partials: 16 waves stride the rows, one column per lane,
// wave partials summed in order; dw2 (cols < Hh) and db1 (cols >= Hh) accumulated (+=).
__global__ __launch_bounds__(POOL_DW_NT) void pool_dw_kernel(const float* part, int nrows, int Hh, float* dw2,
                                                           float* db1) {
  constexpr int NW = POOL_DW_NT / 64;
  __shared__ float red[NW][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, col = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (col < 2 * Hh) {
#pragma unroll 4
    for (int r = w; r < nrows; r += NW) s += part[(int64_t)r * 2 * Hh + col];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && col < 2 * Hh) {
    float tot = red[0][lane];
    for (int i = 1; i < NW; ++i) tot += red[i][lane];
    if (col < Hh) { if (dw2) dw2[col] += tot; }
    else if (db1) db1[col - Hh] += tot;
  }
}

// ------------------------------------------- CLS / masked-mean pooling (no scorer)
// use_attentive_pooling=False (ref:578-580 text CLS, :621-636 audio masked mean).
// weights[b][l] = CLS: [l == 0];  mean: mask[l] / max(sum(mask), 1e-9) (all-masked rows pool to 0).
template <typename T>
__global__ __launch_bounds__(NT) void mean_pool_fwd_kernel(const T* h, const int32_t* mask, int L, int H, int cls,
                                                         float* weights, float* pooled, bf16* pooled_bf16) {
  extern __shared__ float sc[];  // L weights
  __shared__ float red[8];
  const int b = blockIdx.x, tid = threadIdx.x;
  float cnt = 0.f;
  for (int l = tid; l < L; l += NT) {
    const float m = cls ? (l == 0 ? 1.f : 0.f) : (mask ? (mask[b * L + l] != 0 ? 1.f : 0.f) : 1.f);
    sc[l] = m;
    cnt += m;
  }
  cnt = block_sum(cnt, red);  // contains a barrier: sc is complete
  const float inv = cls ? 1.f : 1.f / fmaxf(cnt, 1e-9f);
  for (int l = tid; l < L; l += NT) weights[b * L + l] = sc[l] * inv;
  const int Lr = cls ? 1 : L;  // CLS reads one row
  for (int c = tid * 4; c < H; c += NT * 4) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int l = 0; l < Lr; ++l)
      if (sc[l] != 0.f) acc += ld4(h + (int64_t)(b * L + l) * H + c);
    acc *= inv;
    *reinterpret_cast<f32x4*>(pooled + (int64_t)b * H + c) = acc;
    if (pooled_bf16) store_bf16x4(pooled_bf16 + (int64_t)b * H + c, acc);
  }
}

// dh[b][l][:] += weights[b][l] * dpooled[b][:]; grid (B, ceil(L/16)), rows with weight 0 untouched.
__global__ __launch_bounds__(NT) void weighted_pool_bwd_kernel(const float* weights, const float* dpooled, int L,
                                                             int H, float* dh) {
  const int b = blockIdx.x, l0 = blockIdx.y * 16;
  const float* dp = dpooled + (int64_t)b * H;
  for (int l = l0; l < min(l0 + 16, L); ++l) {
    const float wt = weights[b * L + l];
    if (wt == 0.f) continue;
    for (int c = threadIdx.x * 4; c < H; c += NT * 4) {
      f32x4* o = reinterpret_cast<f32x4*>(dh + (int64_t)(b * L + l) * H + c);
      *o = *o + *reinterpret_cast<const f32x4*>(dp + c) * wt;
    }
  }
}

// ---------------------------------------------------- single-query cross attention
// scores/probs layout: [B][nh][S]
// CrossModalAttention with NQ single-vector queries per sample sharing the same keys/values
// (the positive and the corrupted transcript's text->audio calls, ref:525-542, read one audio
// K/V): one block per (sample, head), so B*nh blocks fill the chip.  Query qi of sample b is
// row qi*B + b of q / out / dout / dq and of the probs ((qi*B + b)*nh + head)*S; its dropout
// uses seed qi and the index (b*nh + head)*S + s (the per-call layout of one query set).
// Rows of K/V are read with 16-B (8 x bf16) loads; the PV / dK / dV passes put 4 columns on a
// lane and spread the key rows over the block's row groups.
template <int NQ>
__global__ __launch_bounds__(NT) void xattn_fwd_kernel(const float* q, const bf16* k, const bf16* v, int64_t ldkv,
                                                     const int32_t* mask, int B, int S, int P, int nh, float scale,
                                                     float drop_p, uint64_t seed0, uint64_t seed1, float* probs,
                                                     float* out) {
  extern __shared__ float sp[];  // NQ * S
  __shared__ float sq[NQ][256];
  __shared__ float red[NQ][NT / 64];
  __shared__ f32x4 racc[NT];
  const int b = blockIdx.x, hh = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int dh = P / nh, c0 = hh * dh;
  for (int c = tid; c < NQ * dh; c += NT) sq[c / dh][c % dh] = q[(int64_t)((c / dh) * B + b) * P + c0 + c % dh];
  __syncthreads();
  // scores
  for (int s = tid; s < S; s += NT) {
    const bf16* kr = k + (int64_t)(b * S + s) * ldkv + c0;
    float acc[NQ];
#pragma unroll
    for (int qi = 0; qi < NQ; ++qi) acc[qi] = 0.f;
    for (int d = 0; d < dh; d += 8) {
      const bf16x8 x = *reinterpret_cast<const bf16x8*>(kr + d);
#pragma unroll
      for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int qi = 0; qi < NQ; ++qi) acc[qi] += (float)x[e] * sq[qi][d + e];
    }
    const bool masked = mask && mask[b * S + s] == 0;
#pragma unroll
    for (int qi = 0; qi < NQ; ++qi) sp[qi * S + s] = masked ? -1e9f : acc[qi] * scale;
  }
  __syncthreads();
  // softmax per query over the block
  float mx[NQ], sm[NQ];
#pragma unroll
  for (int qi = 0; qi < NQ; ++qi) {
    float m = -INFINITY;
    for (int s = tid; s < S; s += NT) m = fmaxf(m, sp[qi * S + s]);
    m = wave_max(m);
    if (lane == 0) red[qi][w] = m;
  }
  __syncthreads();
#pragma unroll
  for (int qi = 0; qi < NQ; ++qi) {
    mx[qi] = fmaxf(fmaxf(red[qi][0], red[qi][1]), fmaxf(red[qi][2], red[qi][3]));
    float t = 0.f;
    for (int s = tid; s < S; s += NT) t += __expf(sp[qi * S + s] - mx[qi]);
    sm[qi] = wave_sum(t);
  }
  __syncthreads();
#pragma unroll
  for (int qi = 0; qi < NQ; ++qi)
    if (lane == 0) red[qi][w] = sm[qi];
  __syncthreads();
  const uint32_t thresh = (uint32_t)(drop_p * 4294967296.0);
  const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
#pragma unroll
  for (int qi = 0; qi < NQ; ++qi) {
    const float inv = 1.f / (red[qi][0] + red[qi][1] + red[qi][2] + red[qi][3]);
    const uint64_t sd = qi ? seed1 : seed0;
    float* pr = probs + ((int64_t)(qi * B + b) * nh + hh) * S;
    for (int s = tid; s < S; s += NT) {
      float pv = __expf(sp[qi * S + s] - mx[qi]) * inv;
      pr[s] = pv;
      if (drop_p > 0.f) pv *= drop_scale(sd, ((uint64_t)b * nh + hh) * S + s, thresh, inv_keep);
      sp[qi * S + s] = pv;
    }
  }
  __syncthreads();
  // out = P·V: lane (row group rg, column quad cq)
  const int nq4 = dh >> 2, RG = NT / nq4;
  const int cq = tid % nq4, rg = tid / nq4;
  f32x4 acc[NQ];
#pragma unroll
  for (int qi = 0; qi < NQ; ++qi) acc[qi] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (rg < RG)
    for (int s = rg; s < S; s += RG) {
      const f32x4 vv = load_bf16x4(v + (int64_t)(b * S + s) * ldkv + c0 + 4 * cq);
#pragma unroll
      for (int qi = 0; qi < NQ; ++qi) acc[qi] += vv * sp[qi * S + s];
    }
#pragma unroll
  for (int qi = 0; qi < NQ; ++qi) {
    racc[tid] = acc[qi];
    __syncthreads();
    if (tid < nq4) {
      f32x4 t = racc[tid];
      for (int r = 1; r < RG; ++r) t += racc[r * nq4 + tid];
      *reinterpret_cast<f32x4*>(out + (int64_t)(qi * B + b) * P + c0 + 4 * tid) = t;
    }
    __syncthreads();
  }
}

// OUT_BF16 = false: dk, dv are fp32 and ACCUMULATED (+=) once for all NQ queries.
// OUT_BF16 = true:  dk, dv are bf16 and WRITTEN (the block is their only writer), and the fp32
//   column sums of this block's dk / dv rows go to part[b][c0 + c] / part[b][P + c0 + c]
//   (row-group partials summed in order), so the key/value bias gradient is a [B, 2P] column
//   sum instead of a zero-fill + RMW + cast + colsum pass over fp32 [B*S, 2P].
// dq is written.
template <int NQ, bool OUT_BF16>
__global__ __launch_bounds__(NT) void xattn_bwd_kernel(const float* q, const bf16* k, const bf16* v, int64_t ldkv,
                                                     const float* probs, const float* dout, const int32_t* mask,
                                                     int B, int S, int P, int nh, float scale, float drop_p,
                                                     uint64_t seed0, uint64_t seed1, float* dq, void* dk_, void* dv_,
                                                     int64_t lddkv, float* part) {
  extern __shared__ float sds[];  // NQ * S: dp, then ds
  __shared__ float sq[NQ][256], sdo[NQ][256], red[NQ][NT / 64];
  __shared__ f32x4 racc[NT];
  const int b = blockIdx.x, hh = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int dh = P / nh, c0 = hh * dh;
  const uint32_t thresh = (uint32_t)(drop_p * 4294967296.0);
  const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  const uint64_t drop_base = ((uint64_t)b * nh + hh) * S;
  for (int c = tid; c < NQ * dh; c += NT) {
    const int qi = c / dh, cc = c % dh;
    sq[qi][cc] = q[(int64_t)(qi * B + b) * P + c0 + cc];
    sdo[qi][cc] = dout[(int64_t)(qi * B + b) * P + c0 + cc];
  }
  __syncthreads();
  // dp[qi][s] = v[s]·dout_qi (times the dropout scale)
  for (int s = tid; s < S; s += NT) {
    const bf16* vr = v + (int64_t)(b * S + s) * ldkv + c0;
    float acc[NQ];
#pragma unroll
    for (int qi = 0; qi < NQ; ++qi) acc[qi] = 0.f;
    for (int d = 0; d < dh; d += 8) {
      const bf16x8 x = *reinterpret_cast<const bf16x8*>(vr + d);
#pragma unroll
      for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int qi = 0; qi < NQ; ++qi) acc[qi] += (float)x[e] * sdo[qi][d + e];
    }
#pragma unroll
    for (int qi = 0; qi < NQ; ++qi) {
      if (drop_p > 0.f) acc[qi] *= drop_scale(qi ? seed1 : seed0, drop_base + s, thresh, inv_keep);
      sds[qi * S + s] = acc[qi];
    }
  }
  __syncthreads();
  float rs[NQ];
#pragma unroll
  for (int qi = 0; qi < NQ; ++qi) {
    const float* pr = probs + ((int64_t)(qi * B + b) * nh + hh) * S;
    float part = 0.f;
    for (int s = tid; s < S; s += NT) part += pr[s] * sds[qi * S + s];
    part = wave_sum(part);
    if (lane == 0) red[qi][w] = part;
  }
  __syncthreads();
#pragma unroll
  for (int qi = 0; qi < NQ; ++qi) rs[qi] = red[qi][0] + red[qi][1] + red[qi][2] + red[qi][3];
#pragma unroll
  for (int qi = 0; qi < NQ; ++qi) {
    const float* pr = probs + ((int64_t)(qi * B + b) * nh + hh) * S;
    for (int s = tid; s < S; s += NT)   // masked keys: no score gradient (masked_fill's backward)
      sds[qi * S + s] = (mask && mask[b * S + s] == 0) ? 0.f : pr[s] * (sds[qi * S + s] - rs[qi]) * scale;
  }
  __syncthreads();
  // dq[qi] = Σ_s ds k[s];  dk[s] += Σ_qi ds q_qi;  dv[s] += Σ_qi p' dout_qi  (4 columns per lane)
  const int nq4 = dh >> 2, RG = NT / nq4;
  const int cq = tid % nq4, rg = tid / nq4, cc = 4 * cq;
  f32x4 dqa[NQ];
#pragma unroll
  for (int qi = 0; qi < NQ; ++qi) dqa[qi] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 csk = {0.f, 0.f, 0.f, 0.f}, csv = {0.f, 0.f, 0.f, 0.f};
  if (rg < RG) {
    f32x4 qv[NQ], dov[NQ];
#pragma unroll
    for (int qi = 0; qi < NQ; ++qi) {
      qv[qi] = f32x4{sq[qi][cc], sq[qi][cc + 1], sq[qi][cc + 2], sq[qi][cc + 3]};
      dov[qi] = f32x4{sdo[qi][cc], sdo[qi][cc + 1], sdo[qi][cc + 2], sdo[qi][cc + 3]};
    }
    for (int s = rg; s < S; s += RG) {
      const f32x4 kk = load_bf16x4(k + (int64_t)(b * S + s) * ldkv + c0 + cc);
      f32x4 dkv = {0.f, 0.f, 0.f, 0.f}, dvv = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int qi = 0; qi < NQ; ++qi) {
        const float ds = sds[qi * S + s];
        float pd = probs[((int64_t)(qi * B + b) * nh + hh) * S + s];
        if (drop_p > 0.f) pd *= drop_scale(qi ? seed1 : seed0, drop_base + s, thresh, inv_keep);
        dqa[qi] += kk * ds;
        dkv += qv[qi] * ds;
        dvv += dov[qi] * pd;
      }
      const int64_t off = (int64_t)(b * S + s) * lddkv + c0 + cc;
      if constexpr (OUT_BF16) {
        store_bf16x4((bf16*)dk_ + off, dkv);
        store_bf16x4((bf16*)dv_ + off, dvv);
        csk += dkv;
        csv += dvv;
      } else {
        *reinterpret_cast<f32x4*>((float*)dk_ + off) += dkv;
        *reinterpret_cast<f32x4*>((float*)dv_ + off) += dvv;
      }
    }
  }
  if constexpr (OUT_BF16) {
#pragma unroll
    for (int kv = 0; kv < 2; ++kv) {
      racc[tid] = kv ? csv : csk;
      __syncthreads();
      if (tid < nq4) {
        f32x4 t = racc[tid];
        for (int r = 1; r < RG; ++r) t += racc[r * nq4 + tid];
        *reinterpret_cast<f32x4*>(part + (int64_t)b * 2 * P + kv * P + c0 + 4 * tid) = t;
      }
      __syncthreads();
    }
  }
#pragma unroll
  for (int qi = 0; qi < NQ; ++qi) {
    racc[tid] = dqa[qi];
    __syncthreads();
    if (tid < nq4) {
      f32x4 t = racc[tid];
      for (int r = 1; r < RG; ++r) t += racc[r * nq4 + tid];
      *reinterpret_cast<f32x4*>(dq + (int64_t)(qi * B + b) * P + c0 + 4 * tid) = t;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- L2 normalize
__global__ __launch_bounds__(NT) void l2norm_fwd_kernel(const float* x, int cols, float* y, float* norms) {
  __shared__ float red[8];
  const int r = blockIdx.x;
  float s = 0.f;
  for (int c = threadIdx.x; c < cols; c += NT) { float v = x[(int64_t)r * cols + c]; s += v * v; }
  s = block_sum(s, red);
  const float n = fmaxf(sqrtf(s), 1e-12f);
  if (threadIdx.x == 0) norms[r] = sqrtf(s);
  for (int c = threadIdx.x; c < cols; c += NT) y[(int64_t)r * cols + c] = x[(int64_t)r * cols + c] / n;
}
__global__ __launch_bounds__(NT) void l2norm_bwd_kernel(const float* y, const float* norms, const float* dy, int cols,
                                                      float* dx) {
  __shared__ float red[8];
  const int r = blockIdx.x;
  const float nr = norms[r];
  float s = 0.f;
  for (int c = threadIdx.x; c < cols; c += NT) s += y[(int64_t)r * cols + c] * dy[(int64_t)r * cols + c];
  s = block_sum(s, red);
  const float inv = 1.f / fmaxf(nr, 1e-12f);
  const bool clamped = nr < 1e-12f;
  for (int c = threadIdx.x; c < cols; c += NT) {
    const int64_t i = (int64_t)r * cols + c;
    dx[i] = clamped ? dy[i] * inv : (dy[i] - y[i] * s) * inv;
  }
}

// ------------------------------------------- batch similarity on the fp32 MFMA
// S[i][j] = Σ_k A[i][k] T[j][k]; one wave per 16x16 output tile (v_mfma_f32_16x16x4_f32).
__global__ __launch_bounds__(64) void similarity_kernel(const float* A, const float* Tm, int B, int NTt, int P,
                                                      float* S) {
  const int lane = threadIdx.x;
  const int i0 = blockIdx.x * 16, j0 = blockIdx.y * 16;
  const int ia = i0 + (lane & 15), jb = j0 + (lane & 15), kk = lane >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < P; k += 4) {
    const float a = (ia < B && k + kk < P) ? A[(int64_t)ia * P + k + kk] : 0.f;
    const float bv = (jb < NTt && k + kk < P) ? Tm[(int64_t)jb * P + k + kk] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + (lane >> 4) * 4 + r, j = j0 + (lane & 15);
    if (i < B && j < NTt) S[(int64_t)i * NTt + j] = acc[r];
  }
}

// ------------------------------------------------------------------- pair loss
__global__ __launch_bounds__(NT) void pair_loss_fwd_kernel(const float* S, int64_t ldS, int off_neg, const float* align,
                                                         int B, int L, float tau, float aw, float gamma, float* s_pos,
                                                         float* s_neg, float* loss) {
  __shared__ float red[8];
  float acc = 0.f, pen = 0.f;
  for (int i = threadIdx.x; i < B; i += NT) {
    const float sp = S[(int64_t)i * ldS + i], sn = S[(int64_t)i * ldS + off_neg + i];
    s_pos[i] = sp;
    s_neg[i] = sn;
    const float x = (sn - sp) / tau;
    float ce = fmaxf(x, 0.f) + log1pf(__expf(-fabsf(x)));
    if (align) {
      float m = 0.f;
      for (int l = 0; l < L; ++l) m += align[(int64_t)i * L + l];
      m /= (float)L;
      ce *= 1.f - sigmoidf_(m) * aw;
    }
    acc += ce;
    pen += fmaxf(sn, 0.f);
  }
  acc = block_sum(acc, red);
  pen = block_sum(pen, red);
  if (threadIdx.x == 0) loss[0] = acc / (float)B + (gamma > 0.f ? gamma * pen / (float)B : 0.f);
}

__global__ __launch_bounds__(NT) void pair_loss_bwd_kernel(const float* s_pos, const float* s_neg, const float* align,
                                                         int B, int L, float tau, float aw, float gamma,
                                                         const float* gscale, float* ds_pos, float* ds_neg,
                                                         float* dalign) {
  const float gs = gscale ? gscale[0] : 1.f;
  for (int i = blockIdx.x * NT + threadIdx.x; i < B; i += gridDim.x * NT) {
    const float sp = s_pos[i], sn = s_neg[i];
    const float x = (sn - sp) / tau;
    const float ce = fmaxf(x, 0.f) + log1pf(__expf(-fabsf(x)));
    float factor = 1.f, sg = 0.f;
    if (align) {
      float m = 0.f;
      for (int l = 0; l < L; ++l) m += align[(int64_t)i * L + l];
      m /= (float)L;
      sg = sigmoidf_(m);
      factor = 1.f - sg * aw;
    }
    const float dce = gs * factor / (float)B;
    const float dx = sigmoidf_(x) * dce / tau;
    ds_pos[i] = -dx;
    ds_neg[i] = dx + ((gamma > 0.f && sn > 0.f) ? gs * gamma / (float)B : 0.f);
    if (align && dalign) {
      const float da = gs * ce / (float)B * (-aw) * sg * (1.f - sg) / (float)L;
      for (int l = 0; l < L; ++l) dalign[(int64_t)i * L + l] = da;
    }
  }
}

// d(aud), d(txt_pos), d(txt_neg) from ds_pos/ds_neg through s = <aud, txt>
__global__ __launch_bounds__(NT) void pair_sim_bwd_kernel(const float* a, const float* tp, const float* tn,
                                                        const float* ds_pos, const float* ds_neg, int P, float* da,
                                                        float* dtp, float* dtn) {
  const int i = blockIdx.x;
  const float gp = ds_pos[i], gn = ds_neg[i];
  for (int c = threadIdx.x; c < P; c += NT) {
    const int64_t o = (int64_t)i * P + c;
    da[o] = gp * tp[o] + gn * tn[o];
    dtp[o] = gp * a[o];
    dtn[o] = gn * a[o];
  }
}

// ------------------------------------ data-parallel global similarity
// Rows of the global matrix S = A_g·[Tpos_g ; Tneg_g]ᵀ ([NB x 2NB], NB = ranks x local batch),
// one block per row i: the reference's metrics on its diagonals (ref train_epoch :1120-1161:
// to_human_readable = sigmoid(s/0.1), clean / corrupt / gap), the pair accuracy s_pos > s_neg and
// the in-batch top-1 retrieval hit (argmax over the NB clean transcripts == i).
// acc (fp64, accumulated): [Σ sigmoid(s_pos/τ), Σ sigmoid(s_neg/τ), Σ [s_pos > s_neg], Σ hit, rows,
//                            loss_w · Σ_r losses[r] (the ranks' batch losses x local batch)]
__global__ __launch_bounds__(NT) void pair_metrics_kernel(const float* S, int64_t ldS, int NB, int off_neg, float tau,
                                                        const float* losses, int nloss, float loss_w, double* acc) {
  __shared__ float rv[8];
  __shared__ int ri[8];
  const int i = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* row = S + (int64_t)i * ldS;
  float best = -INFINITY;
  int bj = 0x7fffffff;
  for (int j = tid; j < NB; j += NT) {
    const float v = row[j];
    if (v > best || (v == best && j < bj)) { best = v; bj = j; }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oj = __shfl_xor(bj, o, 64);
    if (ov > best || (ov == best && oj < bj)) { best = ov; bj = oj; }
  }
  if (lane == 0) { rv[w] = best; ri[w] = bj; }
  __syncthreads();
  if (tid == 0) {
    for (int k = 1; k < NT / 64; ++k)
      if (rv[k] > best || (rv[k] == best && ri[k] < bj)) { best = rv[k]; bj = ri[k]; }
    const float sp = row[i], sn = row[off_neg + i];
    atomicAdd(acc + 0, (double)sigmoidf_(sp / tau));
    atomicAdd(acc + 1, (double)sigmoidf_(sn / tau));
    atomicAdd(acc + 2, sp > sn ? 1.0 : 0.0);
    atomicAdd(acc + 3, bj == i ? 1.0 : 0.0);
    atomicAdd(acc + 4, 1.0);
    if (i == 0 && losses) {
      double ls = 0.0;
      for (int r = 0; r < nloss; ++r) ls += (double)losses[r];
      atomicAdd(acc + 5, ls * (double)loss_w);
    }
  }
}

// Optional in-batch-negative InfoNCE (off by default: the reference's loss has no cross-sample
// term): local audio rows i against all NB clean transcripts of the global batch,
// logits S[i][j]/τ, target row0 + i.  loss += w·gs/B Σ_i CE_i;  dS[i][j] = w·gs/B (softmax_j - δ)/τ.
__global__ __launch_bounds__(NT) void inbatch_ce_kernel(const float* S, int64_t ldS, int B, int NB, int row0, float tau,
                                                      float weight, const float* gscale, float* loss, float* dS,
                                                      int64_t lddS) {
  __shared__ float red[8];
  const int i = blockIdx.x, tid = threadIdx.x;
  const float* row = S + (int64_t)i * ldS;
  const float it = 1.0f / tau;
  float mx = -INFINITY;
  for (int j = tid; j < NB; j += NT) mx = fmaxf(mx, row[j] * it);
  mx = block_max(mx, red);
  float sum = 0.f;
  for (int j = tid; j < NB; j += NT) sum += __expf(row[j] * it - mx);
  sum = block_sum(sum, red);
  const float lse = mx + __logf(sum);
  const float c = weight * (gscale ? gscale[0] : 1.f) / (float)B;
  const int t = row0 + i;
  for (int j = tid; j < NB; j += NT) {
    const float p = __expf(row[j] * it - lse);
    dS[(int64_t)i * lddS + j] = c * (p - (j == t ? 1.f : 0.f)) * it;
  }
  if (tid == 0) atomicAdd(loss, c * (lse - row[t] * it) / (gscale ? gscale[0] : 1.f));
}

// out[r][p] += Σ_c X[r*sxr + c*sxc] · Y[c][p]  (small fp32 products of the in-batch backward:
// dA = dS·T_g and dT_g = dSᵀ·A); one block per output row.
__global__ __launch_bounds__(NT) void rowmat_f32_kernel(const float* X, int64_t sxr, int64_t sxc, const float* Y, int C,
                                                      int P, float* out) {
  const int r = blockIdx.x;
  for (int p0 = threadIdx.x * 4; p0 < P; p0 += NT * 4) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < C; ++c) {
      const float x = X[(int64_t)r * sxr + (int64_t)c * sxc];
      acc += x * *reinterpret_cast<const f32x4*>(Y + (int64_t)c * P + p0);
    }
    f32x4* o = reinterpret_cast<f32x4*>(out + (int64_t)r * P + p0);
    *o = *o + acc;
  }
}

}  // namespace

template <typename T>
static int attn_pool_fwd(const T* t, const float* w2, const float* b2, const T* h, const int32_t* mask, int B, int L,
                         int Hh, int H, float* weights, float* pooled, bf16* pooled_bf16, hipStream_t s) {
  if (B <= 0 || L <= 0 || (Hh & 3) || (H & 3) || L > 8192) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(pool_score_kernel<T>, dim3(B, (L + POOL_SC_ROWS - 1) / POOL_SC_ROWS), dim3(NT), 0, s, t, w2, b2,
                     mask, L, Hh, weights);
  STE_CHECK_LAUNCH();
  hipLaunchKernelGGL(pool_softmax_kernel, dim3(B), dim3(NT), 0, s, L, weights);
  STE_CHECK_LAUNCH();
  hipLaunchKernelGGL(pool_wsum_kernel<T>, dim3(B, (H + 255) / 256), dim3(POOL_WS_NT), L * sizeof(float), s, h, weights,
                     L, H, pooled, pooled_bf16);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_attn_pool_fwd(const void* t, const float* w2, const float* b2, const void* h, const int32_t* mask,
                                 int B, int L, int Hh, int H, float* weights, float* pooled, void* pooled_bf16,
                                 void* stream) {
  return attn_pool_fwd((const bf16*)t, w2, b2, (const bf16*)h, mask, B, L, Hh, H, weights, pooled, (bf16*)pooled_bf16,
                       (hipStream_t)stream);
}

extern "C" int ste_attn_pool_fwd_f32(const float* t, const float* w2, const float* b2, const float* h,
                                     const int32_t* mask, int B, int L, int Hh, int H, float* weights, float* pooled,
                                     void* pooled_bf16, void* stream) {
  return attn_pool_fwd(t, w2, b2, h, mask, B, L, Hh, H, weights, pooled, (bf16*)pooled_bf16, (hipStream_t)stream);
}

extern "C" int ste_attn_pool_bwd_work_floats(int B, int L, int Hh) {
  if (B <= 0 || L <= 0 || Hh <= 0) return STE_ERR_SHAPE;
  const int rows = pool_dz_rows(B, L);
  return B * L + B * ((L + rows - 1) / rows) * 2 * Hh + B;   // + the scorer bias' per-sample terms
}

template <typename T>
static int attn_pool_bwd(const T* t, const float* w2, const T* h, const float* weights, const float* dpooled,
                         const int32_t* mask, int B, int L, int Hh, int H, float* dh, T* dt, bf16* dt_lo, float* dw2,
                         float* db2, float* db1, float* work, hipStream_t s) {
  if (B <= 0 || L <= 0 || (Hh & 3) || (H & 3) || Hh > 4 * NT || !work || !dt) return STE_ERR_SHAPE;
  const int rows = pool_dz_rows(B, L), nchunk = (L + rows - 1) / rows;
  float* part = work + (int64_t)B * L;
  float* db2_part = part + (int64_t)B * nchunk * 2 * Hh;
  hipLaunchKernelGGL(pool_dp_kernel<T>, dim3(B, (L + POOL_DP_ROWS - 1) / POOL_DP_ROWS), dim3(NT), 0, s, h, dpooled, L,
                     H, work);
  STE_CHECK_LAUNCH();
  hipLaunchKernelGGL(pool_dscore_kernel, dim3(B), dim3(NT), 0, s, weights, mask, L, work, db2, db2_part);
  STE_CHECK_LAUNCH();
  if (db2) {
    if (int e = ste_rowsum_ordered(db2_part, B, 1, 1, db2, s)) return e;
  }
  hipLaunchKernelGGL(pool_dz_kernel<T>, dim3(B, nchunk), dim3(NT), 0, s, t, w2, weights, dpooled, work, L, Hh, H, dh,
                     dt, dt_lo, part, rows);
  STE_CHECK_LAUNCH();
  if (dw2 || db1) {
    hipLaunchKernelGGL(pool_dw_kernel, dim3((2 * Hh + 63) / 64), dim3(POOL_DW_NT), 0, s, part, B * nchunk, Hh, dw2,
                       db1);
    STE_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int ste_attn_pool_bwd(const void* t, const float* w2, const void* h, const float* weights,
                                 const float* dpooled, const int32_t* mask, int B, int L, int Hh, int H, float* dh,
                                 void* dt, void* dt_lo, float* dw2, float* db2, float* db1, float* work, void* stream) {
  return attn_pool_bwd((const bf16*)t, w2, (const bf16*)h, weights, dpooled, mask, B, L, Hh, H, dh, (bf16*)dt,
                       (bf16*)dt_lo, dw2, db2, db1, work, (hipStream_t)stream);
}

extern "C" int ste_attn_pool_bwd_f32(const float* t, const float* w2, const float* h, const float* weights,
                                     const float* dpooled, const int32_t* mask, int B, int L, int Hh, int H, float* dh,
                                     float* dt, float* dw2, float* db2, float* db1, float* work, void* stream) {
  return attn_pool_bwd(t, w2, h, weights, dpooled, mask, B, L, Hh, H, dh, dt, (bf16*)nullptr, dw2, db2, db1, work,
                       (hipStream_t)stream);
}

template <typename T>
static int mean_pool_fwd(const T* h, const int32_t* mask, int B, int L, int H, int cls, float* weights, float* pooled,
                         bf16* pooled_bf16, hipStream_t s) {
  if (B <= 0 || L <= 0 || (H & 3) || L > 16384) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(mean_pool_fwd_kernel<T>, dim3(B), dim3(NT), L * sizeof(float), s, h, mask, L, H, cls, weights,
                     pooled, pooled_bf16);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_mean_pool_fwd(const void* h, const int32_t* mask, int B, int L, int H, int cls, float* weights,
                                 float* pooled, void* pooled_bf16, void* stream) {
  return mean_pool_fwd((const bf16*)h, mask, B, L, H, cls, weights, pooled, (bf16*)pooled_bf16, (hipStream_t)stream);
}

extern "C" int ste_mean_pool_fwd_f32(const float* h, const int32_t* mask, int B, int L, int H, int cls,
                                     float* weights, float* pooled, void* pooled_bf16, void* stream) {
  return mean_pool_fwd(h, mask, B, L, H, cls, weights, pooled, (bf16*)pooled_bf16, (hipStream_t)stream);
}

extern "C" int ste_weighted_pool_bwd(const float* weights, const float* dpooled, int B, int L, int H, float* dh,
                                     void* stream) {
  if (B <= 0 || L <= 0 || (H & 3)) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(weighted_pool_bwd_kernel, dim3(B, (L + 15) / 16), dim3(NT), 0, (hipStream_t)stream, weights,
                     dpooled, L, H, dh);
  STE_CHECK_LAUNCH();
  return 0;
}

namespace {
bool xattn_shape_ok(int B, int S, int P, int nh, int nq) {
  if (B <= 0 || S <= 0 || nh <= 0 || P > 1024 || P % nh) return false;
  const int dh = P / nh;
  return dh % 8 == 0 && dh <= 256 && nq * S <= 16384;
}
}  // namespace

extern "C" int ste_xattn_fwd(const float* q, const void* k, const void* v, int64_t ldkv, const int32_t* mask, int B,
                             int S, int P, int nh, int nq, float scale, float drop_p, uint64_t seed0, uint64_t seed1,
                             float* probs, float* out, void* stream) {
  if (!xattn_shape_ok(B, S, P, nh, nq) || (nq != 1 && nq != 2) || (ldkv & 7) ||
      (((uintptr_t)k | (uintptr_t)v | (uintptr_t)out) & 15))
    return STE_ERR_SHAPE;
  const size_t lds = (size_t)nq * S * sizeof(float);
  if (nq == 1)
    hipLaunchKernelGGL(xattn_fwd_kernel<1>, dim3(B, nh), dim3(NT), lds, (hipStream_t)stream, q, (const bf16*)k,
                       (const bf16*)v, ldkv, mask, B, S, P, nh, scale, drop_p, seed0, seed1, probs, out);
  else
    hipLaunchKernelGGL(xattn_fwd_kernel<2>, dim3(B, nh), dim3(NT), lds, (hipStream_t)stream, q, (const bf16*)k,
                       (const bf16*)v, ldkv, mask, B, S, P, nh, scale, drop_p, seed0, seed1, probs, out);
  STE_CHECK_LAUNCH();
  return 0;
}

template <bool OUT_BF16>
static int xattn_bwd_launch(const float* q, const void* k, const void* v, int64_t ldkv, const float* probs,
                            const float* dout, const int32_t* mask, int B, int S, int P, int nh, int nq, float scale,
                            float drop_p,
                            uint64_t seed0, uint64_t seed1, float* dq, void* dk, void* dv, int64_t lddkv, float* part,
                            void* stream) {
  if (!xattn_shape_ok(B, S, P, nh, nq) || (nq != 1 && nq != 2) || (ldkv & 7) || lddkv < P ||
      (lddkv & (OUT_BF16 ? 7 : 3)) || (OUT_BF16 && !part) ||
      (((uintptr_t)k | (uintptr_t)v | (uintptr_t)dq | (uintptr_t)dk | (uintptr_t)dv | (uintptr_t)part) & 15))
    return STE_ERR_SHAPE;
  const size_t lds = (size_t)nq * S * sizeof(float);
  if (nq == 1)
    hipLaunchKernelGGL((xattn_bwd_kernel<1, OUT_BF16>), dim3(B, nh), dim3(NT), lds, (hipStream_t)stream, q,
                       (const bf16*)k, (const bf16*)v, ldkv, probs, dout, mask, B, S, P, nh, scale, drop_p, seed0,
                       seed1, dq, dk, dv, lddkv, part);
  else
    hipLaunchKernelGGL((xattn_bwd_kernel<2, OUT_BF16>), dim3(B, nh), dim3(NT), lds, (hipStream_t)stream, q,
                       (const bf16*)k, (const bf16*)v, ldkv, probs, dout, mask, B, S, P, nh, scale, drop_p, seed0,
                       seed1, dq, dk, dv, lddkv, part);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_xattn_bwd(const float* q, const void* k, const void* v, int64_t ldkv, const float* probs,
                             const float* dout, const int32_t* mask, int B, int S, int P, int nh, int nq, float scale,
                             float drop_p, uint64_t seed0, uint64_t seed1, float* dq, float* dk, float* dv,
                             int64_t lddkv, void* stream) {
  return xattn_bwd_launch<false>(q, k, v, ldkv, probs, dout, mask, B, S, P, nh, nq, scale, drop_p, seed0, seed1, dq, dk, dv,
                                 lddkv, nullptr, stream);
}

extern "C" int ste_xattn_bwd_bf16(const float* q, const void* k, const void* v, int64_t ldkv, const float* probs,
                                  const float* dout, const int32_t* mask, int B, int S, int P, int nh, int nq,
                                  float scale, float drop_p, uint64_t seed0, uint64_t seed1, float* dq, void* dk,
                                  void* dv, int64_t lddkv, float* colsum_part, void* stream) {
  return xattn_bwd_launch<true>(q, k, v, ldkv, probs, dout, mask, B, S, P, nh, nq, scale, drop_p, seed0, seed1, dq, dk, dv,
                                lddkv, colsum_part, stream);
}

extern "C" int ste_xattn1_fwd(const float* q, const void* k, const void* v, int64_t ldkv, const int32_t* mask, int B,
                              int S, int P, int nh, float scale, float drop_p, uint64_t seed, float* probs, float* out,
                              void* stream) {
  return ste_xattn_fwd(q, k, v, ldkv, mask, B, S, P, nh, 1, scale, drop_p, seed, seed, probs, out, stream);
}

extern "C" int ste_xattn1_bwd(const float* q, const void* k, const void* v, int64_t ldkv, const float* probs,
                              const float* dout, const int32_t* mask, int B, int S, int P, int nh, float scale,
                              float drop_p, uint64_t seed, float* dq, float* dk, float* dv, int64_t lddkv,
                              void* stream) {
  return ste_xattn_bwd(q, k, v, ldkv, probs, dout, mask, B, S, P, nh, 1, scale, drop_p, seed, seed, dq, dk, dv, lddkv,
                       stream);
}

extern "C" int ste_l2norm_fwd(const float* x, int rows, int cols, float* y, float* norms, void* stream) {
  if (rows <= 0 || cols <= 0) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(l2norm_fwd_kernel, dim3(rows), dim3(NT), 0, (hipStream_t)stream, x, cols, y, norms);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_l2norm_bwd(const float* y, const float* norms, const float* dy, int rows, int cols, float* dx,
                              void* stream) {
  if (rows <= 0 || cols <= 0) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(l2norm_bwd_kernel, dim3(rows), dim3(NT), 0, (hipStream_t)stream, y, norms, dy, cols, dx);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_similarity(const float* a, const float* t, int B, int NTt, int P, float* S, void* stream) {
  if (B <= 0 || NTt <= 0 || P <= 0) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(similarity_kernel, dim3((B + 15) / 16, (NTt + 15) / 16), dim3(64), 0, (hipStream_t)stream, a, t,
                     B, NTt, P, S);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_pair_loss_fwd(const float* S, int64_t ldS, int off_neg, const float* align, int B, int L, float tau,
                                 float aw, float gamma, float* s_pos, float* s_neg, float* loss, void* stream) {
  if (B <= 0) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(pair_loss_fwd_kernel, dim3(1), dim3(NT), 0, (hipStream_t)stream, S, ldS, off_neg, align, B, L,
                     tau, aw, gamma, s_pos, s_neg, loss);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_pair_loss_bwd(const float* s_pos, const float* s_neg, const float* align, int B, int L, float tau,
                                 float aw, float gamma, const float* gscale, float* ds_pos, float* ds_neg,
                                 float* dalign, void* stream) {
  if (B <= 0) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(pair_loss_bwd_kernel, dim3((B + NT - 1) / NT), dim3(NT), 0, (hipStream_t)stream, s_pos, s_neg,
                     align, B, L, tau, aw, gamma, gscale, ds_pos, ds_neg, dalign);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_pair_sim_bwd(const float* a, const float* tp, const float* tn, const float* ds_pos,
                                const float* ds_neg, int B, int P, float* da, float* dtp, float* dtn, void* stream) {
  if (B <= 0 || P <= 0) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(pair_sim_bwd_kernel, dim3(B), dim3(NT), 0, (hipStream_t)stream, a, tp, tn, ds_pos, ds_neg, P,
                     da, dtp, dtn);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_pair_metrics(const float* S, int64_t ldS, int NB, int off_neg, float tau, const float* losses,
                                int nloss, float loss_w, double* acc, void* stream) {
  if (NB <= 0 || ldS < off_neg + NB) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(pair_metrics_kernel, dim3(NB), dim3(NT), 0, (hipStream_t)stream, S, ldS, NB, off_neg, tau, losses,
                     nloss, loss_w, acc);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_inbatch_ce(const float* S, int64_t ldS, int B, int NB, int row0, float tau, float weight,
                              const float* gscale, float* loss, float* dS, int64_t lddS, void* stream) {
  if (B <= 0 || NB <= 0 || row0 < 0 || row0 + B > NB || ldS < NB || lddS < NB) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(inbatch_ce_kernel, dim3(B), dim3(NT), 0, (hipStream_t)stream, S, ldS, B, NB, row0, tau, weight,
                     gscale, loss, dS, lddS);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_rowmat_f32(const float* X, int64_t sxr, int64_t sxc, const float* Y, int R, int C, int P,
                              float* out, void* stream) {
  if (R <= 0 || C <= 0 || (P & 3)) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(rowmat_f32_kernel, dim3(R), dim3(NT), 0, (hipStream_t)stream, X, sxr, sxc, Y, C, P, out);
  STE_CHECK_LAUNCH();
  return 0;
}

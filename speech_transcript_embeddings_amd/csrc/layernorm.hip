// LayerNorm forward/backward, one wavefront per row, fp32 statistics.
// Replaces nn.LayerNorm in both encoders and the heads (see include/ste.h).
// HBM-bound: forward reads x once and writes y once; backward reads dy, x once.
// Rows are processed grid-stride; launches put ~16 waves on every CU so enough row loads
// are in flight to cover HBM latency.  When column sums are wanted (dgamma/dbeta/dsum of
// a trainable layer) the partials of a block are reduced through one reused LDS array and
// written to the caller's workspace, one row of partials per block, which ln_colsum_kernel
// adds in block order (run-to-run deterministic, no same-address atomics); without a
// workspace they are flushed with one atomic per column per block.  Frozen layers compile
// without that LDS.
#include "common.h"
#include "../../include/ste.h"

namespace {

constexpr int NT = 256;  // 4 waves = 4 rows in flight per block

template <int MAXC>
STE_DEV void load_row(const void* base, bool is_bf16, int64_t ld, int row, int cols, int lane, float (&v)[MAXC * 4]) {
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    int col = (lane + c * 64) * 4;
    f32x4 x = {0.f, 0.f, 0.f, 0.f};
    if (col < cols) {
      if (is_bf16) x = load_bf16x4((const bf16*)base + (int64_t)row * ld + col);
      else x = *reinterpret_cast<const f32x4*>((const float*)base + (int64_t)row * ld + col);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) v[c * 4 + e] = x[e];
  }
}

// One row of the forward: v holds the row's input values on entry and its output values
// (after row scale, activation, dropout) on exit; every requested output is written.
// gamma / beta of the lane's columns, loaded once per wave (not per row)
template <int MAXC>
struct LnParams {
  f32x4 g[MAXC], b[MAXC];
  STE_DEV void load(const float* gamma, const float* beta, int cols, int lane) {
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int col = (lane + c * 64) * 4;
      g[c] = col < cols ? *reinterpret_cast<const f32x4*>(gamma + col) : f32x4{0.f, 0.f, 0.f, 0.f};
      b[c] = (beta && col < cols) ? *reinterpret_cast<const f32x4*>(beta + col) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
};

template <int MAXC>
STE_DEV void ln_fwd_row(const ste_ln_fwd_args& a, const LnParams<MAXC>& pr, int row, int lane, float (&v)[MAXC * 4]) {
  const float inv_n = 1.0f / (float)a.cols;
  const uint32_t thresh = (uint32_t)(a.drop_p * 4294967296.0);
  const float inv_keep = a.drop_p > 0.f ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC * 4; ++i) s += v[i];
  const float mean = wave_sum(s) * inv_n;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    int col = (lane + c * 64) * 4;
    if (col < a.cols) {
#pragma unroll
      for (int e = 0; e < 4; ++e) { float d = v[c * 4 + e] - mean; q += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) * inv_n + a.eps);
  if (lane == 0) { a.mean[row] = mean; a.rstd[row] = rstd; }
  const float rs = a.row_scale ? a.row_scale[row] : 1.0f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    int col = (lane + c * 64) * 4;
    if (col >= a.cols) continue;
    const f32x4 g = pr.g[c], b = pr.b[c];
    f32x4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float t = ((v[c * 4 + e] - mean) * rstd * g[e] + b[e]) * rs;
      if (a.act == STE_ACT_SWISH) t = swish_f(t);
      if (a.drop_p > 0.f) t *= drop_scale(a.seed, (uint64_t)row * a.cols + col + e, thresh, inv_keep);
      y[e] = t;
      v[c * 4 + e] = t;
    }
    if (a.y) *reinterpret_cast<f32x4*>(a.y + (int64_t)row * a.ldy + col) = y;
    if (a.ylo) store_bf16x4_split((bf16*)a.yb + (int64_t)row * a.ldyb + col, (bf16*)a.ylo + (int64_t)row * a.ldylo + col, y);
    else if (a.yb) store_bf16x4((bf16*)a.yb + (int64_t)row * a.ldyb + col, y);
    if (a.q8) {  // MX-fp8 copy: 8 lanes x 4 columns = one 32-column block
      float am = fmaxf(fmaxf(fabsf(y[0]), fabsf(y[1])), fmaxf(fabsf(y[2]), fabsf(y[3])));
      am = fmaxf(am, dpp_f<0xB1>(am));    // lane ^ 1
      am = fmaxf(am, dpp_f<0x4E>(am));    // lane ^ 2
      am = fmaxf(am, dpp_f<0x141>(am));   // the other quad of the 8 lanes
      const int ex = mx8_exp(am);
      const float inv = ldexpf(1.0f, -ex);
      uint32_t w = 0;
      w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(y[0] * inv, -448.f), 448.f),
                                          fminf(fmaxf(y[1] * inv, -448.f), 448.f), w, false);
      w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(y[2] * inv, -448.f), 448.f),
                                          fminf(fmaxf(y[3] * inv, -448.f), 448.f), w, true);
      *reinterpret_cast<uint32_t*>((uint8_t*)a.q8 + (int64_t)row * a.ldq8 + col) = w;
      if ((lane & 7) == 0) ((uint8_t*)a.q8s)[(int64_t)row * (a.cols >> 5) + (col >> 5)] = (uint8_t)(ex + 127);
    }
  }
}

template <int MAXC>
__global__ __launch_bounds__(NT) void ln_fwd_kernel(ste_ln_fwd_args a) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * (NT / 64);
  LnParams<MAXC> pa;
  pa.load(a.gamma, a.beta, a.cols, lane);
  // one row in flight per wave (the next-row prefetch the pair kernel uses measured 34.2 -> 34.8 us
  // here at c2 rows: the single kernel already keeps ~16 waves per CU loading)
  for (int row = wave; row < a.rows; row += nwaves) {
    float v[MAXC * 4];
    load_row<MAXC>(a.x, a.x_bf16, a.ldx, row, a.cols, lane, v);
    ln_fwd_row<MAXC>(a, pa, row, lane, v);
  }
}

// Two chained LayerNorms over the same rows, y2 = LN_b(LN_a(x)) (a Conformer layer's final LN
// and the next layer's FFN1 LN): LN_a's output stays in registers for LN_b, saving LN_b's read
// of it and a launch.  b.x is not read.
// LEAN (default): no next-row prefetch and both LayerNorms' gamma / beta re-read per row
// (L1-resident) instead of held in registers: 127 VGPRs and 4 waves per SIMD instead of 172 and 2;
// 98.6 -> 85.8 us at c2 rows in isolation, +0.3 % c2 step (profiles/r4p_ln_pair_ab.txt).
// STE_LN_FWD_PAIR=prefetch: the round-3 form (A/B).
template <int MAXC, bool LEAN = false>
__global__ __launch_bounds__(NT) void ln_fwd_pair_kernel(ste_ln_fwd_args a, ste_ln_fwd_args b) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * (NT / 64);
  if constexpr (LEAN) {
    for (int row = wave; row < a.rows; row += nwaves) {
      float v[MAXC * 4];
      load_row<MAXC>(a.x, a.x_bf16, a.ldx, row, a.cols, lane, v);
      const float *ga = a.gamma, *ba = a.beta, *gb = b.gamma, *bb = b.beta;
      asm volatile("" : "+s"(ga), "+s"(ba), "+s"(gb), "+s"(bb));   // parameter loads stay in the loop
      {
        LnParams<MAXC> pa;
        pa.load(ga, ba, a.cols, lane);
        ln_fwd_row<MAXC>(a, pa, row, lane, v);
      }
      LnParams<MAXC> pb;
      pb.load(gb, bb, b.cols, lane);
      ln_fwd_row<MAXC>(b, pb, row, lane, v);
    }
  } else {
    LnParams<MAXC> pa;
    pa.load(a.gamma, a.beta, a.cols, lane);
    LnParams<MAXC> pb;
    pb.load(b.gamma, b.beta, b.cols, lane);
    float v[MAXC * 4], nx[MAXC * 4];
    if (wave < a.rows) load_row<MAXC>(a.x, a.x_bf16, a.ldx, wave, a.cols, lane, v);
    for (int row = wave; row < a.rows; row += nwaves) {
      if (row + nwaves < a.rows) load_row<MAXC>(a.x, a.x_bf16, a.ldx, row + nwaves, a.cols, lane, nx);
      ln_fwd_row<MAXC>(a, pa, row, lane, v);
      ln_fwd_row<MAXC>(b, pb, row, lane, v);
#pragma unroll
      for (int i = 0; i < MAXC * 4; ++i) v[i] = nx[i];
    }
  }
}
bool ln_fwd_pair_lean() {
  static int v = -1;
  if (v < 0) {
    const char* e = STE_AB_ENV("STE_LN_FWD_PAIR");
    v = (e && e[0] == 'p') ? 0 : 1;
  }
  return v == 1;
}

// Column-sum accumulators of one backward (gamma, beta, and the dxb copy's column sums).
template <int MAXC>
struct LnAcc {
  float dg[MAXC * 4], db[MAXC * 4], dsm[MAXC * 4];
  STE_DEV void zero() {
#pragma unroll
    for (int i = 0; i < MAXC * 4; ++i) { dg[i] = 0.f; db[i] = 0.f; dsm[i] = 0.f; }
  }
};

// One row of the backward: x holds the input row, g the incoming gradient; on exit g holds
// this LN's input gradient (dx, dres included); requested outputs are written.
// PRE: gamma (beta) and the residual row come preloaded in pr / dr (the single kernel: one memory
// round trip per row); otherwise they are read where used (the pair kernel, whose register count
// the preloads would raise from 4 to 3 waves per SIMD: measured 11-35 % slower).
template <int MAXC, bool PRE, bool DRPRE = PRE>
STE_DEV void ln_bwd_row(const ste_ln_bwd_args& a, int row, int lane, float (&x)[MAXC * 4], float (&g)[MAXC * 4],
                        const float* dr, const LnParams<MAXC>* pr, LnAcc<MAXC>& acc) {
  const float inv_n = 1.0f / (float)a.cols;
  const uint32_t thresh = (uint32_t)(a.drop_p * 4294967296.0);
  const float inv_keep = a.drop_p > 0.f ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  const uint32_t in_thresh = (uint32_t)(a.in_drop_p * 4294967296.0);
  const float in_inv_keep = a.in_drop_p > 0.f ? 1.0f / (1.0f - a.in_drop_p) : 1.0f;
  const float mean = a.mean[row], rstd = a.rstd[row];
  const float rs = a.row_scale ? a.row_scale[row] : 1.0f;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    int col = (lane + c * 64) * 4;
    if (col >= a.cols) continue;
    f32x4 gm, bt = {0.f, 0.f, 0.f, 0.f};    // bt used only under swish
    if constexpr (PRE) {
      gm = pr->g[c];
      bt = pr->b[c];
    } else {
      gm = *reinterpret_cast<const f32x4*>(a.gamma + col);
      if (a.act == STE_ACT_SWISH) bt = *reinterpret_cast<const f32x4*>(a.beta + col);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = c * 4 + e;
      const float xh = (x[i] - mean) * rstd;
      float gi = g[i];
      if (a.in_drop_p > 0.f) gi *= drop_scale(a.in_seed, (uint64_t)row * a.cols + col + e, in_thresh, in_inv_keep);
      if (a.act == STE_ACT_SWISH) gi *= swish_d((xh * gm[e] + bt[e]) * rs);
      gi *= rs;
      acc.dg[i] += gi * xh;
      acc.db[i] += gi;
      const float gg = gi * gm[e];
      g[i] = gg;
      x[i] = xh;
      s1 += gg;
      s2 += gg * xh;
    }
  }
  s1 = wave_sum(s1) * inv_n;
  s2 = wave_sum(s2) * inv_n;
  const float ors = a.out_row_scale ? a.out_row_scale[row] : 1.0f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    int col = (lane + c * 64) * 4;
    if (col >= a.cols) continue;
    f32x4 d;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = c * 4 + e;
      d[e] = rstd * (g[i] - s1 - x[i] * s2);
    }
    if (a.dres) {
      if (DRPRE) {   // loaded with the row's other operands (one memory round trip per row)
#pragma unroll
        for (int e = 0; e < 4; ++e) d[e] += dr[c * 4 + e];
      } else {
        d += *reinterpret_cast<const f32x4*>(a.dres + (int64_t)row * a.lddres + col);
      }
    }
    if (a.dx) *reinterpret_cast<f32x4*>(a.dx + (int64_t)row * a.lddx + col) = d;
    if (a.dxb || a.dsum) {
      f32x4 o = d * (a.out_scale * ors);
      if (a.drop_p > 0.f) {
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] *= drop_scale(a.seed, (uint64_t)row * a.cols + col + e, thresh, inv_keep);
      }
      if (a.dxb) store_bf16x4((bf16*)a.dxb + (int64_t)row * a.lddxb + col, o);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc.dsm[c * 4 + e] += o[e];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) g[c * 4 + e] = d[e];
  }
}

// the block's column sums of one backward through one reused LDS array: into the workspace
// (ws[k][block][col], summed by ln_colsum_kernel) or, without one, one atomic per column
template <int MAXC>
STE_DEV void ln_flush(const ste_ln_bwd_args& a, const LnAcc<MAXC>& acc, float (*red)[MAXC * 4 * 64], int lane,
                      int wid) {
  float* const outs[3] = {a.dgamma, a.dbeta, a.dsum};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (!outs[k]) continue;  // uniform
    const float* src = k == 0 ? acc.dg : (k == 1 ? acc.db : acc.dsm);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MAXC * 4; ++i) red[wid][(i >> 2) * 256 + lane * 4 + (i & 3)] = src[i];
    __syncthreads();
    float* part = a.ws ? a.ws + ((int64_t)k * gridDim.x + blockIdx.x) * a.cols : nullptr;
    for (int j = threadIdx.x; j < MAXC * 256; j += NT) {
      const int c = j >> 8, rem = j & 255;
      const int col = (c * 64 + (rem >> 2)) * 4 + (rem & 3);
      if (col >= a.cols) continue;
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < NT / 64; ++w) sum += red[w][j];
      if (part) part[col] = sum;
      else atomicAdd(outs[k] + col, sum);
    }
  }
}

// out_k[col] += Σ_block ws[k][block][col] in a fixed order (CS_SL interleaved slices of the
// blocks, then the slices in order): 16 columns x 64 slices per block, grid (ceil(cols / 16), 3),
// 1024 threads, 8 loads in flight per thread (3 x 64 blocks at 1,024 columns instead of 3 x 16)
constexpr int CS_CW = 16, CS_SL = 1024 / CS_CW;
__global__ __launch_bounds__(1024) void ln_colsum_kernel(const float* __restrict__ ws, int nblk, int cols,
                                                         float* dgamma, float* dbeta, float* dsum) {
  float* const out = blockIdx.y == 0 ? dgamma : (blockIdx.y == 1 ? dbeta : dsum);
  if (!out) return;  // uniform
  __shared__ float red[CS_SL][CS_CW];
  const int c = threadIdx.x % CS_CW, sl = threadIdx.x / CS_CW;
  const int col = blockIdx.x * CS_CW + c;
  float acc = 0.f;
  if (col < cols) {
    const float* p = ws + (int64_t)blockIdx.y * nblk * cols + col;
    int b = sl;
    for (; b + 7 * CS_SL < nblk; b += 8 * CS_SL) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[(int64_t)(b + CS_SL * u) * cols];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; b < nblk; b += CS_SL) acc += p[(int64_t)b * cols];
  }
  red[sl][c] = acc;
  __syncthreads();
  if (sl == 0 && col < cols) {
    float t = red[0][c];
    for (int k = 1; k < CS_SL; ++k) t += red[k][c];
    out[col] += t;
  }
}

template <int MAXC, bool REDUCE>
__global__ __launch_bounds__(NT, REDUCE ? 3 : 1) void ln_bwd_kernel(ste_ln_bwd_args a) {
  __shared__ float red[REDUCE ? NT / 64 : 1][REDUCE ? MAXC * 4 * 64 : 1];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wave = blockIdx.x * (NT / 64) + wid;
  const int nwaves = gridDim.x * (NT / 64);
  LnAcc<MAXC> acc;
  acc.zero();
  // one row in flight per wave: issuing the next row's x / dy / dres a row ahead (round 3,
  // a6ffbd2) raised the column-sum-free kernel to 154 VGPRs and 3 waves per SIMD and made it
  // slower, 94.5 -> 126.2 us at c2 rows (2.3 % of the c2 step).  gamma (beta) preloaded without
  // column sums; with them gamma is read where used (L1-resident) instead, which with the 48
  // accumulators keeps the kernel at 3 waves per SIMD (<= 168 VGPRs) rather than 2 (180)
  LnParams<MAXC> pa;
  if constexpr (!REDUCE) pa.load(a.gamma, a.act == STE_ACT_SWISH ? a.beta : nullptr, a.cols, lane);
  for (int row = wave; row < a.rows; row += nwaves) {
    float x[MAXC * 4], g[MAXC * 4], dr[MAXC * 4];
    load_row<MAXC>(a.x, a.x_bf16, a.ldx, row, a.cols, lane, x);
    load_row<MAXC>(a.dy, a.dy_bf16, a.lddy, row, a.cols, lane, g);
    if (a.dres) load_row<MAXC>(a.dres, false, a.lddres, row, a.cols, lane, dr);
    if constexpr (REDUCE) ln_bwd_row<MAXC, false, true>(a, row, lane, x, g, dr, nullptr, acc);
    else ln_bwd_row<MAXC, true>(a, row, lane, x, g, dr, &pa, acc);
  }
  if constexpr (REDUCE) ln_flush<MAXC>(a, acc, red, lane, wid);
}

// Backward of the forward pair, in reverse: LN_b's backward (a.dy ignored: its dy is b.dy)
// produces d(LN_a output) in registers, which is LN_a's incoming gradient.  b.dx may be NULL
// (the intermediate gradient never touches HBM).
template <int MAXC, bool REDUCE>
// without column sums: b's residual row is issued with its x and dy and the kernel is held to
// 128 VGPRs (4 waves per SIMD; 143 -> 135 us at c2 rows); with them (trainable layers, 2 calls
// per step) the register count would spill, so the residual is read where used
__global__ __launch_bounds__(NT, REDUCE ? 1 : 4) void ln_bwd_pair_kernel(ste_ln_bwd_args a, ste_ln_bwd_args b) {
  __shared__ float red[REDUCE ? NT / 64 : 1][REDUCE ? MAXC * 4 * 64 : 1];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wave = blockIdx.x * (NT / 64) + wid;
  const int nwaves = gridDim.x * (NT / 64);
  LnAcc<MAXC> acc_a, acc_b;
  acc_a.zero();
  acc_b.zero();
  for (int row = wave; row < a.rows; row += nwaves) {
    float x[MAXC * 4], g[MAXC * 4], dr[MAXC * 4];
    load_row<MAXC>(b.x, b.x_bf16, b.ldx, row, b.cols, lane, x);
    load_row<MAXC>(b.dy, b.dy_bf16, b.lddy, row, b.cols, lane, g);
    if (!REDUCE && b.dres) load_row<MAXC>(b.dres, false, b.lddres, row, b.cols, lane, dr);
    ln_bwd_row<MAXC, false, !REDUCE>(b, row, lane, x, g, dr, nullptr, acc_b);
    load_row<MAXC>(a.x, a.x_bf16, a.ldx, row, a.cols, lane, x);
    ln_bwd_row<MAXC, false>(a, row, lane, x, g, nullptr, nullptr, acc_a);
  }
  if constexpr (REDUCE) {
    ln_flush<MAXC>(b, acc_b, red, lane, wid);
    ln_flush<MAXC>(a, acc_a, red, lane, wid);
  }
}

// enough 4-wave blocks for ~16 waves per CU (256 CUs), never more than one wave per row
inline int grid_for(int rows, int cap = 1024) {
  int g = (rows + 3) / 4;
  return g < cap ? g : cap;
}
// column-sum launches: fewer, longer blocks (one partial row or one atomic per column per block)
// (the single column-sum kernel runs 3 waves per SIMD: 768 blocks = 3 per CU; the pair's 2: 512)
constexpr int LN_REDUCE_BLOCKS = 768, LN_PAIR_REDUCE_BLOCKS = 512;
inline int grid_bwd(const ste_ln_bwd_args& a, bool reduce) {
  return grid_for(a.rows, reduce ? LN_REDUCE_BLOCKS : 1024);
}
inline bool ws_ok(const ste_ln_bwd_args& a, int nblk) {
  return !a.ws || a.ws_floats >= 3 * (int64_t)nblk * a.cols;
}
inline void colsum(const ste_ln_bwd_args& a, int nblk, hipStream_t s) {
  if (!a.ws || !(a.dgamma || a.dbeta || a.dsum)) return;
  hipLaunchKernelGGL(ln_colsum_kernel, dim3((unsigned)((a.cols + CS_CW - 1) / CS_CW), 3), dim3(1024), 0, s, (const float*)a.ws,
                     nblk, a.cols, a.dgamma, a.dbeta, a.dsum);
}

}  // namespace

extern "C" int ste_layernorm_fwd(const ste_ln_fwd_args* a, void* stream) {
  if (!a || a->rows <= 0 || a->cols <= 0 || (a->cols & 3) || a->cols > 2048 || !a->mean || !a->rstd)
    return STE_ERR_ARG;
  if (a->q8 && (!a->q8s || (a->cols & 127) || a->ldq8 < a->cols || (a->ldq8 & 3) || (((uintptr_t)a->q8) & 3)))
    return STE_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(grid_for(a->rows));
  if (a->cols <= 256) hipLaunchKernelGGL(ln_fwd_kernel<1>, grid, dim3(NT), 0, s, *a);
  else if (a->cols <= 1024) hipLaunchKernelGGL(ln_fwd_kernel<4>, grid, dim3(NT), 0, s, *a);
  else hipLaunchKernelGGL(ln_fwd_kernel<8>, grid, dim3(NT), 0, s, *a);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_layernorm_fwd_pair(const ste_ln_fwd_args* a, const ste_ln_fwd_args* b, void* stream) {
  if (!a || !b || a->rows <= 0 || a->cols <= 0 || (a->cols & 3) || a->cols > 1024 || b->rows != a->rows ||
      b->cols != a->cols || !a->mean || !a->rstd || !b->mean || !b->rstd)
    return STE_ERR_ARG;
  for (const ste_ln_fwd_args* t : {a, b})
    if (t->q8 && (!t->q8s || (t->cols & 127) || t->ldq8 < t->cols || (t->ldq8 & 3) || (((uintptr_t)t->q8) & 3)))
      return STE_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(grid_for(a->rows));
  if (a->cols <= 256) hipLaunchKernelGGL(ln_fwd_pair_kernel<1>, grid, dim3(NT), 0, s, *a, *b);
  else if (ln_fwd_pair_lean()) hipLaunchKernelGGL((ln_fwd_pair_kernel<4, true>), grid, dim3(NT), 0, s, *a, *b);
  else hipLaunchKernelGGL(ln_fwd_pair_kernel<4>, grid, dim3(NT), 0, s, *a, *b);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_layernorm_bwd_pair(const ste_ln_bwd_args* a, const ste_ln_bwd_args* b, void* stream) {
  if (!a || !b || a->rows <= 0 || a->cols <= 0 || (a->cols & 3) || a->cols > 1024 || b->rows != a->rows ||
      b->cols != a->cols)
    return STE_ERR_ARG;
  if ((a->act == STE_ACT_SWISH && !a->beta) || (b->act == STE_ACT_SWISH && !b->beta)) return STE_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const bool reduce = a->dgamma || a->dbeta || a->dsum || b->dgamma || b->dbeta || b->dsum;
  // one grid for both: atomics as soon as either LN has no workspace
  const bool use_ws = (a->ws || !(a->dgamma || a->dbeta || a->dsum)) && (b->ws || !(b->dgamma || b->dbeta || b->dsum));
  const int nblk = grid_for(a->rows, reduce ? LN_PAIR_REDUCE_BLOCKS : 1024);
  if (reduce && use_ws && (!ws_ok(*a, nblk) || !ws_ok(*b, nblk))) return STE_ERR_ARG;
  ste_ln_bwd_args aa = *a, bb = *b;
  if (!use_ws) aa.ws = bb.ws = nullptr;
  const dim3 grid(nblk);
  if (a->cols <= 256) {
    if (reduce) hipLaunchKernelGGL((ln_bwd_pair_kernel<1, true>), grid, dim3(NT), 0, s, aa, bb);
    else hipLaunchKernelGGL((ln_bwd_pair_kernel<1, false>), grid, dim3(NT), 0, s, aa, bb);
  } else {
    if (reduce) hipLaunchKernelGGL((ln_bwd_pair_kernel<4, true>), grid, dim3(NT), 0, s, aa, bb);
    else hipLaunchKernelGGL((ln_bwd_pair_kernel<4, false>), grid, dim3(NT), 0, s, aa, bb);
  }
  STE_CHECK_LAUNCH();
  if (reduce && use_ws) {
    colsum(bb, nblk, s);
    colsum(aa, nblk, s);
    STE_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int ste_layernorm_bwd(const ste_ln_bwd_args* a, void* stream) {
  if (!a || a->rows <= 0 || a->cols <= 0 || (a->cols & 3) || a->cols > 1024) return STE_ERR_ARG;
  if (a->act == STE_ACT_SWISH && !a->beta) return STE_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const bool reduce = a->dgamma || a->dbeta || a->dsum;
  const int nblk = grid_bwd(*a, reduce);
  if (reduce && !ws_ok(*a, nblk)) return STE_ERR_ARG;
  const dim3 grid(nblk);
  if (a->cols <= 256) {
    if (reduce) hipLaunchKernelGGL((ln_bwd_kernel<1, true>), grid, dim3(NT), 0, s, *a);
    else hipLaunchKernelGGL((ln_bwd_kernel<1, false>), grid, dim3(NT), 0, s, *a);
  } else {
    if (reduce) hipLaunchKernelGGL((ln_bwd_kernel<4, true>), grid, dim3(NT), 0, s, *a);
    else hipLaunchKernelGGL((ln_bwd_kernel<4, false>), grid, dim3(NT), 0, s, *a);
  }
  STE_CHECK_LAUNCH();
  if (reduce) {
    colsum(*a, nblk, s);
    STE_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int64_t ste_layernorm_bwd_ws_floats(int rows, int cols) {
  return rows <= 0 || cols <= 0 ? 0 : 3 * (int64_t)grid_for(rows, LN_REDUCE_BLOCKS) * cols;
}

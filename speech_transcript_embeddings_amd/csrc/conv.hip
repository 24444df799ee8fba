// Conformer convolution-module core: GLU over channels fused with the causal depthwise
// Conv1d (kernel K, left zero-pad K-1, no bias) — tf:models/wav2vec2_bert/
// modeling_wav2vec2_bert.py:198-207.  The GLU output is never materialised in HBM:
// forward recomputes it from `pre` while staging, backward recomputes it for dW and
// emits d(pre) for both GLU halves directly.
//
// Block = (batch b, 64 time rows, 64 channels), 256 threads; the time window with its
// K-1 halo is staged in LDS as fp32 (16-B global loads of 8 channels); each thread owns one
// channel and 16 consecutive rows: its 31 taps (staged through LDS, coalesced) and its
// 16 + 30 window rows sit in registers, so the tap loop reads LDS once per row, not per tap.
// Results leave row-contiguous through the freed staging rows (16-B stores of 8 channels).
#include "common.h"
#include "../../include/ste.h"

namespace {

constexpr int TT = 64, CC = 64, NT = 256, KMAX = 31;
constexpr int RPT = TT / (NT / CC);  // rows per thread (16)

template <int K>
__global__ __launch_bounds__(NT) void glu_dwconv_fwd_kernel(const bf16* __restrict__ pre, const float* __restrict__ w,
                                                          bf16* __restrict__ out, int T, int C) {
  __shared__ float sg[TT + K - 1][CC];
  __shared__ float sw[CC * K];  // the block's taps, staged coalesced (a lane's taps are 124 B apart in w)
  const int b = blockIdx.z, t0 = blockIdx.x * TT, c0 = blockIdx.y * CC;
  const int tid = threadIdx.x;
  for (int i = tid; i < CC * K; i += NT) sw[i] = w[c0 * K + i];
  // stage g = a * sigmoid(gate) for rows t0-(K-1) .. t0+TT-1: 16-B loads of 8 channels of
  // each GLU half, every load of the thread issued before the first use
  constexpr int ITEMS = (TT + K - 1) * (CC / 8), PER = (ITEMS + NT - 1) / NT;
  bf16x8 av[PER], gv[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int i = tid + u * NT, r = i / (CC / 8), c8 = (i % (CC / 8)) * 8;
    const int t = t0 - (K - 1) + r;
    av[u] = bf16x8{};
    gv[u] = bf16x8{};
    if (i < ITEMS && t >= 0 && t < T) {
      const bf16* p = pre + (int64_t)(b * T + t) * (2 * C) + c0 + c8;
      av[u] = *reinterpret_cast<const bf16x8*>(p);
      gv[u] = *reinterpret_cast<const bf16x8*>(p + C);
    }
  }
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int i = tid + u * NT, r = i / (CC / 8), c8 = (i % (CC / 8)) * 8;
    if (i >= ITEMS) continue;
    f32x4 lo, hi;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      lo[e] = (float)av[u][e] * sigmoidf_((float)gv[u][e]);
      hi[e] = (float)av[u][4 + e] * sigmoidf_((float)gv[u][4 + e]);
    }
    *reinterpret_cast<f32x4*>(&sg[r][c8]) = lo;
    *reinterpret_cast<f32x4*>(&sg[r][c8 + 4]) = hi;
  }
  __syncthreads();
  const int c = tid & (CC - 1), rg = tid >> 6;  // 4 row groups of RPT
  float wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wk[k] = sw[c * K + k];  // stride 31 words: conflict-free
  const int rbeg = rg * RPT;
  // the thread's RPT + K - 1 input rows in registers: one LDS read per row instead of one per tap
  float win[RPT + K - 1];
#pragma unroll
  for (int j = 0; j < RPT + K - 1; ++j) win[j] = sg[rbeg + j][c];
  float acc[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) acc[i] = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int i = 0; i < RPT; ++i) acc[i] += wk[k] * win[i + k];  // output row t0+rbeg+i: rows i..i+K-1
  // outputs leave row-contiguous: through the (now free) staging rows, 8 channels per 16-B store
  __syncthreads();
#pragma unroll
  for (int i = 0; i < RPT; ++i) sg[rbeg + i][c] = acc[i];
  __syncthreads();
  for (int i = tid; i < TT * (CC / 8); i += NT) {
    const int r = i / (CC / 8), c8 = (i % (CC / 8)) * 8;
    const int t = t0 + r;
    if (t >= T) continue;
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)sg[r][c8 + e];
    *reinterpret_cast<bf16x8*>(out + (int64_t)(b * T + t) * C + c0 + c8) = o;
  }
}

// DW = false (frozen layers): only the dout window is staged (24 KB LDS -> 6 blocks/CU).
// DW = true: the GLU output window too, and the [4 row groups][64 ch][K] dW partials are
// reduced through the same LDS after the main pass (48 KB).
template <int K, bool DW>
__global__ __launch_bounds__(NT) void glu_dwconv_bwd_kernel(const bf16* __restrict__ pre, const float* __restrict__ w,
                                                          const bf16* __restrict__ dout, bf16* __restrict__ dpre,
                                                          float* __restrict__ dw, int T, int C,
                                                          float* __restrict__ part) {
  constexpr int ROWS = TT + K - 1;
  __shared__ float lds[(DW ? 2 : 1) * ROWS * CC];
  __shared__ float sw[CC * K];
  // DW: the tile's own rows of pre (a | gate, bf16) kept from the staging pass for the GLU
  // backward, which otherwise re-reads them from HBM (72 KB in all: still 2 blocks per CU)
  __shared__ bf16x8 sag[DW ? TT * (CC / 8) * 2 : 1];
  float (*sd)[CC] = reinterpret_cast<float (*)[CC]>(lds);              // dout rows t0 .. t0+TT+K-2
  float (*sg)[CC] = reinterpret_cast<float (*)[CC]>(lds + ROWS * CC);  // g rows t0-(K-1) .. t0+TT-1 (DW only)
  const int b = blockIdx.z, c0 = blockIdx.y * CC;
  const int tid = threadIdx.x;
  const int c = tid & (CC - 1), rg = tid >> 6;
  for (int i = tid; i < CC * K; i += NT) sw[i] = w[c0 * K + i];
  float dwp[DW ? K : 1];
#pragma unroll
  for (int k = 0; k < (DW ? K : 1); ++k) dwp[k] = 0.f;
  // DW: a block walks several 64-row tiles (grid.x < tiles) and keeps its dW partials in
  // registers across them, so each (channel, tap) address takes one atomic per block, not per tile
  const int ntile = (T + TT - 1) / TT;
  // DW (a block walks several tiles): the tile's staging loads (16 B of 8 channels per item) live
  // in registers, and the next tile's are issued right after this tile's reach LDS, so their
  // latency hides under this tile's compute.  Frozen layers (one tile per block) stage directly:
  // the registers would cost them occupancy for nothing.
  constexpr int ITEMS = ROWS * (CC / 8), PER = DW ? (ITEMS + NT - 1) / NT : 1;
  bf16x8 rdv[PER], rav[PER], rgv[PER];
  auto fetch = [&](int t0) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int i = tid + u * NT, r = i / (CC / 8), c8 = (i % (CC / 8)) * 8;
      const int td = t0 + r, tg = t0 - (K - 1) + r;
      rdv[u] = (i < ITEMS && td < T) ? *reinterpret_cast<const bf16x8*>(dout + (int64_t)(b * T + td) * C + c0 + c8)
                                     : bf16x8{};
      const bool ok = i < ITEMS && tg >= 0 && tg < T;
      const bf16* p = pre + (int64_t)(b * T + (ok ? tg : 0)) * (2 * C) + c0 + c8;
      rav[u] = ok ? *reinterpret_cast<const bf16x8*>(p) : bf16x8{};
      rgv[u] = ok ? *reinterpret_cast<const bf16x8*>(p + C) : bf16x8{};
    }
  };
  if (DW && (int)blockIdx.x < ntile) fetch(blockIdx.x * TT);
  for (int tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
  const int t0 = tile * TT;
  __syncthreads();   // sw staged / the previous tile's LDS reads done
  if constexpr (DW) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int i = tid + u * NT, r = i / (CC / 8), c8 = (i % (CC / 8)) * 8;
      if (i >= ITEMS) continue;
      const int tg = t0 - (K - 1) + r;
      const bf16x8 dv = rdv[u], av = rav[u], gv = rgv[u];
#pragma unroll
      for (int e = 0; e < 8; ++e) sd[r][c8 + e] = (float)dv[e];
#pragma unroll
      for (int e = 0; e < 8; ++e) sg[r][c8 + e] = (tg >= 0 && tg < T) ? (float)av[e] * sigmoidf_((float)gv[e]) : 0.f;
      if (r >= K - 1) {   // row t0 + (r - (K-1)) of this tile
        const int q = (r - (K - 1)) * (CC / 8) + c8 / 8;
        sag[2 * q] = av;
        sag[2 * q + 1] = gv;
      }
    }
    if (tile + (int)gridDim.x < ntile) fetch((tile + gridDim.x) * TT);
  } else {
    for (int i = tid; i < ITEMS; i += NT) {  // 16-B loads of 8 channels
      const int r = i / (CC / 8), c8 = (i % (CC / 8)) * 8;
      const int td = t0 + r;
      bf16x8 dv = bf16x8{};
      if (td < T) dv = *reinterpret_cast<const bf16x8*>(dout + (int64_t)(b * T + td) * C + c0 + c8);
#pragma unroll
      for (int e = 0; e < 8; ++e) sd[r][c8 + e] = (float)dv[e];
    }
  }
  __syncthreads();
  float wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wk[k] = sw[c * K + k];
  const int rbeg = rg * RPT;
  // register windows of the thread's RPT + K - 1 staged rows (one LDS read per row)
  float dwin[RPT + K - 1], gwin[DW ? RPT + K - 1 : 1];
#pragma unroll
  for (int j = 0; j < RPT + K - 1; ++j) dwin[j] = sd[rbeg + j][c];
  if (DW) {
#pragma unroll
    for (int j = 0; j < RPT + K - 1; ++j) gwin[j] = sg[rbeg + j][c];
  }
  float dg[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    // dg[t] = Σ_k w[k] * dout[t + (K-1) - k]  -> dwin[i + K-1-k]
    dg[i] = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) dg[i] += wk[k] * dwin[i + (K - 1) - k];
    if (DW) {
      // dW[k] += dout[t] * g[t - (K-1) + k] -> dwin[i] * gwin[i + k]
      const float d0 = dwin[i];
#pragma unroll
      for (int k = 0; k < K; ++k) dwp[k] += d0 * gwin[i + k];
    }
  }
  // GLU backward row-contiguous: dg through the (now free) dout rows, 8 channels per 16-B access
  __syncthreads();
#pragma unroll
  for (int i = 0; i < RPT; ++i) sd[rbeg + i][c] = dg[i];
  __syncthreads();
  for (int i = tid; i < TT * (CC / 8); i += NT) {
    const int r = i / (CC / 8), c8 = (i % (CC / 8)) * 8;
    const int t = t0 + r;
    if (t >= T) continue;
    const int64_t row = (int64_t)(b * T + t);
    bf16x8 av, gv;
    if constexpr (DW) {
      av = sag[2 * i];   // i = r * (CC / 8) + c8 / 8: the staged row r, channels c8..c8+7
      gv = sag[2 * i + 1];
    } else {
      av = *reinterpret_cast<const bf16x8*>(pre + row * 2 * C + c0 + c8);
      gv = *reinterpret_cast<const bf16x8*>(pre + row * 2 * C + C + c0 + c8);
    }
    bf16x8 da, dgate;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = sd[r][c8 + e], sgm = sigmoidf_((float)gv[e]);
      da[e] = (bf16)(d * sgm);
      dgate[e] = (bf16)(d * (float)av[e] * sgm * (1.f - sgm));
    }
    *reinterpret_cast<bf16x8*>(dpre + row * 2 * C + c0 + c8) = da;
    *reinterpret_cast<bf16x8*>(dpre + row * 2 * C + C + c0 + c8) = dgate;
  }
  }  // row tiles
  if (!DW) return;
  // reduce the 4 row groups' partials through the (now free) staging LDS: [rg][c][K+1]
  __syncthreads();
  float* sred = lds;
#pragma unroll
  for (int k = 0; k < K; ++k) sred[(rg * CC + c) * (K + 1) + k] = dwp[k];
  __syncthreads();
  for (int i = tid; i < CC * K; i += NT) {
    const int cc = i / K, k = i % K;
    float sum = 0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g) sum += sred[(g * CC + cc) * (K + 1) + k];
    // ordered mode: the block's partial row (batch, row-tile group) of [C·K], summed in order by
    // ste_rowsum_ordered; else one atomic per (channel, tap) per block
    if (part) part[((int64_t)blockIdx.z * gridDim.x + blockIdx.x) * C * K + (c0 + cc) * K + k] = sum;
    else atomicAdd(dw + (c0 + cc) * K + k, sum);
  }
}

}  // namespace

extern "C" int ste_glu_dwconv_fwd(const void* pre, const float* w, void* out, int B, int T, int C, int K,
                                  void* stream) {
  if (B <= 0 || T <= 0 || C <= 0 || (C % CC) != 0 || K != KMAX) return STE_ERR_SHAPE;
  dim3 grid((T + TT - 1) / TT, C / CC, B);
  hipLaunchKernelGGL(glu_dwconv_fwd_kernel<KMAX>, grid, dim3(NT), 0, (hipStream_t)stream, (const bf16*)pre, w,
                     (bf16*)out, T, C);
  STE_CHECK_LAUNCH();
  return 0;
}

namespace {
// ~8 row tiles per dW block: 8x fewer partials (or same-address atomics) on dW, still >= 2
// blocks per CU at B = 64 (measured 1/2/4/8/24 tiles: 237/200/196/186/188 us at T = 499)
constexpr unsigned DW_TILES_PER_BLOCK = 8;
unsigned dw_row_groups(int T) { return ((T + TT - 1) / TT + DW_TILES_PER_BLOCK - 1) / DW_TILES_PER_BLOCK; }
}  // namespace

extern "C" int64_t ste_glu_dwconv_bwd_ws_floats(int B, int T, int C, int K) {
  return (int64_t)B * dw_row_groups(T) * C * K;
}

extern "C" int ste_glu_dwconv_bwd(const void* pre, const float* w, const void* dout, void* dpre, float* dw, int B,
                                  int T, int C, int K, float* ws, int64_t ws_floats, void* stream) {
  if (B <= 0 || T <= 0 || C <= 0 || (C % CC) != 0 || K != KMAX) return STE_ERR_SHAPE;
  dim3 grid((T + TT - 1) / TT, C / CC, B);
  if (dw) {
    grid.x = dw_row_groups(T);
    // with a workspace: per-block partial rows summed in order afterwards (deterministic dW)
    const int64_t rows = (int64_t)B * grid.x;
    float* part = (ws && ws_floats >= rows * C * K) ? ws : nullptr;
    hipLaunchKernelGGL((glu_dwconv_bwd_kernel<KMAX, true>), grid, dim3(NT), 0, (hipStream_t)stream, (const bf16*)pre,
                       w, (const bf16*)dout, (bf16*)dpre, dw, T, C, part);
    STE_CHECK_LAUNCH();
    if (part) return ste_rowsum_ordered(part, rows, C * K, 1, dw, stream);
    return 0;
  }
  hipLaunchKernelGGL((glu_dwconv_bwd_kernel<KMAX, false>), grid, dim3(NT), 0, (hipStream_t)stream, (const bf16*)pre,
                     w, (const bf16*)dout, (bf16*)dpre, dw, T, C, nullptr);
  STE_CHECK_LAUNCH();
  return 0;
}

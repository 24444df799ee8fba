// Conformer convolution-module core: GLU over channels fused with the causal depthwise
// Conv1d (kernel K, left zero-pad K-1, no bias) — tf:models/wav2vec2_bert/
// modeling_wav2vec2_bert.py:198-207.  The GLU output is never materialised in HBM:
// forward recomputes it from `pre` while staging, backward recomputes it for dW and
// emits d(pre) for both GLU halves directly.
//
// Block = (batch b, 64 time rows, 64 channels), 256 threads; the time window with its
// K-1 halo is staged in LDS as fp32; each thread owns one channel and 16 consecutive
// rows (the taps held in registers).
#include "common.h"
#include "../../include/ste.h"

namespace {

constexpr int TT = 64, CC = 64, NT = 256, KMAX = 31;

template <int K>
__global__ __launch_bounds__(NT) void glu_dwconv_fwd_kernel(const bf16* __restrict__ pre, const float* __restrict__ w,
                                                          bf16* __restrict__ out, int T, int C) {
  __shared__ float sg[TT + K - 1][CC];
  const int b = blockIdx.z, t0 = blockIdx.x * TT, c0 = blockIdx.y * CC;
  const int tid = threadIdx.x;
  // stage g = a * sigmoid(gate) for rows t0-(K-1) .. t0+TT-1
  for (int i = tid; i < (TT + K - 1) * (CC / 4); i += NT) {
    const int r = i / (CC / 4), c4 = (i % (CC / 4)) * 4;
    const int t = t0 - (K - 1) + r;
    f32x4 g = {0.f, 0.f, 0.f, 0.f};
    if (t >= 0 && t < T) {
      const bf16* p = pre + (int64_t)(b * T + t) * (2 * C) + c0 + c4;
      f32x4 av = load_bf16x4(p), gv = load_bf16x4(p + C);
#pragma unroll
      for (int e = 0; e < 4; ++e) g[e] = av[e] * sigmoidf_(gv[e]);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) sg[r][c4 + e] = g[e];
  }
  __syncthreads();
  const int c = tid & (CC - 1), rg = tid >> 6;  // 4 row groups of 16
  float wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wk[k] = w[(c0 + c) * K + k];
  const int rbeg = rg * 16;
#pragma unroll 2
  for (int i = 0; i < 16; ++i) {
    const int r = rbeg + i;  // output row t0 + r uses sg[r .. r+K-1]
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) acc += wk[k] * sg[r + k][c];
    const int t = t0 + r;
    if (t < T) out[(int64_t)(b * T + t) * C + c0 + c] = (bf16)acc;
  }
}

// DW = false (frozen layers): only the dout window is staged (24 KB LDS -> 6 blocks/CU).
// DW = true: the GLU output window too, and the [4 row groups][64 ch][K] dW partials are
// reduced through the same LDS after the main pass (48 KB).
template <int K, bool DW>
__global__ __launch_bounds__(NT) void glu_dwconv_bwd_kernel(const bf16* __restrict__ pre, const float* __restrict__ w,
                                                          const bf16* __restrict__ dout, bf16* __restrict__ dpre,
                                                          float* __restrict__ dw, int T, int C) {
  constexpr int ROWS = TT + K - 1;
  __shared__ float lds[(DW ? 2 : 1) * ROWS * CC];
  float (*sd)[CC] = reinterpret_cast<float (*)[CC]>(lds);              // dout rows t0 .. t0+TT+K-2
  float (*sg)[CC] = reinterpret_cast<float (*)[CC]>(lds + ROWS * CC);  // g rows t0-(K-1) .. t0+TT-1 (DW only)
  const int b = blockIdx.z, t0 = blockIdx.x * TT, c0 = blockIdx.y * CC;
  const int tid = threadIdx.x;
  for (int i = tid; i < ROWS * (CC / 4); i += NT) {
    const int r = i / (CC / 4), c4 = (i % (CC / 4)) * 4;
    const int td = t0 + r;
    f32x4 dv = {0.f, 0.f, 0.f, 0.f};
    if (td < T) dv = load_bf16x4(dout + (int64_t)(b * T + td) * C + c0 + c4);
#pragma unroll
    for (int e = 0; e < 4; ++e) sd[r][c4 + e] = dv[e];
    if (DW) {
      const int tg = t0 - (K - 1) + r;
      f32x4 g = {0.f, 0.f, 0.f, 0.f};
      if (tg >= 0 && tg < T) {
        const bf16* p = pre + (int64_t)(b * T + tg) * (2 * C) + c0 + c4;
        f32x4 av = load_bf16x4(p), gv = load_bf16x4(p + C);
#pragma unroll
        for (int e = 0; e < 4; ++e) g[e] = av[e] * sigmoidf_(gv[e]);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) sg[r][c4 + e] = g[e];
    }
  }
  __syncthreads();
  const int c = tid & (CC - 1), rg = tid >> 6;
  float wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wk[k] = w[(c0 + c) * K + k];
  float dwp[DW ? K : 1];
#pragma unroll
  for (int k = 0; k < (DW ? K : 1); ++k) dwp[k] = 0.f;
  const int rbeg = rg * 16;
  for (int i = 0; i < 16; ++i) {
    const int r = rbeg + i;
    const int t = t0 + r;
    // dg[t] = Σ_k w[k] * dout[t + (K-1) - k]  -> sd[r + K-1-k]
    float dg = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) dg += wk[k] * sd[r + (K - 1) - k][c];
    if (DW) {
      // dW[k] += dout[t] * g[t - (K-1) + k] -> sd[r] * sg[r + k]
      const float d0 = sd[r][c];
#pragma unroll
      for (int k = 0; k < K; ++k) dwp[k] += d0 * sg[r + k][c];
    }
    if (t < T) {
      const int64_t row = (int64_t)(b * T + t);
      const float av = (float)pre[row * 2 * C + c0 + c];
      const float gv = (float)pre[row * 2 * C + C + c0 + c];
      const float sgm = sigmoidf_(gv);
      dpre[row * 2 * C + c0 + c] = (bf16)(dg * sgm);
      dpre[row * 2 * C + C + c0 + c] = (bf16)(dg * av * sgm * (1.f - sgm));
    }
  }
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
    atomicAdd(dw + (c0 + cc) * K + k, sum);
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

extern "C" int ste_glu_dwconv_bwd(const void* pre, const float* w, const void* dout, void* dpre, float* dw, int B,
                                  int T, int C, int K, void* stream) {
  if (B <= 0 || T <= 0 || C <= 0 || (C % CC) != 0 || K != KMAX) return STE_ERR_SHAPE;
  dim3 grid((T + TT - 1) / TT, C / CC, B);
  if (dw)
    hipLaunchKernelGGL((glu_dwconv_bwd_kernel<KMAX, true>), grid, dim3(NT), 0, (hipStream_t)stream, (const bf16*)pre,
                       w, (const bf16*)dout, (bf16*)dpre, dw, T, C);
  else
    hipLaunchKernelGGL((glu_dwconv_bwd_kernel<KMAX, false>), grid, dim3(NT), 0, (hipStream_t)stream, (const bf16*)pre,
                       w, (const bf16*)dout, (bf16*)dpre, dw, T, C);
  STE_CHECK_LAUNCH();
  return 0;
}

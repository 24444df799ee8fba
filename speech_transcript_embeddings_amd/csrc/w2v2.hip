// wav2vec2 raw-waveform front end: the kernels around the GEMMs of
//   feature encoder   tf:models/wav2vec2/modeling_wav2vec2.py:254-272,302-323,382-419
//                     (conv0 1->C k=10 s=5 + GroupNorm(C groups) + GELU; convs 1..6 + GELU)
//   pos_conv_embed    tf:…/modeling_wav2vec2.py:326-379 (weight-normed grouped Conv1d k=128,
//                     pad 64, SamePad, GELU) and the encoder prologue :678-692
//   frame mask        tf:…/modeling_wav2vec2.py:997-1036 (_get_feat_extract_output_lengths,
//                     _get_feature_vector_attention_mask)
//   do_normalize      tf:models/wav2vec2/feature_extraction_wav2vec2.py zero_mean_unit_var_norm
//
// Layout: every activation is time-major [B*T, C] (channels contiguous), so a strided Conv1d
// (kernel k, stride s) is a GEMM whose A operand is a VIEW of the input with row stride s*C
// (row t = rows s*t .. s*t+k-1, k*C contiguous elements): no im2col copy.  The grouped
// positional conv uses the same trick on a group-major zero-padded copy [G][B*Tp+K][Cg]
// (row t of the implicit im2col = K*Cg contiguous elements starting at t*Cg).  The GEMMs
// themselves are ste_gemm launches (engine side, wav2vec2.py); this file holds conv0 (C_in=1,
// 10 MACs per output: VALU), GroupNorm, the col2im fold of the backward, the positional-conv
// packing / epilogues, weight norm, and the masks.
#include "common.h"
#include "../../include/ste.h"

namespace {

constexpr int NT = 256;
constexpr int KMAX0 = 16;  // conv0 taps held in registers

// ------------------------------------------------------------------ conv0 forward
// y[b, t, c] = Σ_j w[c, j] · x[b, s·t + j]   (no bias: conv_bias=False)
__global__ __launch_bounds__(NT) void conv0_fwd_kernel(const float* __restrict__ x, int64_t ldx,
                                                       const float* __restrict__ w, float* __restrict__ y, int T0,
                                                       int C, int K0, int S) {
  constexpr int TT = 32;
  __shared__ float sx[TT * 8 + KMAX0];
  const int b = blockIdx.y, t0 = blockIdx.x * TT;
  const int nt = min(TT, T0 - t0);
  const int nsamp = S * (nt - 1) + K0;
  const float* xb = x + (int64_t)b * ldx + (int64_t)S * t0;
  for (int i = threadIdx.x; i < nsamp; i += NT) sx[i] = xb[i];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += NT) {
    float wk[KMAX0];
#pragma unroll
    for (int j = 0; j < KMAX0; ++j) wk[j] = j < K0 ? w[c * K0 + j] : 0.f;
    for (int t = 0; t < nt; ++t) {
      const float* xs = sx + S * t;
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < KMAX0; ++j)
        if (j < K0) acc = fmaf(wk[j], xs[j], acc);
      y[((int64_t)b * T0 + t0 + t) * C + c] = acc;
    }
  }
}

// ------------------------------------------------------------------ GroupNorm(C, C)
// per (b, c) statistics over time (biased variance, two passes in fp64)
__global__ __launch_bounds__(NT) void gn_stats_kernel(const float* __restrict__ y, int T0, int C, float eps,
                                                      float* __restrict__ mean, float* __restrict__ rstd) {
  __shared__ double sred[NT];
  __shared__ double smean[64];
  const int b = blockIdx.y, cl = threadIdx.x & 63, r = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const bool ok = c < C;
  const float* yb = y + (int64_t)b * T0 * C + c;
  double s = 0.0;
  if (ok)
    for (int t = r; t < T0; t += 4) s += (double)yb[(int64_t)t * C];
  sred[threadIdx.x] = s;
  __syncthreads();
  if (r == 0) smean[cl] = (sred[cl] + sred[cl + 64] + sred[cl + 128] + sred[cl + 192]) / (double)T0;
  __syncthreads();
  const double mu = smean[cl];
  double q = 0.0;
  if (ok)
    for (int t = r; t < T0; t += 4) {
      const double d = (double)yb[(int64_t)t * C] - mu;
      q += d * d;
    }
  __syncthreads();
  sred[threadIdx.x] = q;
  __syncthreads();
  if (r == 0 && ok) {
    const double var = (sred[cl] + sred[cl + 64] + sred[cl + 128] + sred[cl + 192]) / (double)T0;
    mean[b * C + c] = (float)mu;
    rstd[b * C + c] = (float)(1.0 / sqrt(var + (double)eps));
  }
}

// h = bf16(gelu((y - mean)·rstd·γ + β)), 4 channels per thread
__global__ __launch_bounds__(NT) void gn_gelu_fwd_kernel(const float* __restrict__ y, const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, const float* __restrict__ g,
                                                         const float* __restrict__ be, int T0, int C, int64_t n4,
                                                         bf16* __restrict__ h) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n4; i += (int64_t)gridDim.x * NT) {
    const int64_t e = i * 4;
    const int64_t row = e / C;
    const int c = (int)(e - row * C);
    const int b = (int)(row / T0);
    const f32x4 v = *reinterpret_cast<const f32x4*>(y + e);
    f32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int bc = b * C + c + k;
      o[k] = gelu_f((v[k] - mean[bc]) * rstd[bc] * g[c + k] + be[c + k]);
    }
    store_bf16x4(h + e, o);
  }
}

// backward, pass 1: per (b, c) s1 = Σ_t dz, s2 = Σ_t dz·x̂ with dz = dh·gelu'(z)
__global__ __launch_bounds__(NT) void gn_bwd_reduce_kernel(const float* __restrict__ dh, const float* __restrict__ y,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ rstd, const float* __restrict__ g,
                                                           const float* __restrict__ be, int T0, int C,
                                                           float* __restrict__ s1, float* __restrict__ s2) {
  __shared__ double r1[NT], r2[NT];
  const int b = blockIdx.y, cl = threadIdx.x & 63, r = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double a1 = 0.0, a2 = 0.0;
  if (c < C) {
    const float mu = mean[b * C + c], rs = rstd[b * C + c], gc = g[c], bc = be[c];
    const int64_t base = (int64_t)b * T0 * C + c;
    for (int t = r; t < T0; t += 4) {
      const float xh = (y[base + (int64_t)t * C] - mu) * rs;
      const float dz = dh[base + (int64_t)t * C] * gelu_d(xh * gc + bc);
      a1 += dz;
      a2 += (double)dz * xh;
    }
  }
  r1[threadIdx.x] = a1;
  r2[threadIdx.x] = a2;
  __syncthreads();
  if (r == 0 && c < C) {
    s1[b * C + c] = (float)(r1[cl] + r1[cl + 64] + r1[cl + 128] + r1[cl + 192]);
    s2[b * C + c] = (float)(r2[cl] + r2[cl + 64] + r2[cl + 128] + r2[cl + 192]);
  }
}

// dγ[c] += Σ_b s2[b,c]; dβ[c] += Σ_b s1[b,c]
__global__ __launch_bounds__(NT) void gn_param_grad_kernel(const float* __restrict__ s1, const float* __restrict__ s2,
                                                           int B, int C, float* __restrict__ dg,
                                                           float* __restrict__ db) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= C) return;
  float a1 = 0.f, a2 = 0.f;
  for (int b = 0; b < B; ++b) {
    a1 += s1[b * C + c];
    a2 += s2[b * C + c];
  }
  if (dg) dg[c] += a2;
  if (db) db[c] += a1;
}

// backward, pass 2: conv0 weight gradient partials.  dy = γ·rstd·(dz - s1/T - x̂·s2/T) is
// recomputed per element; partial[blk][c][j] = Σ_{t in blk} dy[b,t,c]·x[b, s·t + j]
__global__ __launch_bounds__(NT) void conv0_dw_kernel(const float* __restrict__ dh, const float* __restrict__ y,
                                                      const float* __restrict__ mean, const float* __restrict__ rstd,
                                                      const float* __restrict__ g, const float* __restrict__ be,
                                                      const float* __restrict__ s1, const float* __restrict__ s2,
                                                      const float* __restrict__ x, int64_t ldx, int T0, int C, int K0,
                                                      int S, int tchunk, float* __restrict__ part) {
  constexpr int TT = 32;
  __shared__ float sx[TT * 8 + KMAX0];
  const int b = blockIdx.y, tb = blockIdx.x * tchunk, te = min(T0, tb + tchunk);
  const float invT = 1.0f / (float)T0;
  float* pout = part + ((int64_t)b * gridDim.x + blockIdx.x) * C * K0;
  for (int cb = 0; cb < C; cb += NT) {
    const int c = cb + threadIdx.x;
    const bool ok = c < C;
    float mu = 0.f, rs = 0.f, gc = 0.f, bc = 0.f, m1 = 0.f, m2 = 0.f;
    if (ok) {
      mu = mean[b * C + c]; rs = rstd[b * C + c]; gc = g[c]; bc = be[c];
      m1 = s1[b * C + c] * invT; m2 = s2[b * C + c] * invT;
    }
    float acc[KMAX0];
#pragma unroll
    for (int j = 0; j < KMAX0; ++j) acc[j] = 0.f;
    for (int t0 = tb; t0 < te; t0 += TT) {
      const int nt = min(TT, te - t0);
      __syncthreads();
      const int nsamp = S * (nt - 1) + K0;
      const float* xb = x + (int64_t)b * ldx + (int64_t)S * t0;
      for (int i = threadIdx.x; i < nsamp; i += NT) sx[i] = xb[i];
      __syncthreads();
      if (!ok) continue;
      for (int t = 0; t < nt; ++t) {
        const int64_t e = ((int64_t)b * T0 + t0 + t) * C + c;
        const float xh = (y[e] - mu) * rs;
        const float dz = dh[e] * gelu_d(xh * gc + bc);
        const float dy = gc * rs * (dz - m1 - xh * m2);
        const float* xs = sx + S * t;
#pragma unroll
        for (int j = 0; j < KMAX0; ++j)
          if (j < K0) acc[j] = fmaf(dy, xs[j], acc[j]);
      }
    }
    if (ok)
#pragma unroll
      for (int j = 0; j < KMAX0; ++j)
        if (j < K0) pout[c * K0 + j] = acc[j];
  }
}

// out[i] += Σ_s part[s·n + i]   (fixed order: deterministic)
__global__ __launch_bounds__(NT) void slab_sum_kernel(float* __restrict__ out, const float* __restrict__ part,
                                                      int64_t n, int S) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    float a = 0.f;
    for (int s = 0; s < S; ++s) a += part[(int64_t)s * n + i];
    out[i] += a;
  }
}

// ------------------------------------------------------------------ col2im fold
// out[b, ti, c] = act'(z[b,ti,c]) · Σ_{to, j: s·to + j = ti} dcol[b·To + to, j·C + c]
template <bool OUT_BF16>
__global__ __launch_bounds__(NT) void conv_fold_kernel(const float* __restrict__ dcol, int64_t ldd,
                                                       const bf16* __restrict__ z, int Ti, int To, int C, int k, int s,
                                                       int64_t n4, void* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n4; i += (int64_t)gridDim.x * NT) {
    const int64_t e = i * 4;
    const int64_t row = e / C;
    const int c = (int)(e - row * C);
    const int b = (int)(row / Ti), ti = (int)(row - (int64_t)b * Ti);
    int lo = ti - k + 1;
    lo = lo <= 0 ? 0 : (lo + s - 1) / s;
    const int hi = min(To - 1, ti / s);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int to = lo; to <= hi; ++to) {
      const int j = ti - s * to;
      acc += *reinterpret_cast<const f32x4*>(dcol + ((int64_t)b * To + to) * ldd + (int64_t)j * C + c);
    }
    if (z) {
      const f32x4 zz = load_bf16x4(z + e);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] *= gelu_d(zz[q]);
    }
    if (OUT_BF16) store_bf16x4((bf16*)out + e, acc);
    else *reinterpret_cast<f32x4*>((float*)out + e) = acc;
  }
}

// [A][P][Q] -> [A][Q][P] (bf16 -> bf16, or fp32 accumulate into fp32)
template <typename T, bool ACC>
__global__ __launch_bounds__(NT) void perm12_kernel(const T* __restrict__ src, T* __restrict__ dst, int P, int Q,
                                                    int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int64_t a = i / ((int64_t)P * Q);
    const int rem = (int)(i - a * P * Q);
    const int p = rem / Q, q = rem - p * Q;
    T* d = dst + a * P * Q + (int64_t)q * P + p;
    if (ACC) *d += src[i];
    else *d = src[i];
  }
}

// ------------------------------------------------------------------ positional conv
// out [G][B·Tp + K][Cg] bf16: out[g][b·Tp + u][ci] = x[b, u - padl, g·Cg + ci] (0 outside [0,T))
__global__ __launch_bounds__(NT) void pos_pack_kernel(const float* __restrict__ x, int B, int T, int D, int Cg, int Tp,
                                                      int K, int padl, int64_t n8, bf16* __restrict__ out) {
  const int cg8 = Cg / 8;
  const int64_t rows = (int64_t)B * Tp + K;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n8; i += (int64_t)gridDim.x * NT) {
    const int ci = (int)(i % cg8) * 8;
    const int64_t gr = i / cg8;
    const int g = (int)(gr / rows);
    const int64_t row = gr - (int64_t)g * rows;
    bf16x8 v = {};
    if (row < (int64_t)B * Tp) {
      const int b = (int)(row / Tp), t = (int)(row - (int64_t)b * Tp) - padl;
      if (t >= 0 && t < T) {
        const float* p = x + ((int64_t)b * T + t) * D + g * Cg + ci;
        const f32x4 a = *reinterpret_cast<const f32x4*>(p), c = *reinterpret_cast<const f32x4*>(p + 4);
        v = bf16x8{(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)c[0], (bf16)c[1], (bf16)c[2], (bf16)c[3]};
      }
    }
    *reinterpret_cast<bf16x8*>(out + gr * Cg + ci) = v;
  }
}

// MODE 0 (post):  out = x + gelu(cpad + bias)
// MODE 1 (dpc):   out = dxe · gelu'(cpad + bias)
// MODE 2 (unpad): out = (dxe + cpad) · maskf[row]   (cpad = dX of the conv)
template <int MODE>
__global__ __launch_bounds__(NT) void pos_elem_kernel(const float* __restrict__ cpad, const float* __restrict__ bias,
                                                      const float* __restrict__ src, const float* __restrict__ maskf,
                                                      int T, int D, int Tp, int64_t n4, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n4; i += (int64_t)gridDim.x * NT) {
    const int64_t e = i * 4;
    const int64_t row = e / D;
    const int c = (int)(e - row * D);
    const int b = (int)(row / T), t = (int)(row - (int64_t)b * T);
    const f32x4 cv = *reinterpret_cast<const f32x4*>(cpad + ((int64_t)b * Tp + t) * D + c);
    const f32x4 sv = *reinterpret_cast<const f32x4*>(src + e);
    f32x4 o;
    if (MODE == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = sv[q] + gelu_f(cv[q] + bias[c + q]);
    } else if (MODE == 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = sv[q] * gelu_d(cv[q] + bias[c + q]);
    } else {
      const float m = maskf ? maskf[row] : 1.0f;
      o = (sv + cv) * m;
    }
    *reinterpret_cast<f32x4*>(out + e) = o;
  }
}

// weight norm over dims (0, 1) for each kernel tap j (nn.utils.parametrizations.weight_norm,
// dim=2): W[o, i, j] = g[j] · v[o, i, j] / ‖v[:, :, j]‖.  One block per tap.  Writes the
// forward B operand wr[grp][co][j][ci] and the flipped one of the input gradient
// wf[grp][ci][K-1-j][co] (bf16), and norms[j].
__global__ __launch_bounds__(NT) void wnorm_fwd_kernel(const float* __restrict__ v, const float* __restrict__ gp,
                                                       int D, int Cg, int K, float* __restrict__ norms,
                                                       bf16* __restrict__ wr, bf16* __restrict__ wf) {
  __shared__ double sred[NT];
  const int j = blockIdx.x;
  const int n = D * Cg;
  double s = 0.0;
  for (int e = threadIdx.x; e < n; e += NT) {
    const double a = v[(int64_t)e * K + j];
    s += a * a;
  }
  sred[threadIdx.x] = s;
  __syncthreads();
  for (int o = NT / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) sred[threadIdx.x] += sred[threadIdx.x + o];
    __syncthreads();
  }
  const float nrm = (float)sqrt(sred[0]);
  if (threadIdx.x == 0) norms[j] = nrm;
  const float sc = gp[j] / nrm;
  for (int e = threadIdx.x; e < n; e += NT) {
    const int o = e / Cg, ci = e - o * Cg;
    const int grp = o / Cg, co = o - grp * Cg;
    const bf16 w = (bf16)(v[(int64_t)e * K + j] * sc);
    wr[(((int64_t)grp * Cg + co) * K + j) * Cg + ci] = w;
    wf[(((int64_t)grp * Cg + ci) * K + (K - 1 - j)) * Cg + co] = w;
  }
}

// dW (wr layout, fp32) -> dg[j] += s_j/n_j, dv[o,i,j] += (g_j/n_j)·dW - (g_j·s_j/n_j³)·v,
// s_j = Σ_{o,i} dW·v
__global__ __launch_bounds__(NT) void wnorm_bwd_kernel(const float* __restrict__ dwr, const float* __restrict__ v,
                                                       const float* __restrict__ gp, const float* __restrict__ norms,
                                                       int D, int Cg, int K, float* __restrict__ dv,
                                                       float* __restrict__ dg) {
  __shared__ double sred[NT];
  const int j = blockIdx.x;
  const int n = D * Cg;
  double s = 0.0;
  for (int e = threadIdx.x; e < n; e += NT) {
    const int o = e / Cg, ci = e - o * Cg;
    const int grp = o / Cg, co = o - grp * Cg;
    s += (double)dwr[(((int64_t)grp * Cg + co) * K + j) * Cg + ci] * (double)v[(int64_t)e * K + j];
  }
  sred[threadIdx.x] = s;
  __syncthreads();
  for (int o = NT / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) sred[threadIdx.x] += sred[threadIdx.x + o];
    __syncthreads();
  }
  const float nrm = norms[j], gj = gp[j];
  const float sj = (float)sred[0];
  if (threadIdx.x == 0 && dg) dg[j] += sj / nrm;
  if (!dv) return;
  const float a = gj / nrm, c = gj * sj / (nrm * nrm * nrm);
  for (int e = threadIdx.x; e < n; e += NT) {
    const int o = e / Cg, ci = e - o * Cg;
    const int grp = o / Cg, co = o - grp * Cg;
    const int64_t iv = (int64_t)e * K + j;
    dv[iv] += a * dwr[(((int64_t)grp * Cg + co) * K + j) * Cg + ci] - c * v[iv];
  }
}

// ------------------------------------------------------------------ masks / normalisation
struct ConvStack {
  int n;
  int k[16], s[16];
};

// per clip: valid samples = Σ mask (or N), conv output lengths, mask[b, t] = t < L
// (L <= 0: transformers' index -1 assignment marks every frame valid)
__global__ __launch_bounds__(NT) void frame_mask_kernel(const int64_t* __restrict__ mask, int N, int Tf, ConvStack cs,
                                                        float* __restrict__ maskf, int* __restrict__ mask32) {
  __shared__ long long sred[NT];
  const int b = blockIdx.x;
  long long s = 0;
  if (mask)
    for (int n = threadIdx.x; n < N; n += NT) s += mask[(int64_t)b * N + n];
  else if (threadIdx.x == 0)
    s = N;
  sred[threadIdx.x] = s;
  __syncthreads();
  for (int o = NT / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) sred[threadIdx.x] += sred[threadIdx.x + o];
    __syncthreads();
  }
  long long L = sred[0];
  for (int i = 0; i < cs.n; ++i) {
    const long long d = L - cs.k[i];
    L = (d >= 0 ? d / cs.s[i] : -((-d + cs.s[i] - 1) / cs.s[i])) + 1;  // floor division
  }
  if (L <= 0) L = Tf;
  for (int t = threadIdx.x; t < Tf; t += NT) {
    const int on = t < L;
    if (maskf) maskf[(int64_t)b * Tf + t] = (float)on;
    if (mask32) mask32[(int64_t)b * Tf + t] = on;
  }
}

// Wav2Vec2FeatureExtractor(do_normalize=True): (x - mean)/sqrt(var + 1e-7) over the clip's
// first len samples (population variance), padding_value after.  One block per clip.
__global__ __launch_bounds__(NT) void wave_norm_kernel(const float* __restrict__ x, int64_t ldx,
                                                       const int* __restrict__ lens, int N, float pad,
                                                       float* __restrict__ out) {
  __shared__ double sred[NT];
  const int b = blockIdx.x;
  const int len = lens ? min(lens[b], N) : N;
  const float* xb = x + (int64_t)b * ldx;
  double s = 0.0;
  for (int n = threadIdx.x; n < len; n += NT) s += xb[n];
  sred[threadIdx.x] = s;
  __syncthreads();
  for (int o = NT / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) sred[threadIdx.x] += sred[threadIdx.x + o];
    __syncthreads();
  }
  const double mu = len > 0 ? sred[0] / len : 0.0;
  __syncthreads();
  double q = 0.0;
  for (int n = threadIdx.x; n < len; n += NT) {
    const double d = xb[n] - mu;
    q += d * d;
  }
  sred[threadIdx.x] = q;
  __syncthreads();
  for (int o = NT / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) sred[threadIdx.x] += sred[threadIdx.x + o];
    __syncthreads();
  }
  const double inv = len > 0 ? 1.0 / sqrt(sred[0] / len + 1e-7) : 0.0;
  for (int n = threadIdx.x; n < N; n += NT)
    out[(int64_t)b * N + n] = n < len ? (float)((xb[n] - mu) * inv) : pad;
}

// dropout (GEMM epilogue index row·ld + col) and row mask applied to a gradient in place
__global__ __launch_bounds__(NT) void drop_rows_kernel(float* __restrict__ x, int N, int64_t n, float p, uint64_t seed,
                                                       const float* __restrict__ maskf) {
  const uint32_t thresh = (uint32_t)(p * 4294967296.0);
  const float inv_keep = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    float v = x[i];
    if (p > 0.f) v *= drop_scale(seed, (uint64_t)i, thresh, inv_keep);
    if (maskf) v *= maskf[i / N];
    x[i] = v;
  }
}

int grid_for(int64_t n) {
  const int64_t b = (n + NT - 1) / NT;
  return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

}  // namespace

extern "C" int ste_w2v_conv0_fwd(const float* wave, int64_t ldw, const float* w0, int B, int N, int T0, int C, int K0,
                                 int S0, float* y, void* stream) {
  if (B <= 0 || T0 <= 0 || C <= 0 || K0 <= 0 || K0 > KMAX0 || S0 <= 0 || S0 > 8 || ldw < N ||
      (int64_t)S0 * (T0 - 1) + K0 > N)
    return STE_ERR_SHAPE;
  hipLaunchKernelGGL(conv0_fwd_kernel, dim3((T0 + 31) / 32, B), dim3(NT), 0, (hipStream_t)stream, wave, ldw, w0, y, T0,
                     C, K0, S0);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_w2v_gn_fwd(const float* y, const float* gamma, const float* beta, int B, int T0, int C, float eps,
                              float* mean, float* rstd, void* h, void* stream) {
  if (B <= 0 || T0 <= 0 || C <= 0 || (C & 3)) return STE_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(gn_stats_kernel, dim3((C + 63) / 64, B), dim3(NT), 0, s, y, T0, C, eps, mean, rstd);
  STE_CHECK_LAUNCH();
  const int64_t n4 = (int64_t)B * T0 * C / 4;
  hipLaunchKernelGGL(gn_gelu_fwd_kernel, dim3(grid_for(n4)), dim3(NT), 0, s, y, mean, rstd, gamma, beta, T0, C, n4,
                     (bf16*)h);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t ste_w2v_gn_bwd_work(int B, int T0, int C, int K0) {
  const int tchunk = 256;
  const int nchunk = (T0 + tchunk - 1) / tchunk;
  return (int64_t)2 * B * C + (int64_t)B * nchunk * C * K0;
}

extern "C" int ste_w2v_gn_bwd(const float* dh, const float* y, const float* mean, const float* rstd,
                              const float* gamma, const float* beta, const float* wave, int64_t ldw, int B, int N,
                              int T0, int C, int K0, int S0, float* dgamma, float* dbeta, float* dw0, float* work,
                              int64_t work_floats, void* stream) {
  if (B <= 0 || T0 <= 0 || C <= 0 || K0 <= 0 || K0 > KMAX0 || S0 <= 0 || S0 > 8 || !work) return STE_ERR_SHAPE;
  if (work_floats < ste_w2v_gn_bwd_work(B, T0, C, K0)) return STE_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  float* s1 = work;
  float* s2 = work + (int64_t)B * C;
  hipLaunchKernelGGL(gn_bwd_reduce_kernel, dim3((C + 63) / 64, B), dim3(NT), 0, s, dh, y, mean, rstd, gamma, beta, T0,
                     C, s1, s2);
  STE_CHECK_LAUNCH();
  if (dgamma || dbeta) {
    hipLaunchKernelGGL(gn_param_grad_kernel, dim3((C + NT - 1) / NT), dim3(NT), 0, s, s1, s2, B, C, dgamma, dbeta);
    STE_CHECK_LAUNCH();
  }
  if (dw0) {
    const int tchunk = 256;
    const int nchunk = (T0 + tchunk - 1) / tchunk;
    float* part = work + (int64_t)2 * B * C;
    hipLaunchKernelGGL(conv0_dw_kernel, dim3(nchunk, B), dim3(NT), 0, s, dh, y, mean, rstd, gamma, beta, s1, s2, wave,
                       ldw, T0, C, K0, S0, tchunk, part);
    STE_CHECK_LAUNCH();
    const int64_t n = (int64_t)C * K0;
    hipLaunchKernelGGL(slab_sum_kernel, dim3(grid_for(n)), dim3(NT), 0, s, dw0, part, n, B * nchunk);
    STE_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int ste_w2v_slab_sum(float* out, const float* part, int64_t n, int S, void* stream) {
  if (n <= 0 || S <= 0) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(slab_sum_kernel, dim3(grid_for(n)), dim3(NT), 0, (hipStream_t)stream, out, part, n, S);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_w2v_conv_fold(const float* dcol, int64_t ldd, const void* z, int B, int Ti, int To, int C, int k,
                                 int s, void* out, int out_bf16, void* stream) {
  if (B <= 0 || Ti <= 0 || To <= 0 || C <= 0 || (C & 3) || k <= 0 || s <= 0 || ldd < (int64_t)k * C || (ldd & 3) ||
      (int64_t)s * (To - 1) + k > Ti)
    return STE_ERR_SHAPE;
  const int64_t n4 = (int64_t)B * Ti * C / 4;
  if (out_bf16)
    hipLaunchKernelGGL(conv_fold_kernel<true>, dim3(grid_for(n4)), dim3(NT), 0, (hipStream_t)stream, dcol, ldd,
                       (const bf16*)z, Ti, To, C, k, s, n4, out);
  else
    hipLaunchKernelGGL(conv_fold_kernel<false>, dim3(grid_for(n4)), dim3(NT), 0, (hipStream_t)stream, dcol, ldd,
                       (const bf16*)z, Ti, To, C, k, s, n4, out);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_w2v_perm12(const void* src, void* dst, int A, int P, int Q, int fp32_accumulate, void* stream) {
  if (A <= 0 || P <= 0 || Q <= 0) return STE_ERR_SHAPE;
  const int64_t n = (int64_t)A * P * Q;
  if (fp32_accumulate)
    hipLaunchKernelGGL((perm12_kernel<float, true>), dim3(grid_for(n)), dim3(NT), 0, (hipStream_t)stream,
                       (const float*)src, (float*)dst, P, Q, n);
  else
    hipLaunchKernelGGL((perm12_kernel<bf16, false>), dim3(grid_for(n)), dim3(NT), 0, (hipStream_t)stream,
                       (const bf16*)src, (bf16*)dst, P, Q, n);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_w2v_pos_pack(const float* x, int B, int T, int D, int G, int K, int padl, void* out, void* stream) {
  if (B <= 0 || T <= 0 || G <= 0 || D % G || (D / G) % 8 || K <= 0 || padl < 0 || padl >= K) return STE_ERR_SHAPE;
  const int Cg = D / G, Tp = T + K - 1;
  const int64_t n8 = (int64_t)G * ((int64_t)B * Tp + K) * Cg / 8;
  hipLaunchKernelGGL(pos_pack_kernel, dim3(grid_for(n8)), dim3(NT), 0, (hipStream_t)stream, x, B, T, D, Cg, Tp, K, padl,
                     n8, (bf16*)out);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_w2v_pos_elem(int mode, const float* cpad, const float* bias, const float* src, const float* maskf,
                                int B, int T, int D, int Tp, float* out, void* stream) {
  if (B <= 0 || T <= 0 || D <= 0 || (D & 3) || Tp < T || mode < 0 || mode > 2 || (mode < 2 && !bias))
    return STE_ERR_SHAPE;
  const int64_t n4 = (int64_t)B * T * D / 4;
  hipStream_t s = (hipStream_t)stream;
  if (mode == 0)
    hipLaunchKernelGGL(pos_elem_kernel<0>, dim3(grid_for(n4)), dim3(NT), 0, s, cpad, bias, src, maskf, T, D, Tp, n4, out);
  else if (mode == 1)
    hipLaunchKernelGGL(pos_elem_kernel<1>, dim3(grid_for(n4)), dim3(NT), 0, s, cpad, bias, src, maskf, T, D, Tp, n4, out);
  else
    hipLaunchKernelGGL(pos_elem_kernel<2>, dim3(grid_for(n4)), dim3(NT), 0, s, cpad, bias, src, maskf, T, D, Tp, n4, out);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_w2v_wnorm_fwd(const float* v, const float* g, int D, int Cg, int K, float* norms, void* wr,
                                 void* wf, void* stream) {
  if (D <= 0 || Cg <= 0 || D % Cg || K <= 0) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(wnorm_fwd_kernel, dim3(K), dim3(NT), 0, (hipStream_t)stream, v, g, D, Cg, K, norms, (bf16*)wr,
                     (bf16*)wf);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_w2v_wnorm_bwd(const float* dwr, const float* v, const float* g, const float* norms, int D, int Cg,
                                 int K, float* dv, float* dg, void* stream) {
  if (D <= 0 || Cg <= 0 || D % Cg || K <= 0) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(wnorm_bwd_kernel, dim3(K), dim3(NT), 0, (hipStream_t)stream, dwr, v, g, norms, D, Cg, K, dv, dg);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_w2v_frame_mask(const int64_t* mask, int B, int N, int Tf, int nconv, const int* kernels,
                                  const int* strides, float* maskf, int* mask32, void* stream) {
  if (B <= 0 || N <= 0 || Tf <= 0 || nconv <= 0 || nconv > 16 || !kernels || !strides) return STE_ERR_SHAPE;
  ConvStack cs;
  cs.n = nconv;
  for (int i = 0; i < nconv; ++i) {
    if (kernels[i] <= 0 || strides[i] <= 0) return STE_ERR_SHAPE;
    cs.k[i] = kernels[i];
    cs.s[i] = strides[i];
  }
  hipLaunchKernelGGL(frame_mask_kernel, dim3(B), dim3(NT), 0, (hipStream_t)stream, mask, N, Tf, cs, maskf, mask32);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_w2v_wave_norm(const float* wave, int64_t ldw, const int* lengths, int B, int N, float pad,
                                 float* out, void* stream) {
  if (B <= 0 || N <= 0 || ldw < N) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(wave_norm_kernel, dim3(B), dim3(NT), 0, (hipStream_t)stream, wave, ldw, lengths, N, pad, out);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_w2v_drop_rows(float* x, int M, int N, float p, uint64_t seed, const float* maskf, void* stream) {
  if (M <= 0 || N <= 0 || p < 0.f || p >= 1.f) return STE_ERR_SHAPE;
  const int64_t n = (int64_t)M * N;
  hipLaunchKernelGGL(drop_rows_kernel, dim3(grid_for(n)), dim3(NT), 0, (hipStream_t)stream, x, N, n, p, seed, maskf);
  STE_CHECK_LAUNCH();
  return 0;
}

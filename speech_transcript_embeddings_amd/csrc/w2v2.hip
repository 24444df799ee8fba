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
// Per (b, c) reductions over time, one pass: a block sums GN_ROWS rows of one clip for every
// channel (16-B loads of 4 channels, fp64 partial sums, row groups combined in LDS) into
// part[b][chunk][2][C]; a finalize kernel sums the chunks.
//   MODE 0 (forward):  Σ y, Σ y²
//   MODE 1 (backward): Σ dz, Σ dz·x̂ with x̂ = (y - mean)·rstd, dz = dh·gelu'(x̂·γ + β)
constexpr int GN_ROWS = 512;

template <int MODE>
__global__ __launch_bounds__(NT) void gn_partial_kernel(const float* __restrict__ y, const float* __restrict__ dh,
                                                        const float* __restrict__ mean, const float* __restrict__ rstd,
                                                        const float* __restrict__ g, const float* __restrict__ be,
                                                        int T0, int C, double* __restrict__ part) {
  __shared__ double sred[NT * 8];
  const int Q = C >> 2, groups = NT / Q;
  const int b = blockIdx.y, chunk = blockIdx.x, nchunk = gridDim.x;
  const int q = threadIdx.x % Q, rg = threadIdx.x / Q;
  const int t0 = chunk * GN_ROWS, t1 = min(T0, t0 + GN_ROWS);
  double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (rg < groups) {
    const int c = q * 4;
    f32x4 mu = {}, rs = {}, gc = {}, bc = {};
    if (MODE == 1) {
      mu = *reinterpret_cast<const f32x4*>(mean + b * C + c);
      rs = *reinterpret_cast<const f32x4*>(rstd + b * C + c);
      gc = *reinterpret_cast<const f32x4*>(g + c);
      bc = *reinterpret_cast<const f32x4*>(be + c);
    }
    for (int t = t0 + rg; t < t1; t += groups) {
      const int64_t off = ((int64_t)b * T0 + t) * C + c;
      const f32x4 v = *reinterpret_cast<const f32x4*>(y + off);
      if (MODE == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          a[k] += (double)v[k];
          a[4 + k] += (double)v[k] * (double)v[k];
        }
      } else {
        const f32x4 d = *reinterpret_cast<const f32x4*>(dh + off);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float xh = (v[k] - mu[k]) * rs[k];
          const float dz = d[k] * gelu_d(xh * gc[k] + bc[k]);
          a[k] += (double)dz;
          a[4 + k] += (double)dz * (double)xh;
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) sred[k * NT + threadIdx.x] = a[k];
  __syncthreads();
  if (rg == 0) {
    for (int r = 1; r < groups; ++r)
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] += sred[k * NT + r * Q + q];
    double* p = part + ((int64_t)b * nchunk + chunk) * 2 * C + q * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      p[k] = a[k];
      p[C + k] = a[4 + k];
    }
  }
}

// MODE 0: mean, rstd (biased variance) from Σy, Σy².  MODE 1: s1 = Σdz, s2 = Σdz·x̂ (fp32).
template <int MODE>
__global__ __launch_bounds__(NT) void gn_finalize_kernel(const double* __restrict__ part, int nchunk, int T0, int C,
                                                         float eps, float* __restrict__ o1, float* __restrict__ o2) {
  const int b = blockIdx.y, c = blockIdx.x * NT + threadIdx.x;
  if (c >= C) return;
  double s1 = 0.0, s2 = 0.0;
  for (int k = 0; k < nchunk; ++k) {
    const double* p = part + ((int64_t)b * nchunk + k) * 2 * C;
    s1 += p[c];
    s2 += p[C + c];
  }
  if (MODE == 0) {
    const double mu = s1 / T0;
    const double var = fmax(s2 / T0 - mu * mu, 0.0);
    o1[b * C + c] = (float)mu;
    o2[b * C + c] = (float)(1.0 / sqrt(var + (double)eps));
  } else {
    o1[b * C + c] = (float)s1;
    o2[b * C + c] = (float)s2;
  }
}

// h = bf16(gelu((y - mean)·rstd·γ + β)): a block per 8 rows, 4 channels per thread
__global__ __launch_bounds__(NT) void gn_gelu_fwd_kernel(const float* __restrict__ y, const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, const float* __restrict__ g,
                                                         const float* __restrict__ be, int rows, int T0, int C,
                                                         bf16* __restrict__ h) {
  const int Q = C >> 2;
  const int r0 = blockIdx.x * 8;
  for (int i = threadIdx.x; i < 8 * Q; i += NT) {
    const int row = r0 + i / Q, c = (i % Q) * 4;
    if (row >= rows) break;
    const int bc = (row / T0) * C + c;
    const int64_t e = (int64_t)row * C + c;
    const f32x4 v = *reinterpret_cast<const f32x4*>(y + e);
    const f32x4 mu = *reinterpret_cast<const f32x4*>(mean + bc), rs = *reinterpret_cast<const f32x4*>(rstd + bc);
    const f32x4 gc = *reinterpret_cast<const f32x4*>(g + c), bb = *reinterpret_cast<const f32x4*>(be + c);
    f32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = gelu_f((v[k] - mu[k]) * rs[k] * gc[k] + bb[k]);
    store_bf16x4(h + e, o);
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

// ACC: out[i] += Σ_s part[s·n + i];  else out[g·n + i] = Σ_{s in group g of SG} part[s·n + i]
// (fixed order: deterministic; the grouped form splits long sums over blockIdx.y)
template <bool ACC>
__global__ __launch_bounds__(NT) void slab_sum_kernel(float* __restrict__ out, const float* __restrict__ part,
                                                      int64_t n, int S, int SG) {
  const int s0 = ACC ? 0 : blockIdx.y * SG, s1 = ACC ? S : min(S, s0 + SG);
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    float a = 0.f;
    for (int s = s0; s < s1; ++s) a += part[(int64_t)s * n + i];
    if (ACC) out[i] += a;
    else out[(int64_t)blockIdx.y * n + i] = a;
  }
}

// ------------------------------------------------------------------ col2im fold
// out[b, ti, c] = act'(z[b,ti,c]) · Σ_{to, j: s·to + j = ti} dcol[b·To + to, j·C + c]
template <bool OUT_BF16>
__global__ __launch_bounds__(NT) void conv_fold_kernel(const float* __restrict__ dcol, int64_t ldd,
                                                       const bf16* __restrict__ z, int rows, int Ti, int To, int C,
                                                       int k, int s, void* __restrict__ out) {
  const int Q = C >> 2;
  const int r0 = blockIdx.x * 8;
  for (int i = threadIdx.x; i < 8 * Q; i += NT) {
    const int row = r0 + i / Q, c = (i % Q) * 4;
    if (row >= rows) break;
    const int b = row / Ti, ti = row - b * Ti;
    int lo = ti - k + 1;
    lo = lo <= 0 ? 0 : (lo + s - 1) / s;
    const int hi = min(To - 1, ti / s);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int to = lo; to <= hi; ++to) {
      const int j = ti - s * to;
      acc += *reinterpret_cast<const f32x4*>(dcol + ((int64_t)b * To + to) * ldd + j * C + c);
    }
    const int64_t e = (int64_t)row * C + c;
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
                                                      int K, int padl, int n8, bf16* __restrict__ out) {
  const int cg8 = Cg / 8;
  const int rows = B * Tp + K;
  for (int i = blockIdx.x * NT + threadIdx.x; i < n8; i += gridDim.x * NT) {
    const int gr = i / cg8, ci = (i - gr * cg8) * 8;
    const int g = gr / rows, row = gr - g * rows;
    bf16x8 v = {};
    if (row < B * Tp) {
      const int b = row / Tp, t = row - b * Tp - padl;
      if (t >= 0 && t < T) {
        const float* p = x + ((int64_t)b * T + t) * D + g * Cg + ci;
        const f32x4 a = *reinterpret_cast<const f32x4*>(p), c = *reinterpret_cast<const f32x4*>(p + 4);
        v = bf16x8{(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)c[0], (bf16)c[1], (bf16)c[2], (bf16)c[3]};
      }
    }
    *reinterpret_cast<bf16x8*>(out + (int64_t)gr * Cg + ci) = v;
  }
}

// MODE 0 (post):  out = x + gelu(cpad + bias)
// MODE 1 (dpc):   out = dxe · gelu'(cpad + bias)
// MODE 2 (unpad): out = (dxe + cpad) · maskf[row]   (cpad = dX of the conv)
template <int MODE>
__global__ __launch_bounds__(NT) void pos_elem_kernel(const float* __restrict__ cpad, const float* __restrict__ bias,
                                                      const float* __restrict__ src, const float* __restrict__ maskf,
                                                      int T, int D, int Tp, int n4, float* __restrict__ out) {
  const int Q = D >> 2;
  for (int i = blockIdx.x * NT + threadIdx.x; i < n4; i += gridDim.x * NT) {
    const int row = i / Q, c = (i - row * Q) * 4;
    const int b = row / T, t = row - b * T;
    const int64_t e = (int64_t)row * D + c;
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

namespace {
struct GnPlan {
  int nchunk;        // GN_ROWS-row chunks per clip (GroupNorm partial sums)
  int tchunk, nc0;   // conv0 weight-gradient rows per block, blocks per clip
  int64_t part_f, s12_f, dw_f, dw2_f;  // work sections, in floats
};
GnPlan gn_plan(int B, int T0, int C, int K0) {
  GnPlan p;
  p.nchunk = (T0 + GN_ROWS - 1) / GN_ROWS;
  int nc0 = (1024 + B - 1) / B;
  nc0 = max(1, min(nc0, (T0 + 31) / 32));
  p.tchunk = ((T0 + nc0 - 1) / nc0 + 31) / 32 * 32;
  p.nc0 = (T0 + p.tchunk - 1) / p.tchunk;
  p.part_f = (int64_t)B * p.nchunk * 2 * C * 2;  // doubles
  p.s12_f = (int64_t)2 * B * C;
  p.dw_f = (int64_t)B * p.nc0 * C * K0;
  p.dw2_f = (int64_t)((B * p.nc0 + 31) / 32) * C * K0;
  return p;
}
bool gn_shape_ok(int B, int T0, int C) { return B > 0 && T0 > 0 && C > 0 && (C & 3) == 0 && C <= 4 * NT; }
}  // namespace

extern "C" int64_t ste_w2v_gn_work(int B, int T0, int C, int K0) {
  if (!gn_shape_ok(B, T0, C)) return 0;
  const GnPlan p = gn_plan(B, T0, C, K0);
  return p.part_f + p.s12_f + p.dw_f + p.dw2_f;
}

extern "C" int ste_w2v_gn_fwd(const float* y, const float* gamma, const float* beta, int B, int T0, int C, float eps,
                              float* mean, float* rstd, void* h, float* work, int64_t work_floats, void* stream) {
  if (!gn_shape_ok(B, T0, C) || !work || work_floats < ste_w2v_gn_work(B, T0, C, 1)) return STE_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  const GnPlan p = gn_plan(B, T0, C, 1);
  double* part = reinterpret_cast<double*>(work);
  hipLaunchKernelGGL(gn_partial_kernel<0>, dim3(p.nchunk, B), dim3(NT), 0, s, y, nullptr, nullptr, nullptr, nullptr,
                     nullptr, T0, C, part);
  STE_CHECK_LAUNCH();
  hipLaunchKernelGGL(gn_finalize_kernel<0>, dim3((C + NT - 1) / NT, B), dim3(NT), 0, s, part, p.nchunk, T0, C, eps,
                     mean, rstd);
  STE_CHECK_LAUNCH();
  const int rows = B * T0;
  hipLaunchKernelGGL(gn_gelu_fwd_kernel, dim3((rows + 7) / 8), dim3(NT), 0, s, y, mean, rstd, gamma, beta, rows, T0, C,
                     (bf16*)h);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_w2v_gn_bwd(const float* dh, const float* y, const float* mean, const float* rstd,
                              const float* gamma, const float* beta, const float* wave, int64_t ldw, int B, int N,
                              int T0, int C, int K0, int S0, float* dgamma, float* dbeta, float* dw0, float* work,
                              int64_t work_floats, void* stream) {
  if (!gn_shape_ok(B, T0, C) || K0 <= 0 || K0 > KMAX0 || S0 <= 0 || S0 > 8 || !work ||
      (int64_t)S0 * (T0 - 1) + K0 > N || ldw < N)
    return STE_ERR_SHAPE;
  if (work_floats < ste_w2v_gn_work(B, T0, C, K0)) return STE_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  const GnPlan p = gn_plan(B, T0, C, K0);
  double* part = reinterpret_cast<double*>(work);
  float* s1 = work + p.part_f;
  float* s2 = s1 + (int64_t)B * C;
  hipLaunchKernelGGL(gn_partial_kernel<1>, dim3(p.nchunk, B), dim3(NT), 0, s, y, dh, mean, rstd, gamma, beta, T0, C,
                     part);
  STE_CHECK_LAUNCH();
  hipLaunchKernelGGL(gn_finalize_kernel<1>, dim3((C + NT - 1) / NT, B), dim3(NT), 0, s, part, p.nchunk, T0, C, 0.f, s1,
                     s2);
  STE_CHECK_LAUNCH();
  if (dgamma || dbeta) {
    hipLaunchKernelGGL(gn_param_grad_kernel, dim3((C + NT - 1) / NT), dim3(NT), 0, s, s1, s2, B, C, dgamma, dbeta);
    STE_CHECK_LAUNCH();
  }
  if (dw0) {
    float* dpart = s1 + p.s12_f;
    float* dpart2 = dpart + p.dw_f;
    hipLaunchKernelGGL(conv0_dw_kernel, dim3(p.nc0, B), dim3(NT), 0, s, dh, y, mean, rstd, gamma, beta, s1, s2, wave,
                       ldw, T0, C, K0, S0, p.tchunk, dpart);
    STE_CHECK_LAUNCH();
    const int64_t n = (int64_t)C * K0;
    const int S = B * p.nc0, S2 = (S + 31) / 32;
    hipLaunchKernelGGL(slab_sum_kernel<false>, dim3(grid_for(n), S2), dim3(NT), 0, s, dpart2, dpart, n, S, 32);
    STE_CHECK_LAUNCH();
    hipLaunchKernelGGL(slab_sum_kernel<true>, dim3(grid_for(n)), dim3(NT), 0, s, dw0, dpart2, n, S2, 0);
    STE_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int ste_w2v_slab_sum(float* out, const float* part, int64_t n, int S, void* stream) {
  if (n <= 0 || S <= 0) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(slab_sum_kernel<true>, dim3(grid_for(n)), dim3(NT), 0, (hipStream_t)stream, out, part, n, S, 0);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_w2v_conv_fold(const float* dcol, int64_t ldd, const void* z, int B, int Ti, int To, int C, int k,
                                 int s, void* out, int out_bf16, void* stream) {
  if (B <= 0 || Ti <= 0 || To <= 0 || C <= 0 || (C & 3) || k <= 0 || s <= 0 || ldd < (int64_t)k * C || (ldd & 3) ||
      (int64_t)s * (To - 1) + k > Ti || (int64_t)B * Ti >= (1ll << 31))
    return STE_ERR_SHAPE;
  const int rows = B * Ti;
  if (out_bf16)
    hipLaunchKernelGGL(conv_fold_kernel<true>, dim3((rows + 7) / 8), dim3(NT), 0, (hipStream_t)stream, dcol, ldd,
                       (const bf16*)z, rows, Ti, To, C, k, s, out);
  else
    hipLaunchKernelGGL(conv_fold_kernel<false>, dim3((rows + 7) / 8), dim3(NT), 0, (hipStream_t)stream, dcol, ldd,
                       (const bf16*)z, rows, Ti, To, C, k, s, out);
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
  if ((int64_t)G * ((int64_t)B * Tp + K) * Cg / 8 >= (1ll << 31)) return STE_ERR_SHAPE;
  const int n8 = G * (B * Tp + K) * Cg / 8;
  hipLaunchKernelGGL(pos_pack_kernel, dim3(grid_for(n8)), dim3(NT), 0, (hipStream_t)stream, x, B, T, D, Cg, Tp, K, padl,
                     n8, (bf16*)out);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_w2v_pos_elem(int mode, const float* cpad, const float* bias, const float* src, const float* maskf,
                                int B, int T, int D, int Tp, float* out, void* stream) {
  if (B <= 0 || T <= 0 || D <= 0 || (D & 3) || Tp < T || mode < 0 || mode > 2 || (mode < 2 && !bias) ||
      (int64_t)B * T * D / 4 >= (1ll << 31))
    return STE_ERR_SHAPE;
  const int n4 = B * T * D / 4;
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

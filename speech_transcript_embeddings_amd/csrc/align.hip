// WordLevelAlignmentModule core (ref:training/trainer_unfreeze.py:214-310, config 4):
// nn.MultiheadAttention(P, 4 heads, batch_first) from text tokens (queries) to audio
// frames (keys/values) with key_padding_mask, probabilities dropout, plus the rank-1
// backward of the confidence head's last Linear.  Head dim P/4 = 192 at full size:
// the L x T score tiles are small (64 x 499 per (b,h)), so these are SIMT kernels —
// 8 queries per block share every key/value row they stream.
#include "common.h"
#include "../../include/ste.h"

namespace {

constexpr int NT = 256, QB = 8, KB = 16, DMAX = 256;

// q bf16 [B*L, ldq] (head h at cols h*d), kv bf16 [B*T, ldkv] (K at h*d, V at P + h*d)
__global__ __launch_bounds__(NT) void align_fwd_kernel(const bf16* q, int64_t ldq, const bf16* kv, int64_t ldkv,
                                                     const int32_t* kmask, int L, int T, int P, int nh, float scale,
                                                     float drop_p, uint64_t seed, float* probs, bf16* out,
                                                     int64_t ldo) {
  extern __shared__ float ss[];  // QB * T
  __shared__ float sq[QB][DMAX];
  const int l0 = blockIdx.x * QB, h = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int d = P / nh;
  const int nq = min(QB, L - l0);
  for (int i = tid; i < QB * d; i += NT) {
    const int qi = i / d, c = i % d;
    sq[qi][c] = qi < nq ? (float)q[(int64_t)(b * L + l0 + qi) * ldq + h * d + c] * scale : 0.f;
  }
  __syncthreads();
  for (int t = tid; t < T; t += NT) {
    const bf16* kr = kv + (int64_t)(b * T + t) * ldkv + h * d;
    float acc[QB];
#pragma unroll
    for (int qi = 0; qi < QB; ++qi) acc[qi] = 0.f;
    for (int c = 0; c < d; c += 8) {
      const bf16x8 kk = *reinterpret_cast<const bf16x8*>(kr + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float kf = (float)kk[e];
#pragma unroll
        for (int qi = 0; qi < QB; ++qi) acc[qi] += kf * sq[qi][c + e];
      }
    }
    const bool valid = kmask == nullptr || kmask[b * T + t] != 0;
#pragma unroll
    for (int qi = 0; qi < QB; ++qi) ss[qi * T + t] = valid ? acc[qi] : -INFINITY;
  }
  __syncthreads();
  const uint32_t thresh = (uint32_t)(drop_p * 4294967296.0);
  const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  for (int qi = w; qi < nq; qi += NT / 64) {
    float* row = ss + qi * T;
    float mx = -INFINITY;
    for (int t = lane; t < T; t += 64) mx = fmaxf(mx, row[t]);
    mx = wave_max(mx);
    float sum = 0.f;
    for (int t = lane; t < T; t += 64) { const float e = __expf(row[t] - mx); row[t] = e; sum += e; }
    sum = wave_sum(sum);
    const float inv = 1.f / sum;
    const int64_t prow = (((int64_t)b * nh + h) * L + l0 + qi) * T;
    for (int t = lane; t < T; t += 64) {
      float p = row[t] * inv;
      probs[prow + t] = p;
      if (drop_p > 0.f) p *= drop_scale(seed, (uint64_t)(prow + t), thresh, inv_keep);
      row[t] = p;
    }
  }
  __syncthreads();
  for (int i = tid; i < nq * d; i += NT) {
    const int qi = i / d, c = i % d;
    const float* pr = ss + qi * T;
    const bf16* vc = kv + (int64_t)(b * T) * ldkv + P + h * d + c;
    float acc = 0.f;
    for (int t = 0; t < T; ++t) acc += pr[t] * (float)vc[(int64_t)t * ldkv];
    out[(int64_t)(b * L + l0 + qi) * ldo + h * d + c] = (bf16)acc;
  }
}

// dS (scaled by `scale`) -> dsbuf [B,nh,L,T]; dq bf16 [B*L, lddq]
__global__ __launch_bounds__(NT) void align_bwd_q_kernel(const bf16* q, int64_t ldq, const bf16* kv, int64_t ldkv,
                                                       const float* probs, const bf16* dout, int64_t lddo, int L,
                                                       int T, int P, int nh, float scale, float drop_p,
                                                       uint64_t seed, float* dsbuf, bf16* dq, int64_t lddq) {
  extern __shared__ float ss[];  // QB * T
  __shared__ float sdo[QB][DMAX];
  const int l0 = blockIdx.x * QB, h = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int d = P / nh;
  const int nq = min(QB, L - l0);
  for (int i = tid; i < QB * d; i += NT) {
    const int qi = i / d, c = i % d;
    sdo[qi][c] = qi < nq ? (float)dout[(int64_t)(b * L + l0 + qi) * lddo + h * d + c] : 0.f;
  }
  __syncthreads();
  const uint32_t thresh = (uint32_t)(drop_p * 4294967296.0);
  const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  for (int t = tid; t < T; t += NT) {
    const bf16* vr = kv + (int64_t)(b * T + t) * ldkv + P + h * d;
    float acc[QB];
#pragma unroll
    for (int qi = 0; qi < QB; ++qi) acc[qi] = 0.f;
    for (int c = 0; c < d; c += 8) {
      const bf16x8 vv = *reinterpret_cast<const bf16x8*>(vr + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float vf = (float)vv[e];
#pragma unroll
        for (int qi = 0; qi < QB; ++qi) acc[qi] += vf * sdo[qi][c + e];
      }
    }
#pragma unroll
    for (int qi = 0; qi < QB; ++qi) {
      float dp = acc[qi];
      if (drop_p > 0.f && qi < nq)
        dp *= drop_scale(seed, (uint64_t)((((int64_t)b * nh + h) * L + l0 + qi) * T + t), thresh, inv_keep);
      ss[qi * T + t] = dp;
    }
  }
  __syncthreads();
  for (int qi = w; qi < nq; qi += NT / 64) {
    const int64_t prow = (((int64_t)b * nh + h) * L + l0 + qi) * T;
    float* row = ss + qi * T;
    float acc = 0.f;
    for (int t = lane; t < T; t += 64) acc += probs[prow + t] * row[t];
    acc = wave_sum(acc);
    for (int t = lane; t < T; t += 64) {
      const float ds = probs[prow + t] * (row[t] - acc) * scale;
      row[t] = ds;
      dsbuf[prow + t] = ds;
    }
  }
  __syncthreads();
  for (int i = tid; i < nq * d; i += NT) {
    const int qi = i / d, c = i % d;
    const float* dr = ss + qi * T;
    const bf16* kc = kv + (int64_t)(b * T) * ldkv + h * d + c;
    float acc = 0.f;
    for (int t = 0; t < T; ++t) acc += dr[t] * (float)kc[(int64_t)t * ldkv];
    dq[(int64_t)(b * L + l0 + qi) * lddq + h * d + c] = (bf16)acc;
  }
}

// dk[t] = Σ_l ds[l][t] q[l] ; dv[t] = Σ_l p'[l][t] dO[l]  -> dkv fp32 [B*T, lddkv] (K at h*d, V at P+h*d)
__global__ __launch_bounds__(NT) void align_bwd_kv_kernel(const bf16* q, int64_t ldq, const float* probs,
                                                        const float* dsbuf, const bf16* dout, int64_t lddo, int L,
                                                        int T, int P, int nh, float drop_p, uint64_t seed,
                                                        float* dkv, int64_t lddkv) {
  __shared__ float sds[64][KB], sp[64][KB];
  const int t0 = blockIdx.x * KB, h = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x;
  const int d = P / nh;
  const int nt = min(KB, T - t0);
  const uint32_t thresh = (uint32_t)(drop_p * 4294967296.0);
  const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  // each thread owns (t, c) pairs: KB x d outputs for dk and dv
  float ak[12], av[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) { ak[i] = 0.f; av[i] = 0.f; }
  for (int lc = 0; lc < L; lc += 64) {
    const int nl = min(64, L - lc);
    __syncthreads();
    for (int i = tid; i < 64 * KB; i += NT) {
      const int li = i / KB, ti = i % KB;
      float dsv = 0.f, pv = 0.f;
      if (li < nl && ti < nt) {
        const int64_t idx = (((int64_t)b * nh + h) * L + lc + li) * T + t0 + ti;
        dsv = dsbuf[idx];
        pv = probs[idx];
        if (drop_p > 0.f) pv *= drop_scale(seed, (uint64_t)idx, thresh, inv_keep);
      }
      sds[li][ti] = dsv;
      sp[li][ti] = pv;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const int o = tid + NT * i;
      if (o >= KB * d) break;
      const int ti = o / d, c = o % d;
      float s1 = ak[i], s2 = av[i];
      for (int li = 0; li < nl; ++li) {
        const int64_t row = (int64_t)(b * L + lc + li);
        s1 += sds[li][ti] * (float)q[row * ldq + h * d + c];
        s2 += sp[li][ti] * (float)dout[row * lddo + h * d + c];
      }
      ak[i] = s1;
      av[i] = s2;
    }
  }
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int o = tid + NT * i;
    if (o >= KB * d) break;
    const int ti = o / d, c = o % d;
    if (ti < nt) {
      float* r = dkv + (int64_t)(b * T + t0 + ti) * lddkv;
      r[h * d + c] = ak[i];
      r[P + h * d + c] = av[i];
    }
  }
}

// out[m][k] = a[m] * w[k] * act'(z[m][k]); dw[k] += Σ_m a[m] z[m][k]; db += Σ_m a[m]
__global__ __launch_bounds__(NT) void rank1_bwd_kernel(const float* a, const float* w, const bf16* z, int M, int K,
                                                     int act, bf16* out, float* dw, float* db) {
  const int k = blockIdx.x * NT + threadIdx.x;
  if (k >= K) return;
  float accw = 0.f, accb = 0.f;
  for (int m = 0; m < M; ++m) {
    const float am = a[m];
    const float zv = (float)z[(int64_t)m * K + k];
    float g = 1.f;
    if (act == STE_ACT_RELU_BWD) g = zv > 0.f ? 1.f : 0.f;
    else if (act == STE_ACT_TANH_BWD_OUT) g = 1.f - zv * zv;
    out[(int64_t)m * K + k] = (bf16)(am * w[k] * g);
    accw += am * zv;
    accb += am;
  }
  if (dw) atomicAdd(dw + k, accw);
  if (db && k == 0) atomicAdd(db, accb);
}

}  // namespace

extern "C" int ste_align_attn_fwd(const void* q, int64_t ldq, const void* kv, int64_t ldkv, const int32_t* kmask,
                                  int B, int L, int T, int P, int nh, float drop_p, uint64_t seed, float* probs,
                                  void* out, int64_t ldo, void* stream) {
  const int d = P / nh;
  if (B <= 0 || L <= 0 || T <= 0 || P % nh || d > DMAX || d % 8 || QB * T * 4 > 64 * 1024) return STE_ERR_SHAPE;
  dim3 grid((L + QB - 1) / QB, nh, B);
  hipLaunchKernelGGL(align_fwd_kernel, grid, dim3(NT), QB * T * sizeof(float), (hipStream_t)stream, (const bf16*)q,
                     ldq, (const bf16*)kv, ldkv, kmask, L, T, P, nh, 1.0f / sqrtf((float)d), drop_p, seed, probs,
                     (bf16*)out, ldo);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_align_attn_bwd(const void* q, int64_t ldq, const void* kv, int64_t ldkv, const float* probs,
                                  const void* dout, int64_t lddo, int B, int L, int T, int P, int nh, float drop_p,
                                  uint64_t seed, float* dsbuf, void* dq, int64_t lddq, float* dkv, int64_t lddkv,
                                  void* stream) {
  const int d = P / nh;
  if (B <= 0 || L <= 0 || T <= 0 || P % nh || d > DMAX || d % 8 || QB * T * 4 > 64 * 1024 || KB * d > 12 * NT)
    return STE_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((L + QB - 1) / QB, nh, B);
  hipLaunchKernelGGL(align_bwd_q_kernel, grid, dim3(NT), QB * T * sizeof(float), s, (const bf16*)q, ldq,
                     (const bf16*)kv, ldkv, probs, (const bf16*)dout, lddo, L, T, P, nh, 1.0f / sqrtf((float)d),
                     drop_p, seed, dsbuf, (bf16*)dq, lddq);
  STE_CHECK_LAUNCH();
  dim3 grid2((T + KB - 1) / KB, nh, B);
  hipLaunchKernelGGL(align_bwd_kv_kernel, grid2, dim3(NT), 0, s, (const bf16*)q, ldq, probs, dsbuf,
                     (const bf16*)dout, lddo, L, T, P, nh, drop_p, seed, dkv, lddkv);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_rank1_bwd(const float* a, const float* w, const void* z, int M, int K, int act, void* out,
                             float* dw, float* db, void* stream) {
  if (M <= 0 || K <= 0) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(rank1_bwd_kernel, dim3((K + NT - 1) / NT), dim3(NT), 0, (hipStream_t)stream, a, w,
                     (const bf16*)z, M, K, act, (bf16*)out, dw, db);
  STE_CHECK_LAUNCH();
  return 0;
}

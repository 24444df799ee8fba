// fp32 self-attention forward of the text encoder (XLM-R SDPA semantics,
// tf:models/xlm_roberta/modeling_xlm_roberta.py:186-250): softmax(Q·Kᵀ·scale + key mask)·V with
// probs dropout, on fp32 q / k / v (the precise-forward QKV GEMM's fp32 output).
//
// Why fp32 here: the loss gradient differences the positive and the corrupted transcript
// (80 % shared tokens), so bf16 rounding of the text encoder's forward activations reappeared
// as 1-2.5 % errors in every gradient downstream of the transcript embeddings.  The
// text side is 3.4 % of the step's FLOPs and runs on the side stream, so its forward is
// computed to fp32 accuracy (split-bf16 GEMMs + this kernel); its backward keeps the bf16
// kernels, fed by the bf16 copies (q/k/v, O + O_lo) and the LSE this kernel saves in the same
// convention as attention.hip (natural log, masked keys at the finfo.min score, dropout index
// ((b·H + h)·T + q)·T + key), so ste_attention_bwd runs on them unchanged.
//
// One block per (sample, head, 64-query tile), 4 waves x 16 query rows.  Keys in chunks of 64
// staged in LDS (fp32 K at a 65-float row stride: lane j reads row j, conflict-free), one key
// per lane; the online softmax's running max / sum are wave-uniform per row; O[row][c] lives
// on lane c.  VALU fp32 throughout (T is short: 16-128 tokens).
#include "common.h"
#include "../../include/ste.h"

namespace {

constexpr int HD = 64, QT = 64, KC = 64, NT = 256, KLD = HD + 1;
constexpr float NEG_MASK = -3.4028234663852886e38f;   // finfo(float32).min, as attention.hip

STE_DEV float key_flag32(const int32_t* mask, int bT, int key, int T) {
  if (key >= T) return -1.f;
  return (mask == nullptr || mask[bT + key] != 0) ? 1.f : 0.f;
}

template <bool DROP>
__global__ __launch_bounds__(NT) void attn_f32_fwd_kernel(ste_attn_args a, float* o32, int64_t ldo32) {
  __shared__ float sK[KC * KLD];
  __shared__ float sV[KC * HD];
  __shared__ float sQ[QT * HD];
  __shared__ float sP[NT / 64][KC];
  __shared__ float sF[KC];
  const int T = a.T, H = a.H;
  const int ntile = (T + QT - 1) / QT;
  const int tile = blockIdx.x % ntile, bh = blockIdx.x / ntile, h = bh % H, b = bh / H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int bT = b * T, q0 = tile * QT;
  const float* Q = (const float*)a.q + h * HD;
  const float* K = (const float*)a.k + h * HD;
  const float* V = (const float*)a.v + h * HD;
  for (int i = tid; i < QT * HD / 4; i += NT) {
    const int r = i >> 4, c = (i & 15) * 4;
    const f32x4 v = q0 + r < T ? *reinterpret_cast<const f32x4*>(Q + (int64_t)(bT + q0 + r) * a.ldq + c)
                               : f32x4{0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<f32x4*>(sQ + r * HD + c) = v;
  }
  const uint32_t thresh = (uint32_t)(a.drop_p * 4294967296.0);
  const float inv_keep = DROP ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  float m[16], l[16], o[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    m[r] = -INFINITY;
    l[r] = 0.f;
    o[r] = 0.f;
  }
  for (int k0 = 0; k0 < T; k0 += KC) {
    __syncthreads();  // the previous chunk is consumed (first pass: sQ is staged)
    for (int i = tid; i < KC * HD / 4; i += NT) {
      const int r = i >> 4, c = (i & 15) * 4, key = k0 + r;
      f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
      if (key < T) {
        kv = *reinterpret_cast<const f32x4*>(K + (int64_t)(bT + key) * a.ldk + c);
        vv = *reinterpret_cast<const f32x4*>(V + (int64_t)(bT + key) * a.ldv + c);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) sK[r * KLD + c + e] = kv[e];
      *reinterpret_cast<f32x4*>(sV + r * HD + c) = vv;
    }
    if (tid < KC) sF[tid] = key_flag32(a.key_mask, bT, k0 + tid, T);
    __syncthreads();
    const int nk = min(KC, T - k0);
    const float f = sF[lane];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int q = q0 + w * 16 + r;
      const float* qrow = sQ + (w * 16 + r) * HD;
      float s = 0.f;
#pragma unroll 16
      for (int d = 0; d < HD; ++d) s = fmaf(qrow[d], sK[lane * KLD + d], s);
      float v = s * a.scale;
      v = f > 0.5f ? v : (f < -0.5f ? -INFINITY : NEG_MASK);
      const float mn = fmaxf(m[r], wave_max(v));
      const float alpha = mn == -INFINITY ? 1.f : __expf(m[r] - mn);
      float p = mn == -INFINITY ? 0.f : __expf(v - mn);
      l[r] = l[r] * alpha + wave_sum(p);
      m[r] = mn;
      if (DROP) p *= drop_scale(a.seed, ((uint64_t)(b * H + h) * T + q) * (uint64_t)T + (uint64_t)(k0 + lane), thresh,
                                inv_keep);
      sP[w][lane] = p;
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      float acc = o[r] * alpha;
      for (int j = 0; j < nk; ++j) acc = fmaf(sP[w][j], sV[j * HD + lane], acc);
      o[r] = acc;
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int q = q0 + w * 16 + r;
    if (q >= T) continue;
    const float ov = o[r] / l[r];
    const int64_t row = bT + q;
    if (o32) o32[row * ldo32 + h * HD + lane] = ov;
    if (a.o) {
      const bf16 hi = (bf16)ov;
      ((bf16*)a.o)[row * a.ldo + h * HD + lane] = hi;
      if (a.o_lo) ((bf16*)a.o_lo)[row * a.ldolo + h * HD + lane] = (bf16)(ov - (float)hi);
    }
    // all keys masked (uniform weights): -inf, the convention the backward kernels read as p = 1/T
    if (lane == 0) a.lse[(int64_t)(b * H + h) * T + q] = m[r] == NEG_MASK ? -INFINITY : m[r] + logf(l[r]);
  }
}

}  // namespace

extern "C" int ste_attention_fwd_f32(const ste_attn_args* args, float* o32, int64_t ldo32, void* stream) {
  if (!args || (!o32 && !args->o)) return STE_ERR_ARG;
  const ste_attn_args& a = *args;
  if (!a.q || !a.k || !a.v || !a.lse || a.rel_E) return STE_ERR_ARG;
  if (a.B <= 0 || a.T <= 0 || a.H <= 0) return STE_ERR_SHAPE;
  if ((a.ldq & 3) || (a.ldk & 3) || (a.ldv & 3) || (o32 && ldo32 < (int64_t)a.H * 64) ||
      (((uintptr_t)a.q | (uintptr_t)a.k | (uintptr_t)a.v) & 15))
    return STE_ERR_SHAPE;
  const int ntile = (a.T + QT - 1) / QT;
  const dim3 grid((unsigned)((int64_t)a.B * a.H * ntile));
  if (a.drop_p > 0.f)
    hipLaunchKernelGGL(attn_f32_fwd_kernel<true>, grid, dim3(NT), 0, (hipStream_t)stream, a, o32, ldo32);
  else
    hipLaunchKernelGGL(attn_f32_fwd_kernel<false>, grid, dim3(NT), 0, (hipStream_t)stream, a, o32, ldo32);
  STE_CHECK_LAUNCH();
  return 0;
}

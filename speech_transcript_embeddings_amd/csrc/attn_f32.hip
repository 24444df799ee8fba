// fp32 self-attention forward of the text encoder (XLM-R SDPA semantics,
// tf:models/xlm_roberta/modeling_xlm_roberta.py:186-250): softmax(Q·Kᵀ·scale + key mask)·V with
// probs dropout, on fp32 q / k / v (the precise-forward QKV GEMM's fp32 output).
//
// Why fp32 here: the loss gradient differences the positive and the corrupted transcript
// (80 % shared tokens), so bf16 rounding of the text encoder's forward activations reappeared
// as 1-2.5 % errors in every gradient downstream of the transcript embeddings.  The
// text side is 3.4 % of the step's FLOPs and runs on the side stream, so its forward is
// computed to fp32 accuracy (split-bf16 GEMMs + this kernel), and so is its backward
// (attn_f32_bwd_kernel below: the loss-derived gradients of the clean and corrupted transcripts
// cancel in every text weight and bias, tests/precision_probe_text.py).  The LSE is saved in the
// convention of attention.hip (natural log, masked keys at the finfo.min score, dropout index
// ((b·H + h)·T + q)·T + key), so ste_attention_bwd also runs on bf16 copies of its inputs.
//
// One block per (sample, head, 64-query tile), 4 waves x 16 query rows, keys in chunks of 64.
// Register-blocked VALU fp32 with the softmax row lane-local: lane (r, g) = (l & 15, l >> 4)
// owns query row r and the keys 4kk + g (kk < 16) of a chunk, so a
// row's max / sum is an in-lane reduction plus two cross-lane steps (not six); K rows are read
// from LDS as b128 at a 68-float stride (the 4 simultaneous rows 4kk..4kk+3 hit disjoint bank
// groups; so do the 16 query rows).  P goes to LDS row-major and lane (r, g) accumulates O[r][16g..16g+15] from
// broadcast V reads.  1,024 + 1,024 FMAs per lane per 64-key chunk.
#include "common.h"
#include "../../include/ste.h"

namespace {

constexpr int HD = 64, QT = 64, KC = 64, NT = 256;
constexpr float NEG_MASK = -3.4028234663852886e38f;   // finfo(float32).min, as attention.hip

STE_DEV float key_flag32(const int32_t* mask, int bT, int key, int T) {
  if (key >= T) return -1.f;
  return (mask == nullptr || mask[bT + key] != 0) ? 1.f : 0.f;
}

constexpr int KLD = HD + 4;   // K / V row stride in LDS (floats)
constexpr int PLD = KC + 1;   // P row stride

template <bool DROP>
__global__ __launch_bounds__(NT) void attn_f32_fwd_kernel(ste_attn_args a, float* o32, int64_t ldo32) {
  __shared__ __attribute__((aligned(16))) float sQ[QT * KLD];
  __shared__ __attribute__((aligned(16))) float sK[KC * KLD];
  __shared__ __attribute__((aligned(16))) float sV[KC * KLD];
  __shared__ float sP[NT / 64][16 * PLD];
  __shared__ float sF[KC];
  const int T = a.T, H = a.H;
  const int ntile = (T + QT - 1) / QT;
  const int tile = blockIdx.x % ntile, bh = blockIdx.x / ntile, h = bh % H, b = bh / H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 15, g = lane >> 4;
  const int bT = b * T, q0 = tile * QT, q = q0 + w * 16 + r;
  const float* K = (const float*)a.k + h * HD;
  const float* V = (const float*)a.v + h * HD;
  for (int i = tid; i < QT * HD / 4; i += NT) {
    const int qr = i >> 4, c = (i & 15) * 4;
    *reinterpret_cast<f32x4*>(sQ + qr * KLD + c) =
        q0 + qr < T ? *reinterpret_cast<const f32x4*>((const float*)a.q + h * HD + (int64_t)(bT + q0 + qr) * a.ldq + c)
                    : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const float* qrow = sQ + (w * 16 + r) * KLD;
  const uint32_t thresh = (uint32_t)(a.drop_p * 4294967296.0);
  const float inv_keep = DROP ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  const uint64_t drow = ((uint64_t)(b * H + h) * T + q) * (uint64_t)T;
  float m = -INFINITY, l = 0.f;
  f32x4 o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float* sp = sP[w] + r * PLD;
  for (int k0 = 0; k0 < T; k0 += KC) {
    __syncthreads();   // the previous chunk is consumed
    for (int i = tid; i < KC * HD / 4; i += NT) {
      const int kr = i >> 4, c = (i & 15) * 4, key = k0 + kr;
      f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
      if (key < T) {
        kv = *reinterpret_cast<const f32x4*>(K + (int64_t)(bT + key) * a.ldk + c);
        vv = *reinterpret_cast<const f32x4*>(V + (int64_t)(bT + key) * a.ldv + c);
      }
      *reinterpret_cast<f32x4*>(sK + kr * KLD + c) = kv;
      *reinterpret_cast<f32x4*>(sV + kr * KLD + c) = vv;
    }
    if (tid < KC) sF[tid] = key_flag32(a.key_mask, bT, k0 + tid, T);
    __syncthreads();
    float s[16];
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) s[kk] = 0.f;
#pragma unroll 2
    for (int d = 0; d < HD / 4; ++d) {
      const f32x4 qv = *reinterpret_cast<const f32x4*>(qrow + 4 * d);   // 4 lanes per row: broadcast
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        const f32x4 kv = *reinterpret_cast<const f32x4*>(sK + (4 * kk + g) * KLD + 4 * d);
        s[kk] = fmaf(qv[0], kv[0], fmaf(qv[1], kv[1], fmaf(qv[2], kv[2], fmaf(qv[3], kv[3], s[kk]))));
      }
    }
    float cm = -INFINITY;
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const float f = sF[4 * kk + g];
      float v = s[kk] * a.scale;
      v = f > 0.5f ? v : (f < -0.5f ? -INFINITY : NEG_MASK);
      s[kk] = v;
      cm = fmaxf(cm, v);
    }
    cm = fmaxf(cm, __shfl_xor(cm, 16, 64));
    cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
    const float mn = fmaxf(m, cm);
    const float alpha = mn == -INFINITY ? 1.f : __expf(m - mn);
    float ps = 0.f;
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      float p = mn == -INFINITY ? 0.f : __expf(s[kk] - mn);
      ps += p;
      if (DROP) p *= drop_scale(a.seed, drow + (uint64_t)(k0 + 4 * kk + g), thresh, inv_keep);
      sp[4 * kk + g] = p;
    }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    l = l * alpha + ps;
    m = mn;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] *= alpha;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    const int nk = min(KC, T - k0);
    for (int j = 0; j < nk; ++j) {
      const float p = sp[j];
      const float* vr = sV + j * KLD + 16 * g;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] += p * *reinterpret_cast<const f32x4*>(vr + 4 * i);
    }
  }
  if (q < T) {
    const bool zrow = a.zero_masked_rows && m == NEG_MASK;   // SDPA: a fully masked row -> 0
    const float inv_l = zrow ? 0.f : 1.0f / l;
    const int64_t row = bT + q;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x4 ov = o[i] * inv_l;
      const int col = h * HD + 16 * g + 4 * i;
      if (o32) *reinterpret_cast<f32x4*>(o32 + row * ldo32 + col) = ov;
      if (a.o) {
        if (a.o_lo) store_bf16x4_split((bf16*)a.o + row * a.ldo + col, (bf16*)a.o_lo + row * a.ldolo + col, ov);
        else store_bf16x4((bf16*)a.o + row * a.ldo + col, ov);
      }
    }
    // all keys masked: -inf (uniform weights, the backward reads p = 1/T) or, under SDPA
    // semantics, +inf (zero weights: p = exp(v - inf) = 0 in the backward)
    if (g == 0) a.lse[(int64_t)(b * H + h) * T + q] = m == NEG_MASK ? (zrow ? INFINITY : -INFINITY) : m + logf(l);
  }
}


// ------------------------------------------------------------------------------- backward
// fp32 backward of the kernel above: dV = Pdᵀ·dO, dS = P ∘ (m·dO·Vᵀ − δ), dQ = scale·dS·K,
// dK = scale·dSᵀ·Q, with P recomputed from fp32 q / k and the saved LSE, m the dropout scale of
// the forward's mask (the same counter-based hash and index), Pd = P·m, and δ = dO·O from the
// forward's O hi + lo halves (~16 mantissa bits).  One block per (sample, head) walks the key
// chunks of 64 (dK, dV of the chunk in registers, written once) and, inside, the query tiles of 64
// (dQ of a tile summed over the chunks in order by the same threads: deterministic, no atomics).
// 1,024 threads (4 waves per SIMD: the images take 104 KB, one block per CU, and a 64 x 64 tile is
// too little work per (sample, head) for fewer waves to hide the LDS latency — 256 threads ran at
// 730 us per c2 text layer).  Thread (r, c) = (t >> 4, t & 15): the scores of query row r with keys
// c + 16j; row / key r x columns 4c..4c+3 of the dQ / dK / dV tiles.
constexpr int BWD_NT = 1024;
constexpr int BLD = HD + 4;   // fp32 row stride of the Q / dO / K / V images
constexpr int SLD = KC + 1;   // row stride of the Pd / dS images

template <bool DROP>
__global__ __launch_bounds__(BWD_NT) void attn_f32_bwd_kernel(ste_attn_args a) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  float* sQ = smf;                       // [64][BLD]
  float* sD = sQ + QT * BLD;             // dO
  float* sK = sD + QT * BLD;
  float* sV = sK + KC * BLD;
  float* sP = sV + KC * BLD;             // Pd [q][key]
  float* sS = sP + QT * SLD;             // dS [q][key]
  float* sL = sS + QT * SLD;             // lse[64]
  float* sDl = sL + QT;                  // delta[64]
  float* sF = sDl + QT;                  // key flags[64]
  const int T = a.T, H = a.H;
  const int bh = blockIdx.x, h = bh % H, b = bh / H, bT = b * T;
  const int tid = threadIdx.x, r = tid >> 4, c = tid & 15;
  const float* Qg = (const float*)a.q + h * HD;
  const float* Kg = (const float*)a.k + h * HD;
  const float* Vg = (const float*)a.v + h * HD;
  const float* dOg = (const float*)a.dout + h * HD;
  const bf16* Og = (const bf16*)a.o + h * HD;
  const bf16* Olg = (const bf16*)a.o_lo + h * HD;
  float* dQg = (float*)a.dq + h * HD;
  float* dKg = (float*)a.dk + h * HD;
  float* dVg = (float*)a.dv + h * HD;
  const uint32_t thresh = (uint32_t)(a.drop_p * 4294967296.0);
  const float inv_keep = DROP ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  const float inv_T = 1.0f / (float)T;
  const int nkc = (T + KC - 1) / KC, nqt = (T + QT - 1) / QT;
  // row r0 + r of a [B*T, *] fp32 operand (head h), columns 4c..4c+3, into an image; rows >= T are 0
  auto stage = [&](float* img, const float* src, int64_t ld, int r0) {
    *reinterpret_cast<f32x4*>(img + r * BLD + 4 * c) =
        r0 + r < T ? *reinterpret_cast<const f32x4*>(src + (int64_t)(bT + r0 + r) * ld + 4 * c) : f32x4{0.f, 0.f, 0.f, 0.f};
  };
  for (int kc = 0; kc < nkc; ++kc) {
    const int k0 = kc * KC;
    __syncthreads();   // the previous chunk's images are consumed
    stage(sK, Kg, a.ldk, k0);
    stage(sV, Vg, a.ldv, k0);
    if (tid < KC) sF[tid] = key_flag32(a.key_mask, bT, k0 + tid, T);
    f32x4 dk = {0.f, 0.f, 0.f, 0.f}, dv = {0.f, 0.f, 0.f, 0.f};
    for (int qt = 0; qt < nqt; ++qt) {
      const int q0 = qt * QT, q = q0 + r;
      __syncthreads();   // the previous tile's Q / dO / Pd / dS images are consumed
      stage(sQ, Qg, a.ldq, q0);
      stage(sD, dOg, a.lddo, q0);
      {  // delta = dO·(O_hi + O_lo) of row r: the row's 16 lanes, 4 columns each
        float part = 0.f;
        if (q < T) {
          const int64_t row = bT + q;
          const f32x4 dov = *reinterpret_cast<const f32x4*>(dOg + row * a.lddo + 4 * c);
          const f32x4 oh = load_bf16x4(Og + row * a.ldo + 4 * c);
          const f32x4 ol = load_bf16x4(Olg + row * a.ldolo + 4 * c);
#pragma unroll
          for (int e = 0; e < 4; ++e) part = fmaf(dov[e], oh[e] + ol[e], part);
        }
#pragma unroll
        for (int o = 8; o >= 1; o >>= 1) part += __shfl_xor(part, o, 16);
        if (c == 0) {
          sDl[r] = part;
          sL[r] = q < T ? a.lse[(int64_t)bh * T + q] : INFINITY;   // rows past T: p = 0
        }
      }
      __syncthreads();
      // scores and dP of row r with keys c + 16j
      float sc[4] = {0.f, 0.f, 0.f, 0.f}, dp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
      for (int d = 0; d < HD; d += 4) {
        const f32x4 qv = *reinterpret_cast<const f32x4*>(sQ + r * BLD + d);
        const f32x4 dov = *reinterpret_cast<const f32x4*>(sD + r * BLD + d);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x4 kv = *reinterpret_cast<const f32x4*>(sK + (c + 16 * j) * BLD + d);
          const f32x4 vv = *reinterpret_cast<const f32x4*>(sV + (c + 16 * j) * BLD + d);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            sc[j] = fmaf(qv[e], kv[e], sc[j]);
            dp[j] = fmaf(dov[e], vv[e], dp[j]);
          }
        }
      }
      {
        const float lse = sL[r], dl = sDl[r];
        const uint64_t drow = ((uint64_t)bh * T + (uint64_t)(q < T ? q : 0)) * (uint64_t)T;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int kl = c + 16 * j, key = k0 + kl;
          const float f = sF[kl];
          float p;
          if (lse == INFINITY || f < -0.5f) p = 0.f;                 // zero-weight row / key past T
          else if (lse == -INFINITY) p = inv_T;                       // uniform row (every key masked)
          else p = __expf((f > 0.5f ? sc[j] * a.scale : NEG_MASK) - lse);
          const float m = DROP ? drop_scale(a.seed, drow + (uint64_t)key, thresh, inv_keep) : 1.0f;
          sP[r * SLD + kl] = p * m;
          sS[r * SLD + kl] = p * (m * dp[j] - dl);
        }
      }
      __syncthreads();
      // dV += Pdᵀ·dO, dK += dSᵀ·Q for key r, columns 4c..; dQ tile row r = dS·K
      const int nq = min(QT, T - q0), nk = min(KC, T - k0);
      for (int i = 0; i < nq; ++i) {
        dv += sP[i * SLD + r] * *reinterpret_cast<const f32x4*>(sD + i * BLD + 4 * c);
        dk += sS[i * SLD + r] * *reinterpret_cast<const f32x4*>(sQ + i * BLD + 4 * c);
      }
      f32x4 dq = {0.f, 0.f, 0.f, 0.f};
      for (int kl = 0; kl < nk; ++kl) dq += sS[r * SLD + kl] * *reinterpret_cast<const f32x4*>(sK + kl * BLD + 4 * c);
      if (q < T) {
        float* dst = dQg + (int64_t)(bT + q) * a.lddq + 4 * c;
        f32x4 v = dq * a.scale;
        if (kc > 0) v += *reinterpret_cast<const f32x4*>(dst);   // this thread's own earlier chunk
        *reinterpret_cast<f32x4*>(dst) = v;
      }
    }
    const int key = k0 + r;
    if (key < T) {
      *reinterpret_cast<f32x4*>(dKg + (int64_t)(bT + key) * a.lddk + 4 * c) = dk * a.scale;
      *reinterpret_cast<f32x4*>(dVg + (int64_t)(bT + key) * a.lddv + 4 * c) = dv;
    }
  }
}
constexpr int BWD_F32_LDS = (4 * 64 * BLD + 2 * 64 * SLD + 3 * 64) * 4;

}  // namespace

extern "C" int ste_attention_fwd_f32(const ste_attn_args* args, float* o32, int64_t ldo32, void* stream) {
  if (!args || (!o32 && !args->o)) return STE_ERR_ARG;
  const ste_attn_args& a = *args;
  if (!a.q || !a.k || !a.v || !a.lse || a.rel_E) return STE_ERR_ARG;
  if (a.B <= 0 || a.T <= 0 || a.H <= 0) return STE_ERR_SHAPE;
  if ((a.ldq & 3) || (a.ldk & 3) || (a.ldv & 3) || (o32 && (ldo32 < (int64_t)a.H * 64 || (ldo32 & 3))) ||
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

extern "C" int ste_attention_bwd_f32(const ste_attn_args* args, void* stream) {
  if (!args) return STE_ERR_ARG;
  const ste_attn_args& a = *args;
  if (!a.q || !a.k || !a.v || !a.lse || !a.dout || !a.o || !a.o_lo || !a.dq || !a.dk || !a.dv || a.rel_E)
    return STE_ERR_ARG;
  if (a.B <= 0 || a.T <= 0 || a.H <= 0) return STE_ERR_SHAPE;
  if ((a.ldq & 3) || (a.ldk & 3) || (a.ldv & 3) || (a.lddo & 3) || (a.lddq & 3) || (a.lddk & 3) || (a.lddv & 3) ||
      (a.ldo & 3) || (a.ldolo & 3) ||
      (((uintptr_t)a.q | (uintptr_t)a.k | (uintptr_t)a.v | (uintptr_t)a.dout | (uintptr_t)a.dq | (uintptr_t)a.dk |
        (uintptr_t)a.dv) & 15) ||
      (((uintptr_t)a.o | (uintptr_t)a.o_lo) & 7))
    return STE_ERR_SHAPE;
  if (a.drop_p < 0.f || a.drop_p >= 1.f) return STE_ERR_ARG;
  const dim3 grid((unsigned)((int64_t)a.B * a.H));
  if (a.drop_p > 0.f)
    hipLaunchKernelGGL(attn_f32_bwd_kernel<true>, grid, dim3(BWD_NT), BWD_F32_LDS, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(attn_f32_bwd_kernel<false>, grid, dim3(BWD_NT), BWD_F32_LDS, (hipStream_t)stream, a);
  STE_CHECK_LAUNCH();
  return 0;
}

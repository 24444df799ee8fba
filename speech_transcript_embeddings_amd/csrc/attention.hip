// Fused multi-head attention (head_dim 64) with optional relative-key bias, key-padding
// mask and probability dropout — forward + backward.  Scores / probabilities never
// touch HBM.
//
// Audio (w2v-bert relative_key, tf:models/wav2vec2_bert/modeling_wav2vec2_bert.py:285-327):
//   s[l,r] = (q_l·k_r + q_l·E[clamp(r-l,-left,right)+left]) / sqrt(64) + mask
// Text (XLM-R SDPA, tf:models/xlm_roberta/modeling_xlm_roberta.py:186-250):
//   s[l,r] = q_l·k_r / sqrt(64) + mask, dropout(p) on the probabilities.
// Masked keys get finfo(float32).min exactly like the reference's additive mask, so a
// fully-masked row degenerates to the same uniform distribution.
//
// The relative term is never expanded to T×T×64: per query row the 73 values
// QE[l,j] = q_l·E[j] are produced by one MFMA pass and gathered by distance; in
// backward the score gradients are binned per distance (G[l,j]) and folded back with
// two more small products (dQ += G·E, dE += Gᵀ·Q).
//
// Layout: every MFMA is v_mfma_f32_16x16x32_bf16, one wave owns 16 query (or key)
// rows, tiles of 64 keys (queries) are staged in XOR-swizzled LDS images that are
// read both row-wise (ds_read_b128) and transposed (ds_read_b64_tr_b16).  The
// "swapped" products (Sᵀ = K·Qᵀ) keep the softmax row on the lane, and accumulator
// tiles feed the next MFMA directly as B operands (no LDS round trip for P or dS).
#include "common.h"
#include "../../include/ste.h"

namespace {

constexpr int HD = 64;
constexpr int TQ = 64;
constexpr int TK = 64;
constexpr int NT = 256;
constexpr int TILE = TK * HD * 2;  // 8 KiB bf16 tile [64][64]
constexpr int NREL = 80;           // padded relative-table width (>= left+right+1 = 73)
constexpr float NEG_MASK = -3.4028234663852886e38f;

STE_DEV int swz(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

STE_DEV void tile_ld(bf16x8 (&r)[2], const bf16* base, int64_t ld, int bT, int row0, int T, int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int c = tid + NT * i, row = c >> 3, ch = c & 7;
    if (row0 + row < T) r[i] = *reinterpret_cast<const bf16x8*>(base + (int64_t)(bT + row0 + row) * ld + ch * 8);
    else r[i] = bf16x8{};
  }
}
STE_DEV void tile_st(char* t, const bf16x8 (&r)[2], int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int c = tid + NT * i;
    *reinterpret_cast<bf16x8*>(t + swz(c >> 3, c & 7)) = r[i];
  }
}
// row-major operand fragment: X[row = rb + (l&15)][k = 32s + 8(l>>4) + j]
STE_DEV bf16x8 frag_kc(const char* t, int rb, int s, int lane) {
  int r = rb + (lane & 15);
  return *reinterpret_cast<const bf16x8*>(t + swz(r, s * 4 + (lane >> 4)));
}
STE_DEV int tr_off(int row, int quad) { return row * 128 + ((((quad >> 1) ^ (row & 7))) << 4) + ((quad & 1) << 3); }
// transposed fragment over rows in "accumulator order": lane l gets X[rows(κ)][cb + (l&15)],
// κ = 8g + e  <->  row 32u + 4g + e (e < 4), 32u + 16 + 4g + (e - 4) (e >= 4).
STE_DEV bf16x8 frag_tr(const char* t, int cb, int u, int lane) {
  int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  int r0 = 32 * u + 4 * g + q;
  int quad = (cb >> 2) + p;
  return join_tr(ds_read_tr16(t + tr_off(r0, quad)), ds_read_tr16(t + tr_off(r0 + 16, quad)));
}
// accumulator pair -> B fragment in the same κ order as frag_tr
STE_DEV bf16x8 pack_acc(f32x4 a, f32x4 b) {
  bf16x8 v;
  v[0] = (bf16)a[0]; v[1] = (bf16)a[1]; v[2] = (bf16)a[2]; v[3] = (bf16)a[3];
  v[4] = (bf16)b[0]; v[5] = (bf16)b[1]; v[6] = (bf16)b[2]; v[7] = (bf16)b[3];
  return v;
}

STE_DEV void stage_E(char* sE, const bf16* E, int nrel, int rows, int tid) {
  for (int c = tid; c < rows * 8; c += NT) {
    int row = c >> 3, ch = c & 7;
    bf16x8 v = bf16x8{};
    if (row < nrel) v = *reinterpret_cast<const bf16x8*>(E + row * HD + ch * 8);
    *reinterpret_cast<bf16x8*>(sE + swz(row, ch)) = v;
  }
}
// per-wave QE table: qe[i*NREL + j] = E[j]·Q[q_i] for the wave's 16 queries (qf = Q as B operand)
STE_DEV void build_qe(float* qe, const char* sE, const bf16x8 (&qf)[2], int lane) {
  const int g = lane >> 4, li = lane & 15;
#pragma unroll
  for (int jt = 0; jt < NREL / 16; ++jt) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) acc = mfma16(frag_kc(sE, jt * 16, s, lane), qf[s], acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) qe[li * NREL + jt * 16 + 4 * g + r] = acc[r];
  }
}

STE_DEV float key_flag(const int32_t* mask, int bT, int key, int T) {
  if (key >= T) return -1.f;
  return (mask == nullptr || mask[bT + key] != 0) ? 1.f : 0.f;
}

// 1-D grid of ceil(T/64) x H x B tiles; the tiles of one (batch, head) share an XCD so
// their K/V (or Q/dO) re-reads hit that XCD's L2 instead of HBM.
STE_DEV void tile_of_block(int T, int H, int& tile, int& h, int& b) {
  const int ntile = (T + 63) / 64;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  tile = id % ntile;
  const int bh = id / ntile;
  h = bh % H;
  b = bh / H;
}

// =========================================================================== forward
template <bool REL, bool DROP>
__global__ __launch_bounds__(NT, 2) void attn_fwd_kernel(ste_attn_args a) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  char* sK = sm;
  char* sV = sm + 2 * TILE;
  char* sE = sm + 4 * TILE;                                  // NREL rows x 128 B
  float* sQE = reinterpret_cast<float*>(sE + NREL * 128);    // 4 x 16 x NREL
  float* sMask = sQE + 4 * 16 * NREL;                         // 2 x 64

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
  int tile, h, b;
  tile_of_block(a.T, a.H, tile, h, b);
  const int T = a.T, H = a.H, bT = b * T;
  const int q0 = tile * TQ + w * 16, myq = q0 + li;
  const bf16* Qb = (const bf16*)a.q + h * HD;
  const bf16* Kb = (const bf16*)a.k + h * HD;
  const bf16* Vb = (const bf16*)a.v + h * HD;
  const int left = a.rel_left, right = a.rel_right, nrel = left + right + 1;

  bf16x8 qf[2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
    qf[s] = myq < T ? *reinterpret_cast<const bf16x8*>(Qb + (int64_t)(bT + myq) * a.ldq + 32 * s + 8 * g) : bf16x8{};

  float* qe = sQE + w * 16 * NREL;
  float qe_lo = 0.f, qe_hi = 0.f;
  if (REL) {
    stage_E(sE, (const bf16*)a.rel_E, nrel, NREL, tid);
    __syncthreads();
    build_qe(qe, sE, qf, lane);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    qe_lo = qe[li * NREL];
    qe_hi = qe[li * NREL + nrel - 1];
  }

  const uint32_t thresh = (uint32_t)(a.drop_p * 4294967296.0);
  const float inv_keep = DROP ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  const uint64_t drow = ((uint64_t)(b * H + h) * T + myq) * (uint64_t)T;

  float m = -INFINITY, l = 0.f;
  f32x4 o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = (T + TK - 1) / TK;
  bf16x8 rk[2], rv[2];
  tile_ld(rk, Kb, a.ldk, bT, 0, T, tid);
  tile_ld(rv, Vb, a.ldv, bT, 0, T, tid);
  tile_st(sK, rk, tid);
  tile_st(sV, rv, tid);
  if (tid < 64) sMask[tid] = key_flag(a.key_mask, bT, tid, T);
  __syncthreads();

  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1, kb = kt * TK;
    const bool more = kt + 1 < nkt;
    float mk_next = 0.f;
    if (more) {
      tile_ld(rk, Kb, a.ldk, bT, kb + TK, T, tid);
      tile_ld(rv, Vb, a.ldv, bT, kb + TK, T, tid);
      if (tid < 64) mk_next = key_flag(a.key_mask, bT, kb + TK + tid, T);
    }
    const char* tK = sK + cur * TILE;
    const char* tV = sV + cur * TILE;
    const float* mk = sMask + cur * 64;

    f32x4 s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) s[t] = mfma16(frag_kc(tK, t * 16, ss, lane), qf[ss], s[t]);
    }
    const bool all_lo = (kb + TK - 1) - q0 <= -left;
    const bool all_hi = kb - (q0 + 15) >= right;
    float tmax = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kl = 16 * t + 4 * g + r;
        float bias = 0.f;
        if (REL) {
          if (all_lo) bias = qe_lo;
          else if (all_hi) bias = qe_hi;
          else {
            int d = kb + kl - myq;
            d = d < -left ? -left : (d > right ? right : d);
            bias = qe[li * NREL + d + left];
          }
        }
        float v = (s[t][r] + bias) * a.scale;
        const float f = mk[kl];
        v = f > 0.5f ? v : (f < -0.5f ? -INFINITY : NEG_MASK);
        s[t][r] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mnew = fmaxf(m, tmax);
    const float alpha = (mnew == -INFINITY) ? 1.f : __expf(m - mnew);
    float psum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float p = (mnew == -INFINITY) ? 0.f : __expf(s[t][r] - mnew);
        psum += p;
        if (DROP) p *= drop_scale(a.seed, drow + (uint64_t)(kb + 16 * t + 4 * g + r), thresh, inv_keep);
        s[t][r] = p;
      }
    psum += __shfl_xor(psum, 16, 64);
    psum += __shfl_xor(psum, 32, 64);
    l = l * alpha + psum;
    m = mnew;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16x8 pb = pack_acc(s[2 * u], s[2 * u + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] = mfma16(frag_tr(tV, dt * 16, u, lane), pb, o[dt]);
    }
    if (more) {
      tile_st(sK + (cur ^ 1) * TILE, rk, tid);
      tile_st(sV + (cur ^ 1) * TILE, rv, tid);
      if (tid < 64) sMask[(cur ^ 1) * 64 + tid] = mk_next;
    }
    __syncthreads();
  }
  if (myq < T) {
    const float inv_l = 1.0f / l;
    bf16* O = (bf16*)a.o + (int64_t)(bT + myq) * a.ldo + h * HD;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) store_bf16x4(O + 16 * dt + 4 * g, o[dt] * inv_l);
    if (g == 0) a.lse[(int64_t)(b * H + h) * T + myq] = m + logf(l);
  }
}

// ===================================================================== delta = rowsum(dO*O)
__global__ void attn_delta_kernel(ste_attn_args a) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (b*T + q)*H + h
  const int64_t total = (int64_t)a.B * a.T * a.H;
  if (idx >= total) return;
  const int h = idx % a.H;
  const int64_t row = idx / a.H;
  const int b = row / a.T, q = row % a.T;
  const bf16* dO = (const bf16*)a.dout + row * a.lddo + h * HD;
  const bf16* O = (const bf16*)a.o + row * a.ldo + h * HD;
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < HD; c += 8) {
    bf16x8 x = *reinterpret_cast<const bf16x8*>(dO + c);
    bf16x8 y = *reinterpret_cast<const bf16x8*>(O + c);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc += (float)x[e] * (float)y[e];
  }
  a.delta[(int64_t)(b * a.H + h) * a.T + q] = acc;
}

// ======================================================= backward: dQ (+ relative bins G)
template <bool REL, bool DROP>
__global__ __launch_bounds__(NT, 2) void attn_bwd_dq_kernel(ste_attn_args a) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  char* sK = sm;
  char* sV = sm + TILE;
  char* sE = sm + 2 * TILE;                                   // 96 rows x 128 B
  float* sQE = reinterpret_cast<float*>(sE + 96 * 128);       // 4 x 16 x NREL
  float* sG = sQE + 4 * 16 * NREL;                             // 4 x 16 x 96
  float* sMask = sG + 4 * 16 * 96;                             // 64

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
  int tile, h, b;
  tile_of_block(a.T, a.H, tile, h, b);
  const int T = a.T, H = a.H, bT = b * T;
  const int q0 = tile * TQ + w * 16, myq = q0 + li;
  const bool qvalid = myq < T;
  const bf16* Qb = (const bf16*)a.q + h * HD;
  const bf16* Kb = (const bf16*)a.k + h * HD;
  const bf16* Vb = (const bf16*)a.v + h * HD;
  const bf16* dOb = (const bf16*)a.dout + h * HD;
  const int left = a.rel_left, right = a.rel_right, nrel = left + right + 1;

  bf16x8 qf[2], df[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    qf[s] = qvalid ? *reinterpret_cast<const bf16x8*>(Qb + (int64_t)(bT + myq) * a.ldq + 32 * s + 8 * g) : bf16x8{};
    df[s] = qvalid ? *reinterpret_cast<const bf16x8*>(dOb + (int64_t)(bT + myq) * a.lddo + 32 * s + 8 * g) : bf16x8{};
  }
  const int64_t rowid = (int64_t)(b * H + h) * T + myq;
  const float lse = qvalid ? a.lse[rowid] : 0.f;
  const float dl = qvalid ? a.delta[rowid] : 0.f;

  float* qe = sQE + w * 16 * NREL;
  float* gt = sG + w * 16 * 96;
  float qe_lo = 0.f, qe_hi = 0.f;
  if (REL) {
    stage_E(sE, (const bf16*)a.rel_E, nrel, 96, tid);
    for (int i = lane; i < 16 * 96; i += 64) gt[i] = 0.f;
    __syncthreads();
    build_qe(qe, sE, qf, lane);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    qe_lo = qe[li * NREL];
    qe_hi = qe[li * NREL + nrel - 1];
  }
  const uint32_t thresh = (uint32_t)(a.drop_p * 4294967296.0);
  const float inv_keep = DROP ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  const uint64_t drow = (uint64_t)rowid * (uint64_t)T;

  f32x4 dq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dq[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float glo = 0.f, ghi = 0.f;

  const int nkt = (T + TK - 1) / TK;
  for (int kt = 0; kt < nkt; ++kt) {
    const int kb = kt * TK;
    bf16x8 rk[2], rv[2];
    tile_ld(rk, Kb, a.ldk, bT, kb, T, tid);
    tile_ld(rv, Vb, a.ldv, bT, kb, T, tid);
    float mkv = 0.f;
    if (tid < 64) mkv = key_flag(a.key_mask, bT, kb + tid, T);
    __syncthreads();  // previous tile fully consumed
    tile_st(sK, rk, tid);
    tile_st(sV, rv, tid);
    if (tid < 64) sMask[tid] = mkv;
    __syncthreads();

    f32x4 s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        s[t] = mfma16(frag_kc(sK, t * 16, ss, lane), qf[ss], s[t]);
        dp[t] = mfma16(frag_kc(sV, t * 16, ss, lane), df[ss], dp[t]);
      }
    }
    const bool all_lo = (kb + TK - 1) - q0 <= -left;
    const bool all_hi = kb - (q0 + 15) >= right;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kl = 16 * t + 4 * g + r, key = kb + kl;
        int d = key - myq;
        d = d < -left ? -left : (d > right ? right : d);
        float bias = 0.f;
        if (REL) bias = all_lo ? qe_lo : (all_hi ? qe_hi : qe[li * NREL + d + left]);
        float v = (s[t][r] + bias) * a.scale;
        const float f = sMask[kl];
        float p = 0.f;
        if (qvalid && f > -0.5f) p = __expf((f > 0.5f ? v : NEG_MASK) - lse);
        float dpv = dp[t][r];
        if (DROP) dpv *= drop_scale(a.seed, drow + (uint64_t)key, thresh, inv_keep);
        const float ds = p * (dpv - dl);
        s[t][r] = ds;
        if (REL && f > -0.5f) {
          const int j = d + left;
          if (j == 0) glo += ds;
          else if (j == nrel - 1) ghi += ds;
          else gt[li * 96 + j] = ds;
        }
      }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16x8 pb = pack_acc(s[2 * u], s[2 * u + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dq[dt] = mfma16(frag_tr(sK, dt * 16, u, lane), pb, dq[dt]);
    }
  }

  if (REL) {
    glo += __shfl_xor(glo, 16, 64);
    glo += __shfl_xor(glo, 32, 64);
    ghi += __shfl_xor(ghi, 16, 64);
    ghi += __shfl_xor(ghi, 32, 64);
    if (g == 0) {
      gt[li * 96] = glo;
      gt[li * 96 + nrel - 1] = ghi;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    // dQᵀ += Eᵀ·Gᵀ over j (rows of E), 3 k-steps of 32
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const f32x4 g0 = *reinterpret_cast<const f32x4*>(gt + li * 96 + 32 * u + 4 * g);
      const f32x4 g1 = *reinterpret_cast<const f32x4*>(gt + li * 96 + 32 * u + 16 + 4 * g);
      const bf16x8 pb = pack_acc(g0, g1);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dq[dt] = mfma16(frag_tr(sE, dt * 16, u, lane), pb, dq[dt]);
    }
    if (a.dE && qvalid) {
      float* G = a.gwork + rowid * NREL;
#pragma unroll
      for (int c = 0; c < NREL / 4; c += 4) {
        const int j = (c + g) * 4;  // g-th group writes j in {4g, 16+4g, ...}
        if (j < NREL) *reinterpret_cast<f32x4*>(G + j) = *reinterpret_cast<const f32x4*>(gt + li * 96 + j);
      }
    }
  }
  if (qvalid) {
    bf16* dQ = (bf16*)a.dq + (int64_t)(bT + myq) * a.lddq + h * HD;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) store_bf16x4(dQ + 16 * dt + 4 * g, dq[dt] * a.scale);
  }
}

// ==================================================================== backward: dK, dV
template <bool REL, bool DROP>
__global__ __launch_bounds__(NT, 2) void attn_bwd_dkv_kernel(ste_attn_args a) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  char* sQ = sm;                                              // 2 x TILE
  char* sD = sm + 2 * TILE;                                   // 2 x TILE  (dO)
  char* sE = sm + 4 * TILE;                                   // NREL rows x 128 B
  float* sQE = reinterpret_cast<float*>(sE + NREL * 128);     // 64 x NREL
  float* sLD = sQE + 64 * NREL;                               // 2 x (64 lse + 64 delta)

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
  int tile, h, b;
  tile_of_block(a.T, a.H, tile, h, b);
  const int T = a.T, H = a.H, bT = b * T;
  const int mykey = tile * TK + w * 16 + li;
  const bool kvalid = mykey < T;
  const bool kmasked = kvalid && a.key_mask != nullptr && a.key_mask[bT + mykey] == 0;
  const bf16* Qb = (const bf16*)a.q + h * HD;
  const bf16* Kb = (const bf16*)a.k + h * HD;
  const bf16* Vb = (const bf16*)a.v + h * HD;
  const bf16* dOb = (const bf16*)a.dout + h * HD;
  const int left = a.rel_left, right = a.rel_right, nrel = left + right + 1;

  bf16x8 kf[2], vf[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    kf[s] = kvalid ? *reinterpret_cast<const bf16x8*>(Kb + (int64_t)(bT + mykey) * a.ldk + 32 * s + 8 * g) : bf16x8{};
    vf[s] = kvalid ? *reinterpret_cast<const bf16x8*>(Vb + (int64_t)(bT + mykey) * a.ldv + 32 * s + 8 * g) : bf16x8{};
  }
  if (REL) stage_E(sE, (const bf16*)a.rel_E, nrel, NREL, tid);

  const uint32_t thresh = (uint32_t)(a.drop_p * 4294967296.0);
  const float inv_keep = DROP ? 1.0f / (1.0f - a.drop_p) : 1.0f;
  const int64_t rowbase = (int64_t)(b * H + h) * T;

  f32x4 dk[4], dv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { dk[i] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[i] = dk[i]; }

  const int nqt = (T + TQ - 1) / TQ;
  bf16x8 rq[2], rd[2];
  float ld_next = 0.f;
  auto load_ld = [&](int qb) -> float {
    if (tid < 128) {
      int q = qb + (tid & 63);
      if (q < T) return (tid < 64) ? a.lse[rowbase + q] : a.delta[rowbase + q];
    }
    return 0.f;
  };
  tile_ld(rq, Qb, a.ldq, bT, 0, T, tid);
  tile_ld(rd, dOb, a.lddo, bT, 0, T, tid);
  tile_st(sQ, rq, tid);
  tile_st(sD, rd, tid);
  ld_next = load_ld(0);
  if (tid < 128) sLD[tid] = ld_next;
  __syncthreads();

  for (int qt = 0; qt < nqt; ++qt) {
    const int cur = qt & 1, qb = qt * TQ;
    const bool more = qt + 1 < nqt;
    if (more) {
      tile_ld(rq, Qb, a.ldq, bT, qb + TQ, T, tid);
      tile_ld(rd, dOb, a.lddo, bT, qb + TQ, T, tid);
      ld_next = load_ld(qb + TQ);
    }
    const char* tQ = sQ + cur * TILE;
    const char* tD = sD + cur * TILE;
    const float* sL = sLD + cur * 128;
    if (REL) {
      // QE rows of this q tile: wave w builds rows 16w..16w+15
      bf16x8 qfr[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) qfr[s] = frag_kc(tQ, 16 * w, s, lane);
      build_qe(sQE + 16 * w * NREL, sE, qfr, lane);
      __syncthreads();
    }
    f32x4 s[4], dp[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      s[n] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[n] = s[n];
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        s[n] = mfma16(frag_kc(tQ, 16 * n, ss, lane), kf[ss], s[n]);
        dp[n] = mfma16(frag_kc(tD, 16 * n, ss, lane), vf[ss], dp[n]);
      }
    }
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = 16 * n + 4 * g + r, q = qb + ql;
        float bias = 0.f;
        if (REL) {
          int d = mykey - q;
          d = d < -left ? -left : (d > right ? right : d);
          bias = sQE[ql * NREL + d + left];
        }
        float v = (s[n][r] + bias) * a.scale;
        if (kmasked) v = NEG_MASK;
        float p = (kvalid && q < T) ? __expf(v - sL[ql]) : 0.f;
        float dpv = dp[n][r];
        float pd = p;
        if (DROP) {
          const float dsc = drop_scale(a.seed, (uint64_t)(rowbase + q) * (uint64_t)T + (uint64_t)mykey, thresh, inv_keep);
          pd *= dsc;
          dpv *= dsc;
        }
        const float ds = p * (dpv - sL[64 + ql]);
        s[n][r] = pd;
        dp[n][r] = ds * a.scale;
      }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16x8 pv = pack_acc(s[2 * u], s[2 * u + 1]);
      const bf16x8 pk = pack_acc(dp[2 * u], dp[2 * u + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dv[dt] = mfma16(frag_tr(tD, dt * 16, u, lane), pv, dv[dt]);
        dk[dt] = mfma16(frag_tr(tQ, dt * 16, u, lane), pk, dk[dt]);
      }
    }
    if (more) {
      tile_st(sQ + (cur ^ 1) * TILE, rq, tid);
      tile_st(sD + (cur ^ 1) * TILE, rd, tid);
      if (tid < 128) sLD[(cur ^ 1) * 128 + tid] = ld_next;
    }
    __syncthreads();
  }
  if (kvalid) {
    bf16* dK = (bf16*)a.dk + (int64_t)(bT + mykey) * a.lddk + h * HD;
    bf16* dV = (bf16*)a.dv + (int64_t)(bT + mykey) * a.lddv + h * HD;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      store_bf16x4(dK + 16 * dt + 4 * g, dk[dt]);
      store_bf16x4(dV + 16 * dt + 4 * g, dv[dt]);
    }
  }
}

// ================================================ dE[j][d] += scale * Σ_rows G[row][j] Q[row][d]
// rows = (b, h, q); 256 threads each own 20 (j, d) outputs; rows staged 32 at a time.
__global__ __launch_bounds__(256) void attn_rel_dE_kernel(ste_attn_args a, int64_t rows_per_block) {
  __shared__ float sG[32][NREL];
  __shared__ float sQ[32][HD];
  const int tid = threadIdx.x;
  const int nrel = a.rel_left + a.rel_right + 1;
  const int64_t total = (int64_t)a.B * a.H * a.T;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < total ? r0 + rows_per_block : total;
  float acc[20];
#pragma unroll
  for (int i = 0; i < 20; ++i) acc[i] = 0.f;
  for (int64_t rb = r0; rb < r1; rb += 32) {
    __syncthreads();
    for (int i = tid; i < 32 * NREL; i += 256) {
      int rr = i / NREL, j = i % NREL;
      int64_t row = rb + rr;
      sG[rr][j] = row < r1 ? a.gwork[row * NREL + j] : 0.f;
    }
    for (int i = tid; i < 32 * HD; i += 256) {
      int rr = i / HD, d = i % HD;
      int64_t row = rb + rr;
      float v = 0.f;
      if (row < r1) {
        int q = row % a.T;
        int64_t bh = row / a.T;
        int h = bh % a.H, b = bh / a.H;
        v = (float)((const bf16*)a.q)[(int64_t)(b * a.T + q) * a.ldq + h * HD + d];
      }
      sQ[rr][d] = v;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 20; ++i) {
      const int o = tid + 256 * i;
      if (o < NREL * HD) {
        const int j = o / HD, d = o % HD;
        float s = acc[i];
#pragma unroll 8
        for (int rr = 0; rr < 32; ++rr) s += sG[rr][j] * sQ[rr][d];
        acc[i] = s;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 20; ++i) {
    const int o = tid + 256 * i;
    if (o < nrel * HD) atomicAdd(a.dE + o, acc[i] * a.scale);
  }
}

constexpr int FWD_LDS = 4 * TILE + NREL * 128 + 4 * 16 * NREL * 4 + 2 * 64 * 4;
constexpr int DQ_LDS = 2 * TILE + 96 * 128 + 4 * 16 * NREL * 4 + 4 * 16 * 96 * 4 + 64 * 4;
constexpr int DKV_LDS = 4 * TILE + NREL * 128 + 64 * NREL * 4 + 2 * 128 * 4;

template <template <bool, bool> class K>
struct Dispatch;

int check(const ste_attn_args* a) {
  if (!a || a->B <= 0 || a->T <= 0 || a->H <= 0) return STE_ERR_ARG;
  if ((a->ldq & 7) || (a->ldk & 7) || (a->ldv & 7) || (a->ldo & 7)) return STE_ERR_SHAPE;
  if (a->rel_E && a->rel_left + a->rel_right + 1 > NREL) return STE_ERR_SHAPE;
  if (a->drop_p < 0.f || a->drop_p >= 1.f) return STE_ERR_ARG;
  return 0;
}

}  // namespace

extern "C" int ste_attention_fwd(const ste_attn_args* a, void* stream) {
  if (int e = check(a)) return e;
  if (!a->lse || !a->o) return STE_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)(((a->T + TQ - 1) / TQ) * a->H * a->B));
  const bool rel = a->rel_E != nullptr, drop = a->drop_p > 0.f;
  if (rel && drop) hipLaunchKernelGGL((attn_fwd_kernel<true, true>), grid, dim3(NT), FWD_LDS, s, *a);
  else if (rel) hipLaunchKernelGGL((attn_fwd_kernel<true, false>), grid, dim3(NT), FWD_LDS, s, *a);
  else if (drop) hipLaunchKernelGGL((attn_fwd_kernel<false, true>), grid, dim3(NT), FWD_LDS, s, *a);
  else hipLaunchKernelGGL((attn_fwd_kernel<false, false>), grid, dim3(NT), FWD_LDS, s, *a);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_attention_bwd(const ste_attn_args* a, void* stream) {
  if (int e = check(a)) return e;
  if (!a->dout || !a->o || !a->lse || !a->delta || !a->dq || !a->dk || !a->dv) return STE_ERR_ARG;
  if ((a->lddo & 7) || (a->lddq & 3) || (a->lddk & 3) || (a->lddv & 3)) return STE_ERR_SHAPE;
  if (a->dE && (!a->gwork || !a->rel_E)) return STE_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t nrow = (int64_t)a->B * a->T * a->H;
  hipLaunchKernelGGL(attn_delta_kernel, dim3((unsigned)((nrow + 255) / 256)), dim3(256), 0, s, *a);
  STE_CHECK_LAUNCH();
  dim3 grid((unsigned)(((a->T + TQ - 1) / TQ) * a->H * a->B));
  const bool rel = a->rel_E != nullptr, drop = a->drop_p > 0.f;
#define STE_LAUNCH2(KER, LDS)                                                            \
  if (rel && drop) hipLaunchKernelGGL((KER<true, true>), grid, dim3(NT), LDS, s, *a);    \
  else if (rel) hipLaunchKernelGGL((KER<true, false>), grid, dim3(NT), LDS, s, *a);      \
  else if (drop) hipLaunchKernelGGL((KER<false, true>), grid, dim3(NT), LDS, s, *a);     \
  else hipLaunchKernelGGL((KER<false, false>), grid, dim3(NT), LDS, s, *a);              \
  STE_CHECK_LAUNCH();
  STE_LAUNCH2(attn_bwd_dq_kernel, DQ_LDS)
  STE_LAUNCH2(attn_bwd_dkv_kernel, DKV_LDS)
#undef STE_LAUNCH2
  if (a->dE) {
    const int blocks = 512;
    int64_t rpb = (nrow + blocks - 1) / blocks;
    hipLaunchKernelGGL(attn_rel_dE_kernel, dim3(blocks), dim3(256), 0, s, *a, rpb);
    STE_CHECK_LAUNCH();
  }
  return 0;
}

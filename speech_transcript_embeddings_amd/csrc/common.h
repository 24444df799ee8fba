// Device-side helpers shared by every ste kernel (gfx950 / CDNA4 only).
//
// Conventions used throughout csrc/:
//   * activations that feed MFMA are bf16 (`bf16` = clang's __bf16), accumulation is fp32;
//   * the residual stream, LayerNorm statistics, softmax and loss math are fp32;
//   * a wavefront is 64 lanes (never 32);
//   * every launcher takes the HIP stream it must run on and never synchronises.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define STE_WAVE 64
#define STE_DEV __device__ __forceinline__
#define STE_HD __host__ __device__ __forceinline__

// ---------------------------------------------------------------- conversions
STE_DEV float bf2f(bf16 x) { return (float)x; }
STE_DEV bf16 f2bf(float x) { return (bf16)x; }  // RNE, NaN-preserving (v_cvt_pk_bf16_f32)

STE_DEV f32x4 load_bf16x4(const bf16* p) {
  bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
STE_DEV void store_bf16x4(bf16* p, f32x4 v) {
  bf16x4 o;
  o[0] = (bf16)v[0]; o[1] = (bf16)v[1]; o[2] = (bf16)v[2]; o[3] = (bf16)v[3];
  *reinterpret_cast<bf16x4*>(p) = o;
}
// hi/lo split of fp32 values: hi = bf16(v), lo = bf16(v - hi); hi + lo carries ~16 mantissa
// bits (used where a backward needs the fp32 value of a bf16-stored forward output)
STE_DEV void store_bf16x4_split(bf16* hi_p, bf16* lo_p, f32x4 v) {
  bf16x4 h, l;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    h[i] = (bf16)v[i];
    l[i] = (bf16)(v[i] - (float)h[i]);
  }
  *reinterpret_cast<bf16x4*>(hi_p) = h;
  *reinterpret_cast<bf16x4*>(lo_p) = l;
}

// ---------------------------------------------------------------- wave reductions
// Cross-lane steps without LDS: DPP within each 16-lane row (quad_perm xor 1, xor 2, then
// row_half_mirror and row_mirror, which pair the row's quads and halves), then
// v_permlane32_swap / v_permlane16_swap across the rows (__shfl_xor compiles to ds_bpermute:
// an LDS round trip and an lgkmcnt drain per step).  Every step adds the same two values in
// both partner lanes, so all 64 lanes end with the same bits.  Call with every lane active.
template <int CTRL>
STE_DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
STE_DEV float xrow32_sum(float v) {
  const uint32_t u = __builtin_bit_cast(uint32_t, v);
  auto p = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  const float y = __builtin_bit_cast(float, (uint32_t)p[0]) + __builtin_bit_cast(float, (uint32_t)p[1]);
  const uint32_t w = __builtin_bit_cast(uint32_t, y);
  auto q = __builtin_amdgcn_permlane16_swap(w, w, false, false);
  return __builtin_bit_cast(float, (uint32_t)q[0]) + __builtin_bit_cast(float, (uint32_t)q[1]);
}
STE_DEV float wave_sum(float v) {
  v += dpp_f<0xB1>(v);    // quad_perm [1,0,3,2]: lane ^ 1
  v += dpp_f<0x4E>(v);    // quad_perm [2,3,0,1]: lane ^ 2
  v += dpp_f<0x141>(v);   // row_half_mirror: the other quad of the 8-lane half
  v += dpp_f<0x140>(v);   // row_mirror: the other half of the 16-lane row
  return xrow32_sum(v);
}
STE_DEV float wave_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  const uint32_t u = __builtin_bit_cast(uint32_t, v);
  auto p = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  const float y = fmaxf(__builtin_bit_cast(float, (uint32_t)p[0]), __builtin_bit_cast(float, (uint32_t)p[1]));
  const uint32_t w = __builtin_bit_cast(uint32_t, y);
  auto q = __builtin_amdgcn_permlane16_swap(w, w, false, false);
  return fmaxf(__builtin_bit_cast(float, (uint32_t)q[0]), __builtin_bit_cast(float, (uint32_t)q[1]));
}
STE_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------- activations
// OCP MX block-scale exponent for e4m3 payloads: e = ceil(log2(amax/448)) (the block's largest
// element maps to <= 448, no saturation), -127 (2^-127) for an all-zero block.
STE_DEV int mx8_exp(float amax) {
  if (!(amax > 0.f)) return -127;
  int e2;
  const float m = frexpf(amax * (1.0f / 448.0f), &e2);  // amax/448 = m·2^e2, m in [0.5, 1)
  return max(-127, min(127, (m == 0.5f) ? e2 - 1 : e2));
}
STE_DEV float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }
STE_DEV float swish_f(float x) { return x * sigmoidf_(x); }
STE_DEV float swish_d(float x) {
  float s = sigmoidf_(x);
  return s * (1.0f + x * (1.0f - s));
}
// exact erf GELU (torch nn.GELU() default, approximate='none')
STE_DEV float gelu_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
STE_DEV float gelu_d(float x) {
  float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// ---------------------------------------------------------------- dropout RNG
// Counter-based: keep(seed, idx) is a pure function, so backward regenerates the
// forward mask bit-for-bit without storing it.  murmur3 fmix64 on (seed, idx).
STE_DEV uint32_t ste_hash(uint64_t seed, uint64_t idx) {
  uint64_t x = seed ^ (idx * 0x9E3779B97F4A7C15ull);
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return (uint32_t)x;
}
// returns scale (0 or 1/(1-p)) for element idx
STE_DEV float drop_scale(uint64_t seed, uint64_t idx, uint32_t thresh, float inv_keep) {
  return ste_hash(seed, idx) >= thresh ? inv_keep : 0.0f;
}

// ---------------------------------------------------------------- MFMA wrappers
STE_DEV f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// ds_read_b64_tr_b16: see cdna_hip_programming.md T10.  Within each 16-lane group,
// lane 4q+p passes the address of row q, columns 4p..4p+3; lane i receives
// column i of the 4 rows (row q in element q).
STE_DEV s16x4 ds_read_tr16(const void* lds_ptr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds_ptr));
}
STE_DEV bf16x8 join_tr(s16x4 lo, s16x4 hi) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// MI355X dispatches workgroup i of a launch to XCD i % 8, and each XCD has its own L2.
// Return a logical id such that logically consecutive ids share an XCD (bijective on [0, n)),
// so blocks that re-read the same operands (GEMM tiles of one row panel, attention q-tiles
// of one (batch, head)) hit the same L2.
STE_DEV int xcd_remap(int bid, int n) {
  const int xcd = bid & 7, q = n >> 3, r = n & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}


typedef __attribute__((address_space(3))) void lds_void;
// ds_read_b64_tr_b16 through inline asm: invisible to hipcc's waitcnt pass, which would
// otherwise treat the builtin as aliasing every in-flight global_load_lds and drain them
// with vmcnt(0).  The caller orders the read itself (lgkmcnt(0) + sched_barrier(0) before
// the consuming MFMAs).
STE_DEV s16x4 ds_read_tr16_asm(const char* p) {
  typedef __attribute__((address_space(3))) const char lds_cchar;
  const uint32_t off = (uint32_t)(uintptr_t)(lds_cchar*)p;
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(off) : "memory");
  return r;
}

// A/B switches.  The shipped library reads no environment: STE_AB_ENV(name) is a null pointer
// there, so every switch takes its default.  Builds with -DSTE_AB (_build.py --ab -> libste_ab.so,
// for same-box A/B runs only) read the named variable.
#ifdef STE_AB
#include <cstdlib>
#define STE_AB_ENV(name) getenv(name)
#else
#define STE_AB_ENV(name) ((const char*)nullptr)
#endif

#define STE_CHECK_LAUNCH() do { hipError_t e_ = hipGetLastError(); if (e_ != hipSuccess) return (int)e_; } while (0)

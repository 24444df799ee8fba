// Small elementwise helpers of the hot path (casts, row masks, version string).
#include "common.h"
#include "../../include/ste.h"

namespace {
__global__ void cast_kernel(const float* __restrict__ x, bf16* __restrict__ y, int64_t n) {
  int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (; i + 3 < n; i += stride) store_bf16x4(y + i, *reinterpret_cast<const f32x4*>(x + i));
  if (i < n) for (; i < n; ++i) y[i] = (bf16)x[i];
}
// y [rows][nblk·K] bf16 = nblk blocks of x [rows][K] fp32: block i is hi = bf16(x) or, when bit i
// of `lo_mask` is set, lo = bf16(x - hi).  A GEMM over the concatenated columns of A = [hi|lo] and
// B = [W|W] sums a_hi·W + a_lo·W: the activation to ~16 mantissa bits against the bf16 weight,
// with fp32 accumulation, on the bf16 MFMA (3 blocks, [hi|lo|hi]·[hi|hi|lo], add a_hi·w_lo).
// 4 columns per thread.
__global__ __launch_bounds__(256) void split_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows, int K,
                                                   bf16* __restrict__ y, int nblk, int lo_mask) {
  const int per_row = K >> 2;
  const int64_t total = rows * per_row;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t r = t / per_row;
    const int c = (int)(t - r * per_row) * 4;
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + r * ldx + c);
    bf16x4 hi, lo;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      hi[e] = (bf16)v[e];
      lo[e] = (bf16)(v[e] - (float)hi[e]);
    }
    bf16* o = y + r * nblk * K + c;
    for (int i = 0; i < nblk; ++i) *reinterpret_cast<bf16x4*>(o + (int64_t)i * K) = ((lo_mask >> i) & 1) ? lo : hi;
  }
}
__global__ void scale_rows_kernel(float* x, const float* s, int64_t rows, int cols, int64_t ld) {
  int64_t r = blockIdx.x;
  float f = s[r];
  if ((cols & 3) || (ld & 3)) {
    for (int c = threadIdx.x; c < cols; c += blockDim.x) x[r * ld + c] *= f;
    return;
  }
  for (int c = threadIdx.x * 4; c < cols; c += blockDim.x * 4) {
    f32x4* p = reinterpret_cast<f32x4*>(x + r * ld + c);
    *p = *p * f;
  }
}
__global__ void mask_cvt_kernel(const int64_t* m, float* f, int32_t* i32, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    int64_t v = m[i];
    if (f) f[i] = v != 0 ? 1.0f : 0.0f;
    if (i32) i32[i] = v != 0 ? 1 : 0;
  }
}
// out[c] += Σ_r x[r, c]; block = 64-column stripe x row chunk, 256 threads = 16 cols x 16 row lanes (x4 vector)
__global__ void colsum_kernel(const void* x, int is_bf16, int64_t rows, int cols, int64_t ld, float* out,
                              int64_t rows_per_block, float* part) {
  __shared__ float red[16][65];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + tx * 4;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < rows ? r0 + rows_per_block : rows;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (c < cols) {
    for (int64_t r = r0 + ty; r < r1; r += 16) {
      if (is_bf16) acc += load_bf16x4((const bf16*)x + r * ld + c);
      else acc += *reinterpret_cast<const f32x4*>((const float*)x + r * ld + c);
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) red[ty][tx * 4 + e] = acc[e];
  __syncthreads();
  if (threadIdx.x < 64) {
    const int cc = blockIdx.x * 64 + threadIdx.x;
    float s = 0.f;
#pragma unroll
    for (int y = 0; y < 16; ++y) s += red[y][threadIdx.x];
    if (cc < cols) {
      if (part) part[(int64_t)blockIdx.y * cols + cc] = s;   // this row chunk's partial (ordered 2nd pass)
      else atomicAdd(out + cc, s);
    }
  }
}
// out[b·cols + c] += Σ_r part[(b·R + r)·cols + c] in a fixed order (RS_SL interleaved slices of
// the rows, then the slices in order): the ordered second pass of every deterministic column sum
// (GEMM bias gradients, ste_colsum, depthwise-conv and SpecAugment gradients).  A block owns
// RS_CW columns (64-B row segments) and RS_SL = 64 row slices, so a 1,024-column sum spreads over
// 64 blocks instead of 16 and each thread walks R / 64 rows, 8 loads in flight.
// grid (ceil(cols / RS_CW), batch), 1024 threads
constexpr int RS_CW = 16, RS_SL = 1024 / RS_CW;
__global__ __launch_bounds__(1024) void rowsum_ordered_kernel(const float* __restrict__ part, int64_t R, int cols,
                                                              float* out) {
  __shared__ float red[RS_SL][RS_CW];
  const int c = threadIdx.x % RS_CW, sl = threadIdx.x / RS_CW;
  const int col = blockIdx.x * RS_CW + c;
  float acc = 0.f;
  if (col < cols) {
    const float* p = part + (int64_t)blockIdx.y * R * cols + col;
    int64_t r = sl;
    for (; r + 7 * RS_SL < R; r += 8 * RS_SL) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[(r + RS_SL * u) * cols];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; r < R; r += RS_SL) acc += p[r * cols];
  }
  red[sl][c] = acc;
  __syncthreads();
  if (sl == 0 && col < cols) {
    float t = red[0][c];
    for (int k = 1; k < RS_SL; ++k) t += red[k][c];
    out[(int64_t)blockIdx.y * cols + col] += t;
  }
}
// y[r, c] = alpha * x[r, c] + beta * y[r, c] (fp32, strided rows)
__global__ void axpby2d_kernel(float* y, int64_t ldy, const float* x, int64_t ldx, int64_t rows, int cols,
                               float alpha, float beta) {
  const int64_t r = blockIdx.x;
  for (int c = threadIdx.x; c < cols; c += blockDim.x) {
    float* yp = y + r * ldy + c;
    *yp = alpha * x[r * ldx + c] + (beta != 0.f ? beta * *yp : 0.f);
  }
}
// 2-D copy of 2- or 4-byte elements between strided row-major views
__global__ void copy2d_kernel(char* y, int64_t ldy, const char* x, int64_t ldx, int64_t rows, int cols, int esz) {
  const int64_t r = blockIdx.x;
  for (int c = threadIdx.x; c < cols; c += blockDim.x) {
    if (esz == 4) reinterpret_cast<float*>(y)[r * ldy + c] = reinterpret_cast<const float*>(x)[r * ldx + c];
    else reinterpret_cast<uint16_t*>(y)[r * ldy + c] = reinterpret_cast<const uint16_t*>(x)[r * ldx + c];
  }
}
// y[c, r] = x[r, c] for 2-byte elements: 64 x 64 tiles through LDS (a padded row keeps the
// column reads conflict-free), 16-B global loads and stores on full tiles
__global__ __launch_bounds__(256) void transpose16_kernel(uint16_t* __restrict__ y, int64_t ldy,
                                                          const uint16_t* __restrict__ x, int64_t ldx, int64_t rows,
                                                          int cols) {
  __shared__ uint16_t t[64][64 + 2];
  const int64_t r0 = (int64_t)blockIdx.y * 64;
  const int c0 = blockIdx.x * 64;
  const int tid = threadIdx.x;
  const bool full = r0 + 64 <= rows && c0 + 64 <= cols && !(ldx & 7) && !(ldy & 7);
  if (full) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {  // 64 rows x 8 chunks of 8 elements
      const int idx = tid + 256 * k, rr = idx >> 3, ch = idx & 7;
      typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
      const u16x8 v = *reinterpret_cast<const u16x8*>(x + (r0 + rr) * ldx + c0 + 8 * ch);
#pragma unroll
      for (int e = 0; e < 8; ++e) t[rr][8 * ch + e] = v[e];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int idx = tid + 256 * k, cc = idx >> 3, ch = idx & 7;
      typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
      u16x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = t[8 * ch + e][cc];
      *reinterpret_cast<u16x8*>(y + (int64_t)(c0 + cc) * ldy + r0 + 8 * ch) = v;
    }
    return;
  }
  for (int idx = tid; idx < 64 * 64; idx += 256) {
    const int rr = idx >> 6, cc = idx & 63;
    if (r0 + rr < rows && c0 + cc < cols) t[rr][cc] = x[(r0 + rr) * ldx + c0 + cc];
  }
  __syncthreads();
  for (int idx = tid; idx < 64 * 64; idx += 256) {
    const int cc = idx >> 6, rr = idx & 63;
    if (r0 + rr < rows && c0 + cc < cols) y[(int64_t)(c0 + cc) * ldy + r0 + rr] = t[rr][cc];
  }
}
// SpecAugment rows (spec[r] != 0 and valid[r] != 0): forward x[r,:] = embed; backward
// dembed += Σ dx[r,:] over those rows (block partials + one atomic per column per block) and
// dx[r,:] = 0 (the replaced projection output gets no gradient)
__global__ __launch_bounds__(256) void spec_mask_fwd_kernel(float* x, int64_t ld, const int32_t* spec,
                                                            const float* valid, const float* embed, int64_t rows,
                                                            int cols) {
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    if (!spec[r] || valid[r] == 0.f) continue;
    for (int c = threadIdx.x; c < cols; c += blockDim.x) x[r * ld + c] = embed[c];
  }
}
__global__ __launch_bounds__(256) void spec_mask_bwd_kernel(float* dx, int64_t ld, const int32_t* spec,
                                                            const float* valid, float* dembed, int64_t rows,
                                                            int cols, float* part) {
  for (int c0 = 0; c0 < cols; c0 += blockDim.x) {
    const int c = c0 + threadIdx.x;
    float acc = 0.f;
    for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
      if (!spec[r] || valid[r] == 0.f) continue;
      if (c < cols) {
        acc += dx[r * ld + c];
        dx[r * ld + c] = 0.f;
      }
    }
    if (part) {
      if (c < cols) part[(int64_t)blockIdx.x * cols + c] = acc;
    } else if (dembed && c < cols && acc != 0.f) {
      atomicAdd(dembed + c, acc);
    }
  }
}
}  // namespace

extern "C" int ste_spec_mask_fwd(float* x, int64_t ld, const int32_t* spec, const float* valid, const float* embed,
                                 int64_t rows, int cols, void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  if (!x || !spec || !valid || !embed) return STE_ERR_ARG;
  const int blocks = (int)(rows < 2048 ? rows : 2048);
  hipLaunchKernelGGL(spec_mask_fwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, ld, spec, valid, embed,
                     rows, cols);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t ste_spec_mask_bwd_ws_floats(int64_t rows, int cols) {
  return (rows < 512 ? rows : 512) * (int64_t)cols;
}

extern "C" int ste_spec_mask_bwd(float* dx, int64_t ld, const int32_t* spec, const float* valid, float* dembed,
                                 int64_t rows, int cols, float* ws, int64_t ws_floats, void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  if (!dx || !spec || !valid) return STE_ERR_ARG;
  const int blocks = (int)(rows < 512 ? rows : 512);
  float* part = (dembed && ws && ws_floats >= (int64_t)blocks * cols) ? ws : nullptr;
  hipLaunchKernelGGL(spec_mask_bwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, dx, ld, spec, valid,
                     dembed, rows, cols, part);
  STE_CHECK_LAUNCH();
  if (part) return ste_rowsum_ordered(part, blocks, cols, 1, dembed, stream);
  return 0;
}

extern "C" int ste_rowsum_ordered(const float* part, int64_t rows, int cols, int batch, float* out, void* stream) {
  if (rows <= 0 || cols <= 0 || batch <= 0) return 0;
  if (!part || !out) return STE_ERR_ARG;
  hipLaunchKernelGGL(rowsum_ordered_kernel, dim3((cols + RS_CW - 1) / RS_CW, batch), dim3(1024), 0, (hipStream_t)stream, part,
                     rows, cols, out);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_transpose16(void* y, int64_t ldy, const void* x, int64_t ldx, int64_t rows, int cols,
                               void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  if (ldx < cols || ldy < rows) return STE_ERR_ARG;
  dim3 grid((unsigned)((cols + 63) / 64), (unsigned)((rows + 63) / 64));
  hipLaunchKernelGGL(transpose16_kernel, grid, dim3(256), 0, (hipStream_t)stream, (uint16_t*)y, ldy,
                     (const uint16_t*)x, ldx, rows, cols);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_axpby2d(float* y, int64_t ldy, const float* x, int64_t ldx, int64_t rows, int cols, float alpha,
                           float beta, void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  hipLaunchKernelGGL(axpby2d_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, y, ldy, x, ldx, rows,
                     cols, alpha, beta);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_copy2d(void* y, int64_t ldy, const void* x, int64_t ldx, int64_t rows, int cols, int elem_bytes,
                          void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  if (elem_bytes != 2 && elem_bytes != 4) return STE_ERR_ARG;
  hipLaunchKernelGGL(copy2d_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, (char*)y, ldy,
                     (const char*)x, ldx, rows, cols, elem_bytes);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t ste_colsum_ws_floats(int64_t rows, int cols) {
  return (rows + 511) / 512 * (int64_t)cols;
}

extern "C" int ste_colsum(const void* x, int is_bf16, int64_t rows, int cols, int64_t ld, float* out, float* ws,
                          int64_t ws_floats, void* stream) {
  if (rows <= 0) return 0;
  if ((cols & 3) || (ld & 3)) return STE_ERR_SHAPE;
  const int64_t rpb = 512;
  const int64_t chunks = (rows + rpb - 1) / rpb;
  float* part = (ws && ws_floats >= chunks * cols) ? ws : nullptr;
  dim3 grid((cols + 63) / 64, (unsigned)chunks);
  hipLaunchKernelGGL(colsum_kernel, grid, dim3(256), 0, (hipStream_t)stream, x, is_bf16, rows, cols, ld, out, rpb,
                     part);
  STE_CHECK_LAUNCH();
  if (part) return ste_rowsum_ordered(part, chunks, cols, 1, out, stream);
  return 0;
}

extern "C" int ste_cast_f32_bf16(const float* x, void* y, int64_t n, void* stream) {
  if (n <= 0) return 0;
  int64_t blocks = (n / 4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  // vector path needs 16-B aligned x and 8-B aligned y
  if ((((uintptr_t)x) & 15) || (((uintptr_t)y) & 7)) return STE_ERR_ARG;
  hipLaunchKernelGGL(cast_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x, (bf16*)y, n);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_scale_rows(float* x, const float* scale, int64_t rows, int cols, int64_t ld, void* stream) {
  if (rows <= 0) return 0;
  if (cols <= 0 || ld < cols) return STE_ERR_SHAPE;
  hipLaunchKernelGGL(scale_rows_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, x, scale, rows, cols, ld);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_mask_i64_to_f32(const int64_t* m, float* f, int32_t* i32, int64_t n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(mask_cvt_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, m, f, i32, n);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" int ste_split_bf16(const float* x, int64_t ldx, int64_t rows, int K, void* y, int nblk, int lo_mask,
                              void* stream) {
  if (rows <= 0 || K <= 0 || (K & 3) || (ldx & 3) || ((uintptr_t)x & 15) || ((uintptr_t)y & 7) || nblk < 1 ||
      nblk > 3 || (lo_mask >> nblk))
    return STE_ERR_SHAPE;
  const int64_t work = rows * (K >> 2);
  const unsigned blocks = (unsigned)((work + 255) / 256 < 8192 ? (work + 255) / 256 : 8192);
  hipLaunchKernelGGL(split_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, ldx, rows, K, (bf16*)y, nblk,
                     lo_mask);
  STE_CHECK_LAUNCH();
  return 0;
}

extern "C" const char* ste_version(void) { return "ste-0.1-gfx950"; }

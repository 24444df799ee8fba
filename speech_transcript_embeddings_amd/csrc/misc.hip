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
__global__ void scale_rows_kernel(float* x, const float* s, int64_t rows, int cols, int64_t ld) {
  int64_t r = blockIdx.x;
  float f = s[r];
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
}  // namespace

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
  if ((cols & 3) || (ld & 3)) return STE_ERR_SHAPE;
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

extern "C" const char* ste_version(void) { return "ste-0.1-gfx950"; }

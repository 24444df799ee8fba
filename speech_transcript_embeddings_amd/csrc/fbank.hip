// Batched GPU fbank: the arithmetic of SeamlessM4TFeatureExtractor (w2v-bert-2.0's
// extractor) that the reference runs per clip on CPU DataLoader workers
// (ref:training/trainer_unfreeze.py:856-866 -> tf:models/seamless_m4t/
// feature_extraction_seamless_m4t.py:112-138,240-301, tf:audio_utils.py:809-1017),
// plus the collate padding of ref:training/trainer_unfreeze.py:880-921.
//
// Kernel 1 (one wavefront per 400-sample frame, 4 frames per block):
//   x*2^15 -> remove frame mean -> pre-emphasis 0.97 (y0 *= 0.03) -> povey window
//   -> 512-point radix-2 FFT in LDS (fp32, twiddles from double sincos) -> |X|^2
//   -> 80 kaldi-scale triangular mel filters built in mel space (sparse, per-block
//   table) -> max(1.1920929e-7, .) -> natural log.
// Kernel 2 (one block per clip): per-mel-bin mean and unbiased variance over the clip's
// frames exactly as numpy evaluates them on the extractor's float32 log-mel array
// (tf:…seamless_m4t…:256-261: x.mean(0), x.var(0, ddof=1), (x - mean)/sqrt(var + 1e-7)):
// float32 sums accumulated frame by frame in order (numpy's reduction over a non-contiguous
// axis), IEEE float32 division and square root.  A bin whose frames are all equal (silence at
// the log floor) therefore reproduces the reference's non-zero rounding residue bit for bit.
// Kernel 3 (rows of many clips per block): (x - mean)/std, pad odd frame counts with
// padding_value, stack frame pairs into 160-d rows, zero rows beyond the clip, write the mask.
// HBM-bound: 4 B/sample in, 640 B per stacked frame + mask out.
#include "common.h"
#include "../../include/ste.h"

namespace {

constexpr int FRAME = 400, HOP = 160, NFFT = 512, NBIN = 257, NMEL = 80;
constexpr int MAXNZ = 640;  // non-zero filter taps (501 for these parameters)

__device__ double hz_to_mel(double f) { return 1127.0 * log(1.0 + f / 700.0); }

// Constant tables (built once per call by one block, read by every frame block):
//   [0, 512)   twiddles e^{-2πik/512} (float2 x 256)     [512, 912)  povey window
//   [912, 992) mel start bin  [992, 1072) mel length  [1072, 1152) mel offset (ints)
//   [1152, 1152+MAXNZ) mel weights (kaldi scale, triangles in mel space, fp64 -> fp32)
constexpr int T_TW = 0, T_WIN = 512, T_MSTART = 912, T_MLEN = 992, T_MOFF = 1072, T_MW = 1152;
constexpr int TABLE_FLOATS = 2048;

__global__ __launch_bounds__(256) void fbank_tables_kernel(float* __restrict__ tab) {
  __shared__ double fk[NBIN];
  __shared__ int slen[NMEL], soff[NMEL];
  const int tid = threadIdx.x;
  for (int k = tid; k < NFFT / 2; k += 256) {
    double s, c;
    sincos(-2.0 * M_PI * (double)k / (double)NFFT, &s, &c);
    tab[T_TW + 2 * k] = (float)c;
    tab[T_TW + 2 * k + 1] = (float)s;
  }
  for (int n = tid; n < FRAME; n += 256) {
    const double hann = 0.5 - 0.5 * cos(2.0 * M_PI * (double)n / (double)(FRAME - 1));
    tab[T_WIN + n] = (float)pow(hann, 0.85);
  }
  for (int k = tid; k < NBIN; k += 256) fk[k] = hz_to_mel(31.25 * k);
  __syncthreads();
  const double mel_lo = hz_to_mel(20.0), mel_hi = hz_to_mel(8000.0);
  int start = 0, len = 0;
  double f0 = 0, f1 = 0, f2 = 0;
  if (tid < NMEL) {
    f0 = mel_lo + (mel_hi - mel_lo) * tid / (NMEL + 1);
    f1 = mel_lo + (mel_hi - mel_lo) * (tid + 1) / (NMEL + 1);
    f2 = mel_lo + (mel_hi - mel_lo) * (tid + 2) / (NMEL + 1);
    start = -1;
    for (int k = 0; k < NBIN; ++k) {
      const double wv = fmax(0.0, fmin((fk[k] - f0) / (f1 - f0), (f2 - fk[k]) / (f2 - f1)));
      if (wv > 0.0) { if (start < 0) start = k; ++len; }
    }
    if (start < 0) start = 0;
    slen[tid] = len;
  }
  __syncthreads();
  if (tid == 0) {
    int off = 0;
    for (int m = 0; m < NMEL; ++m) { soff[m] = off; off += slen[m]; }
  }
  __syncthreads();
  if (tid < NMEL) {
    int* ti = reinterpret_cast<int*>(tab);
    ti[T_MSTART + tid] = start;
    ti[T_MLEN + tid] = len;
    ti[T_MOFF + tid] = soff[tid];
    for (int i = 0; i < len && soff[tid] + i < MAXNZ; ++i) {
      const int k = start + i;
      tab[T_MW + soff[tid] + i] = (float)fmax(0.0, fmin((fk[k] - f0) / (f1 - f0), (f2 - fk[k]) / (f2 - f1)));
    }
  }
}

constexpr int FRAMES_PER_WAVE = 4;

__global__ __launch_bounds__(256) void fbank_logmel_kernel(const float* __restrict__ wav, int64_t ld_wav,
                                                         const int32_t* __restrict__ lengths, int Fmax,
                                                         const float* __restrict__ tab, float* __restrict__ work) {
  __shared__ float2 sbuf[4][NFFT];
  __shared__ float2 stw[NFFT / 2];
  __shared__ float swin[FRAME];
  __shared__ int sm_start[NMEL], sm_len[NMEL], sm_off[NMEL];
  __shared__ float sm_w[MAXNZ];
  __shared__ float spow[4][NBIN + 3];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = blockIdx.y;
  for (int k = tid; k < NFFT / 2; k += 256) stw[k] = make_float2(tab[T_TW + 2 * k], tab[T_TW + 2 * k + 1]);
  for (int n = tid; n < FRAME; n += 256) swin[n] = tab[T_WIN + n];
  if (tid < NMEL) {
    const int* ti = reinterpret_cast<const int*>(tab);
    sm_start[tid] = ti[T_MSTART + tid];
    sm_len[tid] = ti[T_MLEN + tid];
    sm_off[tid] = ti[T_MOFF + tid];
  }
  for (int i = tid; i < MAXNZ; i += 256) sm_w[i] = tab[T_MW + i];
  __syncthreads();

  const int len = lengths[b];
  const int F = len >= FRAME ? 1 + (len - FRAME) / HOP : 0;
  for (int fi = 0; fi < FRAMES_PER_WAVE; ++fi) {
  const int f = (blockIdx.x * 4 + w) * FRAMES_PER_WAVE + fi;
  if (f >= F || f >= Fmax) return;  // whole wave exits; no block barrier follows
  const float* x = wav + (int64_t)b * ld_wav + (int64_t)f * HOP;
  float v[7];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int n = lane + 64 * i;
    v[i] = n < FRAME ? x[n] * 32768.0f : 0.f;
    s += v[i];
  }
  const float mean = wave_sum(s) * (1.0f / FRAME);
  float2* buf = sbuf[w];
  // write (x - mean) to LDS, then pre-emphasis + window into bit-reversed complex slots
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int n = lane + 64 * i;
    if (n < FRAME) buf[n].x = v[i] - mean;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  float y[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int n = lane + 64 * i;
    float val = 0.f;
    if (n < FRAME) {
      const float cur = buf[n].x;
      val = (n == 0) ? cur * (1.0f - 0.97f) : cur - 0.97f * buf[n - 1].x;
      val *= swin[n];
    }
    y[i] = val;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int n = lane + 64 * i;
    const int rev = __builtin_bitreverse32((unsigned)n) >> (32 - 9);
    buf[rev] = make_float2(y[i], 0.f);
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  // iterative radix-2 DIT, 256 butterflies per stage, 4 per lane
#pragma unroll
  for (int half = 1; half < NFFT; half <<= 1) {
    const int tstride = (NFFT / 2) / half;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = lane + 64 * i;            // butterfly id 0..255
      const int grp = j / half, pos = j % half;
      const int i0 = grp * 2 * half + pos, i1 = i0 + half;
      const float2 tw = stw[pos * tstride];
      const float2 a = buf[i0], bb = buf[i1];
      const float2 t = make_float2(bb.x * tw.x - bb.y * tw.y, bb.x * tw.y + bb.y * tw.x);
      buf[i0] = make_float2(a.x + t.x, a.y + t.y);
      buf[i1] = make_float2(a.x - t.x, a.y - t.y);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
  }
  float* pw = spow[w];
  for (int k = lane; k < NBIN; k += 64) {
    const float2 z = buf[k];
    pw[k] = z.x * z.x + z.y * z.y;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  float* out = work + ((int64_t)b * Fmax + f) * NMEL;
  for (int m = lane; m < NMEL; m += 64) {
    const int st = sm_start[m], ln = sm_len[m], of = sm_off[m];
    float acc = 0.f;
    for (int i = 0; i < ln; ++i) acc += sm_w[of + i] * pw[st + i];
    out[m] = (float)log((double)fmaxf(acc, 1.192092955078125e-07f));  // float64 log, as numpy
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  }  // frames of this wave
}

// per-clip CMVN statistics: stats[b][m] = mean, stats[b][NMEL + m] = sqrt(var + 1e-7)
__global__ __launch_bounds__(128) void fbank_stats_kernel(const int32_t* __restrict__ lengths, int Fmax,
                                                        const float* __restrict__ work, float* __restrict__ stats) {
  const int b = blockIdx.x, m = threadIdx.x;
  if (m >= NMEL) return;
  const int len = lengths[b];
  const int F = len >= FRAME ? 1 + (len - FRAME) / HOP : 0;
  const float* x = work + (int64_t)b * Fmax * NMEL + m;
  // the sums must run frame by frame in order (numpy's rounding); loads go 48 frames ahead
  // (the chain is load-latency bound; vmcnt holds at most 63 loads in flight)
  constexpr int U = 48;
  float s = 0.f;
  for (int f0 = 0; f0 < F; f0 += U) {
    float v[U];
#pragma unroll
    for (int i = 0; i < U; ++i) v[i] = f0 + i < F ? x[(int64_t)(f0 + i) * NMEL] : 0.f;
#pragma unroll
    for (int i = 0; i < U; ++i) s = __fadd_rn(s, v[i]);   // + 0 past F: exact
  }
  const float mean = F > 0 ? __fdiv_rn(s, (float)F) : 0.f;
  float q = 0.f;
  for (int f0 = 0; f0 < F; f0 += U) {
    float v[U];
#pragma unroll
    for (int i = 0; i < U; ++i) v[i] = f0 + i < F ? x[(int64_t)(f0 + i) * NMEL] : mean;
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const float d = __fsub_rn(v[i], mean);
      if (f0 + i < F) q = __fadd_rn(q, __fmul_rn(d, d));
    }
  }
  const float var = F > 1 ? __fdiv_rn(q, (float)(F - 1)) : 0.f;
  stats[(int64_t)b * 2 * NMEL + m] = mean;
  stats[(int64_t)b * 2 * NMEL + NMEL + m] = __fsqrt_rn(__fadd_rn(var, 1e-7f));
}

constexpr int NORM_ROWS = 8;   // stacked rows per block of the normalise / stack kernel

__global__ __launch_bounds__(256) void fbank_norm_kernel(const int32_t* __restrict__ lengths, int Fmax, int Tmax,
                                                       const float* __restrict__ work,
                                                       const float* __restrict__ stats, float pad_value,
                                                       float* __restrict__ feats, int64_t* __restrict__ mask,
                                                       int mask_mode) {
  const int b = blockIdx.y, tid = threadIdx.x;
  const int len = lengths[b];
  const int F = len >= FRAME ? 1 + (len - FRAME) / HOP : 0;
  const int Tb = (F + 1) / 2;
  const float* x = work + (int64_t)b * Fmax * NMEL;
  const float* st = stats + (int64_t)b * 2 * NMEL;
  const int t0 = blockIdx.x * NORM_ROWS;
  float* o = feats + ((int64_t)b * Tmax + t0) * (2 * NMEL);
  for (int i = tid; i < NORM_ROWS * 2 * NMEL; i += 256) {
    const int t = t0 + i / (2 * NMEL), c = i % (2 * NMEL);
    if (t >= Tmax) break;
    const int f = 2 * t + (c >= NMEL), mm = c % NMEL;
    // beyond the clip: collate zero-padding (mode 0) or the extractor's batch padding value (mode 1)
    float val = mask_mode == 0 ? 0.f : pad_value;
    if (t < Tb) val = f < F ? __fdiv_rn(__fsub_rn(x[(int64_t)f * NMEL + mm], st[mm]), st[NMEL + mm]) : pad_value;
    o[i] = val;
  }
  if (tid < NORM_ROWS) {
    const int t = t0 + tid;
    if (t < Tmax) {
      int64_t mv;
      if (mask_mode == 0) mv = t < Tb ? 1 : 0;
      else mv = (t < Tb && 2 * t + 1 < F) ? 1 : 0;
      mask[(int64_t)b * Tmax + t] = mv;
    }
  }
}

// The constant tables (twiddles, window, mel filters) depend on nothing but the extractor's
// parameters: built once per device into module memory by a single-block launch, then shared by
// every call (the build runs serial fp64 loops: ~40 us that used to be paid per batch).
__device__ float g_fbank_tab[TABLE_FLOATS];

const float* fbank_tables(hipStream_t s) {
  static const float* tab[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!tab[dev]) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_fbank_tab)) != hipSuccess) return nullptr;
    hipLaunchKernelGGL(fbank_tables_kernel, dim3(1), dim3(256), 0, s, (float*)p);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(s) != hipSuccess) return nullptr;
    tab[dev] = (const float*)p;
  }
  return tab[dev];
}

}  // namespace

extern "C" int ste_fbank(const float* wav, int64_t ld_wav, const int32_t* lengths, int B, int Tmax, float pad_value,
                         float* feats, int64_t* mask, int mask_mode, float* work, void* stream) {
  if (B <= 0 || Tmax <= 0 || !wav || !lengths || !feats || !mask || !work) return STE_ERR_ARG;
  const int Fmax = 2 * Tmax;
  hipStream_t s = (hipStream_t)stream;
  const float* tab = fbank_tables(s);
  if (!tab) return STE_ERR_ARG;
  float* logmel = work + TABLE_FLOATS;
  const int fpb = 4 * FRAMES_PER_WAVE;
  hipLaunchKernelGGL(fbank_logmel_kernel, dim3((Fmax + fpb - 1) / fpb, B), dim3(256), 0, s, wav, ld_wav, lengths,
                     Fmax, tab, logmel);
  STE_CHECK_LAUNCH();
  float* stats = work + TABLE_FLOATS + (int64_t)B * Fmax * NMEL;
  hipLaunchKernelGGL(fbank_stats_kernel, dim3(B), dim3(128), 0, s, lengths, Fmax, logmel, stats);
  STE_CHECK_LAUNCH();
  hipLaunchKernelGGL(fbank_norm_kernel, dim3((Tmax + NORM_ROWS - 1) / NORM_ROWS, B), dim3(256), 0, s, lengths, Fmax,
                     Tmax, logmel, stats, pad_value, feats, mask, mask_mode);
  STE_CHECK_LAUNCH();
  return 0;
}

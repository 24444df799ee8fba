// Batched GPU fbank: the arithmetic of SeamlessM4TFeatureExtractor (w2v-bert-2.0's
// extractor) that the reference runs per clip on CPU DataLoader workers
// (ref:training/trainer_unfreeze.py:856-866 -> tf:models/seamless_m4t/
// feature_extraction_seamless_m4t.py:112-138,240-301, tf:audio_utils.py:809-1017),
// plus the collate padding of ref:training/trainer_unfreeze.py:880-921.
//
// Kernel 1 (one wavefront per 400-sample frame, 4 waves per block, 4 frames per wave):
//   x*2^15 -> remove frame mean -> pre-emphasis 0.97 (y0 *= 0.03) -> povey window
//   -> 512-point radix-8 Stockham FFT in registers (fp32, twiddles from double sincos) -> |X|^2
//   -> 80 kaldi-scale triangular mel filters built in mel space (sparse, per-block
//   table) -> max(1.1920929e-7, .) -> natural log.
// Kernel 2 (one block per clip and group of NB mel bins, the group's columns staged into LDS):
// per-mel-bin mean and unbiased variance over the clip's frames exactly as numpy evaluates them
// on the extractor's float32 log-mel array (tf:…seamless_m4t…:256-261: x.mean(0), x.var(0, ddof=1),
// (x - mean)/sqrt(var + 1e-7)): float32 sums accumulated frame by frame in order (numpy's
// reduction over a non-contiguous axis), IEEE float32 division and square root.  A bin whose
// frames are all equal (silence at the log floor) therefore reproduces the reference's non-zero
// rounding residue bit for bit.  The same block then writes (x - mean)/std for its bins, pads odd
// frame counts with padding_value, stacks frame pairs into 160-d rows, zeroes rows beyond the clip
// and (bin group 0) writes the mask.  Clips too long for the LDS columns take the separate
// statistics (kernel 2b) and normalise / stack (kernel 3) kernels.
// HBM-bound: 4 B/sample in, 640 B per stacked frame + mask out.
#include "common.h"
#include "../../include/ste.h"

namespace {

constexpr int FRAME = 400, HOP = 160, NFFT = 512, NBIN = 257, NMEL = 80;
constexpr int MAXNZ = 640;  // non-zero filter taps (501 for these parameters)
constexpr float MEL_FLOOR = 1.192092955078125e-07f;   // tf:audio_utils.py mel_floor (float32 eps)
constexpr float LOG_MEL_FLOOR = -15.942384719848633f; // (float)log((double)MEL_FLOOR), exactly

// Constant tables, compile-time data (fbank_tables.h, made by gen_fbank_tables.py from the
// extractor's float64 formulas, rounded to float32 once), read by every frame block:
//   [0, 512)   twiddles e^{-2πik/512} (float2 x 256)     [512, 912)  povey window
//   [912, 992) mel start bin  [992, 1072) mel length  [1072, 1152) mel offset (ints)
//   [1152, 1152+MAXNZ) mel weights (kaldi scale, triangles in mel space)
// No device state is built at run time: ste_fbank is re-entrant and graph-capturable.
constexpr int T_TW = 0, T_WIN = 512, T_MSTART = 912, T_MLEN = 992, T_MOFF = 1072, T_MW = 1152;
}  // namespace
#include "fbank_tables.h"
namespace {

constexpr int FRAMES_PER_WAVE = 4;
constexpr int XPAD = NFFT + NFFT / 8;   // exchange buffer: one float2 of padding per 8

STE_DEV int xpad(int i) { return i + (i >> 3); }
STE_DEV float2 cmul(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
STE_DEV float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
STE_DEV float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }

// In-register 8-point DFT, natural order in and out (decimation in frequency: one radix-2 layer
// with W8 twiddles, then two 4-point DFTs giving the even and the odd outputs).
STE_DEV void dft8(float2 (&v)[8]) {
  constexpr float C = 0.70710678118654752f;
  float2 a[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) { a[k] = cadd(v[k], v[k + 4]); a[k + 4] = csub(v[k], v[k + 4]); }
  a[5] = make_float2(C * (a[5].x + a[5].y), C * (a[5].y - a[5].x));     // * W8^1
  a[6] = make_float2(a[6].y, -a[6].x);                                  // * W8^2 = -i
  a[7] = make_float2(C * (a[7].y - a[7].x), -C * (a[7].x + a[7].y));    // * W8^3
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float2 b0 = cadd(a[4 * h], a[4 * h + 2]), b2 = csub(a[4 * h], a[4 * h + 2]);
    const float2 b1 = cadd(a[4 * h + 1], a[4 * h + 3]), d = csub(a[4 * h + 1], a[4 * h + 3]);
    const float2 b3 = make_float2(d.y, -d.x);                           // * -i
    v[h] = cadd(b0, b1);          // X[2k + h], k = 0..3
    v[2 + h] = cadd(b2, b3);
    v[4 + h] = csub(b0, b1);
    v[6 + h] = csub(b2, b3);
  }
}

// Frame -> 80 log-mel energies.  The 512-point FFT is a radix-8 Stockham transform held in
// registers (lane j owns points j + 64 r): three passes of dft8, two exchanges through a padded
// per-wave LDS buffer, twiddles e^{-2πik/512} from the fp64-built table; the input needs no
// bit reversal and lane j ends with X[j + 64 r].  (The radix-2 version took 9 LDS round trips
// per frame and half of the kernel's time.)
__global__ __launch_bounds__(256) void fbank_logmel_kernel(const float* __restrict__ wav, int64_t ld_wav,
                                                         const int32_t* __restrict__ lengths, int Fmax,
                                                         float* __restrict__ work) {
  const float* tab = reinterpret_cast<const float*>(g_fbank_tab_bits);
  __shared__ float2 sbuf[4][XPAD];
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
  float2* buf = sbuf[w];
  for (int fi = 0; fi < FRAMES_PER_WAVE; ++fi) {
  const int f = (blockIdx.x * 4 + w) * FRAMES_PER_WAVE + fi;
  if (f >= F || f >= Fmax) return;  // whole wave exits; no block barrier follows
  const float* x = wav + (int64_t)b * ld_wav + (int64_t)f * HOP;
  float c[7];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int n = lane + 64 * i;
    c[i] = n < FRAME ? x[n] * 32768.0f : 0.f;
    s += c[i];
  }
  const float mean = wave_sum(s) * (1.0f / FRAME);
#pragma unroll
  for (int i = 0; i < 7; ++i) c[i] = c[i] - mean;   // n >= FRAME: masked below
  // pre-emphasis (x[n] - 0.97 x[n-1], x[0] * 0.03) and window: x[n-1] is lane-1's value, or
  // lane 63's of the previous row for lane 0
  float2 v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int n = lane + 64 * i;
    float val = 0.f;
    if (i < 7) {
      // lane - 1's value by DPP wave_shr:1 and lane 63's by v_readlane (no ds_bpermute round trips)
      const float up = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, c[i]), 0x138,
                                                                               0xF, 0xF, false));
      const float wrap = i > 0 ? __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, c[i - 1]), 63))
                               : 0.f;
      const float prev = lane > 0 ? up : wrap;
      if (n < FRAME) {
        val = (n == 0) ? c[i] * (1.0f - 0.97f) : c[i] - 0.97f * prev;
        val *= swin[n];
      }
    }
    v[i] = make_float2(val, 0.f);
  }
  // Stockham radix-8: pass Ns in {1, 8, 64}; lane j reads points j + 64 r, twiddles by
  // W512^(r (j mod Ns) 64/Ns), runs dft8 and writes (j/Ns) Ns 8 + (j mod Ns) + r Ns
#pragma unroll
  for (int pass = 0; pass < 3; ++pass) {
    const int Ns = pass == 0 ? 1 : pass == 1 ? 8 : 64;
    if (pass > 0) {
      const int jm = lane & (Ns - 1), step = jm * (64 / Ns);
#pragma unroll
      for (int r = 1; r < 8; ++r) {
        const int k = r * step;                       // < 512
        float2 tw = stw[k & 255];
        if (k & 256) tw = make_float2(-tw.x, -tw.y);
        v[r] = cmul(v[r], tw);
      }
    }
    dft8(v);
    if (pass < 2) {
      const int base = (lane / Ns) * Ns * 8 + (lane & (Ns - 1));
#pragma unroll
      for (int r = 0; r < 8; ++r) buf[xpad(base + r * Ns)] = v[r];
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = buf[xpad(lane + 64 * r)];
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
  }
  // lane j holds X[j + 64 r]: power of bins 0..256
  float* pw = spow[w];
#pragma unroll
  for (int r = 0; r < 5; ++r) {
    const int k = lane + 64 * r;
    if (k < NBIN) pw[k] = v[r].x * v[r].x + v[r].y * v[r].y;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  float* out = work + ((int64_t)b * Fmax + f) * NMEL;
  for (int m = lane; m < NMEL; m += 64) {
    const int st = sm_start[m], ln = sm_len[m], of = sm_off[m];
    float acc = 0.f;
    for (int i = 0; i < ln; ++i) acc += sm_w[of + i] * pw[st + i];
    // the reference logs the float64 mel energies and rounds to float32 (np.log(...).astype(float32)):
    // the float64 log rounded once, as there (one scalar per mel bin per frame: cheap here).  At the
    // floor (silent frames) that exact constant matters most: a clip's identical rows leave numpy's
    // CMVN rounding residue in the output
    out[m] = acc > MEL_FLOOR ? (float)log((double)acc) : LOG_MEL_FLOOR;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  }  // frames of this wave
}

// per-clip CMVN statistics: stats[b][m] = mean, stats[b][NMEL + m] = sqrt(var + 1e-7)
// The sums must run frame by frame in order (numpy's rounding), so one thread per mel bin owns
// each chain; the block's 1024 threads stage the clip's log-mel rows through LDS in chunks of
// STATS_CH frames with all of a chunk's loads in flight at once, and the next chunk's loads are
// issued into registers before the 80 chains walk the current one.
constexpr int STATS_NT = 1024, STATS_CH = 128, STATS_PER = STATS_CH * NMEL / STATS_NT;   // 10
__global__ __launch_bounds__(STATS_NT) void fbank_stats_kernel(const int32_t* __restrict__ lengths, int Fmax,
                                                             const float* __restrict__ work,
                                                             float* __restrict__ stats) {
  __shared__ float sx[2][STATS_CH * NMEL];   // 80 KB
  const int b = blockIdx.x, tid = threadIdx.x;
  const int len = lengths[b];
  const int F = len >= FRAME ? 1 + (len - FRAME) / HOP : 0;
  const float* x = work + (int64_t)b * Fmax * NMEL;
  const int nch = (F + STATS_CH - 1) / STATS_CH;
  float s = 0.f, q = 0.f, mean = 0.f;
  float r[STATS_PER];
  auto fetch = [&](int c) {   // chunk c (of the 2 * nch chunk visits) -> registers
    const int f0 = (c % nch) * STATS_CH, n = min(STATS_CH, F - f0) * NMEL;
#pragma unroll
    for (int i = 0; i < STATS_PER; ++i) {
      const int e = tid + i * STATS_NT;
      r[i] = e < n ? x[(int64_t)f0 * NMEL + e] : 0.f;
    }
  };
  if (nch > 0) fetch(0);
  for (int c = 0; c < 2 * nch; ++c) {
    float* buf = sx[c & 1];
#pragma unroll
    for (int i = 0; i < STATS_PER; ++i) buf[tid + i * STATS_NT] = r[i];
    __syncthreads();
    if (c + 1 < 2 * nch) fetch(c + 1);
    if (tid < NMEL) {
      const int f0 = (c % nch) * STATS_CH, nf = min(STATS_CH, F - f0);
      if (c < nch) {
        for (int i = 0; i < nf; ++i) s = __fadd_rn(s, buf[i * NMEL + tid]);
        if (c == nch - 1) mean = __fdiv_rn(s, (float)F);
      } else {
        for (int i = 0; i < nf; ++i) {
          const float d = __fsub_rn(buf[i * NMEL + tid], mean);
          q = __fadd_rn(q, __fmul_rn(d, d));
        }
      }
    }
  }
  if (tid < NMEL) {
    const float var = F > 1 ? __fdiv_rn(q, (float)(F - 1)) : 0.f;
    stats[(int64_t)b * 2 * NMEL + tid] = mean;
    stats[(int64_t)b * 2 * NMEL + NMEL + tid] = __fsqrt_rn(__fadd_rn(var, 1e-7f));
  }
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

// CMVN statistics and the normalise / stack / pad / mask step in one kernel, for a group of NB mel
// bins of one clip per block (NB·B blocks instead of B): the group's log-mel columns are staged
// whole into LDS, transposed (bin-major, so a chain reads 4 frames per ds_read_b128), the NB
// statistics chains run exactly as fbank_stats_kernel's (frame-ordered float32 sums, IEEE
// division and square root: numpy's rounding), and the block then writes its bins' columns of
// every stacked row from LDS.  The block of bin group 0 also writes the mask.  Used when
// NB · Fp · 4 B fits the 64 KB of LDS (NB = 16 up to 10 s clips, NB = 4 up to 40 s); longer
// clips take fbank_stats_kernel + fbank_norm_kernel.
constexpr int SN_NT = 256;
template <int NB>
__global__ __launch_bounds__(SN_NT) void fbank_stats_norm_kernel(const int32_t* __restrict__ lengths, int Fmax, int Fp,
                                                                int Tmax, const float* __restrict__ work,
                                                                float* __restrict__ stats, float pad_value,
                                                                float* __restrict__ feats, int64_t* __restrict__ mask,
                                                                int mask_mode) {
  extern __shared__ float4 sn_lds4[];
  float* col = reinterpret_cast<float*>(sn_lds4);   // [NB][Fp]
  __shared__ float s_mean[NB], s_std[NB];
  const int b = blockIdx.y, m0 = blockIdx.x * NB, tid = threadIdx.x;
  const int len = lengths[b];
  const int F = min(len >= FRAME ? 1 + (len - FRAME) / HOP : 0, Fmax);
  const int Tb = (F + 1) / 2;
  const float* x = work + (int64_t)b * Fmax * NMEL + m0;
  // stage: lane (f, j) reads bin m0 + j of frame f (NB-float runs of a 320-B row), writes col[j][f]
#pragma unroll 16
  for (int e = tid; e < F * NB; e += SN_NT) {
    const int f = e / NB, j = e % NB;
    col[j * Fp + f] = x[(int64_t)f * NMEL + j];
  }
  __syncthreads();
  if (tid < NB) {
    // one chain per bin, frame by frame, 4 frames per ds_read_b128
    const float* c = col + tid * Fp;
    const float4* c4 = reinterpret_cast<const float4*>(c);
    const int F4 = F & ~3;
    float sum = 0.f;
#pragma unroll 4
    for (int f = 0; f < F4; f += 4) {
      const float4 v = c4[f >> 2];
      sum = __fadd_rn(__fadd_rn(__fadd_rn(__fadd_rn(sum, v.x), v.y), v.z), v.w);
    }
    for (int f = F4; f < F; ++f) sum = __fadd_rn(sum, c[f]);
    const float mean = F > 0 ? __fdiv_rn(sum, (float)F) : 0.f;
    float q = 0.f;
    auto sq = [&](float a) {
      const float d = __fsub_rn(a, mean);
      q = __fadd_rn(q, __fmul_rn(d, d));
    };
#pragma unroll 4
    for (int f = 0; f < F4; f += 4) {
      const float4 v = c4[f >> 2];
      sq(v.x);
      sq(v.y);
      sq(v.z);
      sq(v.w);
    }
    for (int f = F4; f < F; ++f) sq(c[f]);
    const float var = F > 1 ? __fdiv_rn(q, (float)(F - 1)) : 0.f;
    const float sd = __fsqrt_rn(__fadd_rn(var, 1e-7f));
    s_mean[tid] = mean;
    s_std[tid] = sd;
    stats[(int64_t)b * 2 * NMEL + m0 + tid] = mean;
    stats[(int64_t)b * 2 * NMEL + NMEL + m0 + tid] = sd;
  }
  __syncthreads();
  // stacked row t = [frame 2t | frame 2t + 1]: this block's columns m0 + j of both halves
  float* o = feats + (int64_t)b * Tmax * (2 * NMEL) + m0;
  const float fill = mask_mode == 0 ? 0.f : pad_value;
  auto value = [&](int t, int h, int j) {
    const int f = 2 * t + h;
    // beyond the clip: collate zero-padding (mode 0) or the extractor's batch padding value (mode 1)
    if (t >= Tb) return fill;
    return f < F ? __fdiv_rn(__fsub_rn(col[j * Fp + f], s_mean[j]), s_std[j]) : pad_value;
  };
#pragma unroll 4
  for (int e = tid; e < Tmax * 2 * NB; e += SN_NT) {
    const int t = e / (2 * NB), r = e % (2 * NB), h = r / NB, j = r % NB;
    o[(int64_t)t * (2 * NMEL) + h * NMEL + j] = value(t, h, j);
  }
  if (blockIdx.x == 0) {
    for (int t = tid; t < Tmax; t += SN_NT) {
      int64_t mv;
      if (mask_mode == 0) mv = t < Tb ? 1 : 0;
      else mv = (t < Tb && 2 * t + 1 < F) ? 1 : 0;
      mask[(int64_t)b * Tmax + t] = mv;
    }
  }
}

template <int NB>
void launch_stats_norm(int B, int Fmax, int Fp, int Tmax, const int32_t* lengths, const float* work, float* stats,
                       float pad_value, float* feats, int64_t* mask, int mask_mode, hipStream_t s) {
  hipLaunchKernelGGL(fbank_stats_norm_kernel<NB>, dim3(NMEL / NB, B), dim3(SN_NT), (size_t)NB * Fp * 4, s,
                     lengths, Fmax, Fp, Tmax, work, stats, pad_value, feats, mask, mask_mode);
}

bool stats_norm(int B, int Fmax, int Tmax, const int32_t* lengths, const float* work, float* stats, float pad_value,
                float* feats, int64_t* mask, int mask_mode, hipStream_t s) {
  // the largest bin group whose columns fit 64 KB of LDS (with the static mean / std rows)
  const int Fp = (Fmax + 3) & ~3;
  const int64_t col_bytes = (int64_t)Fp * 4, lds = 65536 - 256;
  if (16 * col_bytes <= lds)
    launch_stats_norm<16>(B, Fmax, Fp, Tmax, lengths, work, stats, pad_value, feats, mask, mask_mode, s);
  else if (8 * col_bytes <= lds)
    launch_stats_norm<8>(B, Fmax, Fp, Tmax, lengths, work, stats, pad_value, feats, mask, mask_mode, s);
  else if (4 * col_bytes <= lds)
    launch_stats_norm<4>(B, Fmax, Fp, Tmax, lengths, work, stats, pad_value, feats, mask, mask_mode, s);
  else if (2 * col_bytes <= lds)
    launch_stats_norm<2>(B, Fmax, Fp, Tmax, lengths, work, stats, pad_value, feats, mask, mask_mode, s);
  else
    return false;
  return true;
}

}  // namespace

extern "C" int ste_fbank(const float* wav, int64_t ld_wav, const int32_t* lengths, int B, int Tmax, float pad_value,
                         float* feats, int64_t* mask, int mask_mode, float* work, void* stream) {
  if (B <= 0 || Tmax <= 0 || !wav || !lengths || !feats || !mask || !work) return STE_ERR_ARG;
  const int Fmax = 2 * Tmax;
  hipStream_t s = (hipStream_t)stream;
  float* logmel = work;
  const int fpb = 4 * FRAMES_PER_WAVE;
  hipLaunchKernelGGL(fbank_logmel_kernel, dim3((Fmax + fpb - 1) / fpb, B), dim3(256), 0, s, wav, ld_wav, lengths,
                     Fmax, logmel);
  STE_CHECK_LAUNCH();
  float* stats = work + (int64_t)B * Fmax * NMEL;
  // fused statistics + normalise; A/B builds: STE_FBANK_SN=old takes the separate kernels
  const char* e = STE_AB_ENV("STE_FBANK_SN");
  const bool fused = !(e && e[0] == 'o') &&
                     stats_norm(B, Fmax, Tmax, lengths, logmel, stats, pad_value, feats, mask, mask_mode, s);
  if (!fused) {
    hipLaunchKernelGGL(fbank_stats_kernel, dim3(B), dim3(STATS_NT), 0, s, lengths, Fmax, logmel, stats);
    STE_CHECK_LAUNCH();
    hipLaunchKernelGGL(fbank_norm_kernel, dim3((Tmax + NORM_ROWS - 1) / NORM_ROWS, B), dim3(256), 0, s, lengths, Fmax,
                       Tmax, logmel, stats, pad_value, feats, mask, mask_mode);
  }
  STE_CHECK_LAUNCH();
  return 0;
}

/*
 * ste.h — C ABI of libste.so, the MI355X (gfx950) kernels behind the
 * speech<->transcript contrastive training step.
 *
 * Every entry point takes plain device pointers, sizes and a hipStream_t (passed
 * as void*), enqueues work on that stream and returns 0 or a ste/hip error code.
 * Nothing here allocates, frees or synchronises, so every call is hipGraph
 * capturable.  Inputs are borrowed; outputs are caller-allocated.
 *
 * Each declaration cites the reference interface it replaces.  "tf:" paths are
 * relative to transformers/ (the reference pins transformers 4.50.2, uv.lock:1813);
 * "ref:" paths are relative to /root/reference.
 */
#ifndef STE_H_
#define STE_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define STE_OK 0
#define STE_ERR_ARG 1001
#define STE_ERR_SHAPE 1002

/* ------------------------------------------------------------------ GEMM --
 * Replaces nn.Linear / kernel-size-1 nn.Conv1d forward and both backward
 * products: tf:models/wav2vec2_bert/modeling_wav2vec2_bert.py:119-226,229-337,
 * tf:models/xlm_roberta/modeling_xlm_roberta.py:186-398,
 * ref:training/trainer_unfreeze.py:66-310 (projection / attention / fusion heads).
 *
 * C = epilogue(alpha * A.B), bf16 operands, fp32 accumulation.
 *   a_kc=1: A[m*lda+k]   a_kc=0: A[k*lda+m]
 *   b_kc=1: B[n*ldb+k]   b_kc=0: B[k*ldb+n]
 * Epilogue, in order: v = alpha*(acc + bias[n]);
 *   act in {SWISH,GELU,TANH,RELU}: C2 <- v (bf16, pre-activation, optional); v = act(v)
 *   act in {*_BWD}: v *= act'(Z[m,n])           (Z: bf16, row stride ldz)
 *   drop_p>0: v *= keep(seed, m*drop_ld+n)/(1-drop_p)
 *   row_scale: v *= row_scale[m]
 *   colsum: colsum[n] += v                      (bias gradients; see below)
 *   R: v += R[m,n]                              (fp32, or bf16 if r_bf16)
 *   beta != 0: v += beta*C[m,n]
 *   C <- v (fp32, or bf16 if c_bf16);  C3 <- bf16(v) (optional)
 * Contract: KC operands need K%8==0 and ld%8==0; KM operands need (M or N)%8==0
 * and ld%8==0; for N >= 8, C, C2, C3, R, Z and bias start 16-B aligned with
 * 16-B-multiple row strides (the epilogue moves 8 columns per lane).  Any N (ragged
 * last columns are handled element-wise).
 * Weight gradients (a_kc=0, b_kc=0: dW = dYᵀ·X over K = batch·time rows, plain
 * epilogue alpha/beta only): given a workspace ws (fp32, ws_bytes), a shape whose
 * 256x256 tiles cannot fill the chip is split along K into S slabs
 * (S·M·N·4 <= ws_bytes), each reduced by one 256x256 MFMA workgroup, then
 * C = beta·C + alpha·Σ slabs.  ws may be NULL (no split).
 * Column sums are run-to-run deterministic when ws holds at least
 * ste_gemm_colsum_ws_floats(args) floats: each wave writes its rows' partial sums there
 * and ste_rowsum_ordered adds them in a fixed order (colsum launches are never split, so
 * ws is free for them); without such a ws they go through fp32 atomics.
 * Narrow outputs (a_kc=1, b_kc=1, batch 1, no colsum, N%8==0, K%64==0 with >= 40
 * K-tiles, at most CUs/2 tiles of 256x256, 2·M·N·4 <= ws_bytes): given ws, the
 * product runs as 2 K-slabs and a reduction that applies the full epilogue (same
 * results and dropout mask as without ws, up to fp32 summation order).
 */
enum {
  STE_ACT_NONE = 0,
  STE_ACT_SWISH = 1,
  STE_ACT_GELU = 2,
  STE_ACT_TANH = 3,
  STE_ACT_RELU = 4,
  STE_ACT_SWISH_BWD = 11,
  STE_ACT_GELU_BWD = 12,
  STE_ACT_TANH_BWD_OUT = 13,
  STE_ACT_RELU_BWD = 14
};

typedef struct {
  int M, N, K, batch;
  const void* A; int64_t lda; int a_kc;
  const void* B; int64_t ldb; int b_kc;
  int64_t strideA, strideB, strideC, strideR;
  void* C; int64_t ldc; int c_bf16;
  void* C2; int64_t ldc2;
  void* C3; int64_t ldc3;
  const float* bias;
  const void* R; int64_t ldr; int r_bf16;
  const void* Z; int64_t ldz;
  float* colsum;
  const float* row_scale;
  float alpha, beta;
  int act;
  float drop_p; uint64_t seed; int64_t drop_ld;
  float* ws; int64_t ws_bytes;      /* split-K workspace: weight gradients, narrow outputs (optional) */
  int c3_lo;                        /* C3 <- bf16(v - bf16(v)), the low half, instead of bf16(v):
                                       with C = bf16(v) the two make the [hi | lo] split image the
                                       next precise-forward GEMM reads (see ste_split_bf16) */
} ste_gemm_args;

int ste_gemm(const ste_gemm_args* args, void* stream);
/* Workspace floats for deterministic column sums of this launch (0 without colsum): an upper
 * bound over ste_gemm and ste_gemm_f32's tile shapes. */
int64_t ste_gemm_colsum_ws_floats(const ste_gemm_args* args);
/* Host-only (never touches the GPU): the output tile (tm, tn) that the GEMM kernels give tile id
 * t (after their XCD remap) of a num_m x num_n tile grid — groups of 8 m-tiles, m fastest within a
 * group.  For tests of the order. */
int ste_gemm_tile_map(int t, int num_m, int num_n, int* tm, int* tn);

/* The same contract with fp32 A, B (and fp32 C2 / Z) on the exact-f32 matrix core
 * (v_mfma_f32_16x16x4_f32): the projection, cross-attention query / output, fusion and text
 * pooling-scorer Linears of the heads (ref:training/trainer_unfreeze.py:66-99,125-168,171-211,
 * 470-477), computed in fp32 as the reference does.  KC operands need K % 4 == 0 and
 * ld % 4 == 0, KM operands (M or N) % 4 == 0; A, B 16-B aligned; batch 1.  A weight gradient
 * (plain epilogue, fp32 C) with K >= 1024 whose tiles cannot fill the chip is split along K
 * into slabs of ws (when given) summed in slab order. */
int ste_gemm_f32(const ste_gemm_args* args, void* stream);

/* Which kernel ste_gemm would launch for these args (no launch, host-only):
 * STE_GEMM_KERNEL_SMALL/BIG/8PH + variant, variant = (a_kc ? 0 : 2) + (b_kc ? 0 : 1).
 * Lets profilers and bench.py attribute per-launch time to the rocprof kernel name. */
#define STE_GEMM_KERNEL_SMALL 0
#define STE_GEMM_KERNEL_BIG 4
#define STE_GEMM_KERNEL_8PH 8
#define STE_GEMM_KERNEL_SPLITK 12
int ste_gemm_kernel(const ste_gemm_args* args);
/* The rocprofv3 kernel name (template arguments included) of that launch, NUL-terminated
 * into buf[len]; bench.py keys its HIP-event timings and PMC traffic by it. */
int ste_gemm_kernel_name(const ste_gemm_args* args, char* buf, int len);

/* MX-fp8 forward GEMM (BASELINE config 5, "fp8 MFMA GEMMs"): the nn.Linear forwards of the
 * Conformer layers (tf:…wav2vec2_bert…:134-154 FFN, :229-337 q/k/v/o, :157-226 pointwise convs)
 * with both operands in OCP e4m3 and one E8M0 scale per 32 consecutive k of a row (OCP MX
 * block scaling), on v_mfma_scale_f32_16x16x128_f8f6f4.  args as for ste_gemm with a_kc =
 * b_kc = 1 and A/B pointing at e4m3 bytes (lda/ldb in bytes, multiples of 16, K % 128 == 0,
 * batch 1, no split-K); a_scales [M][K/32], b_scales [N][K/32] bytes.  Every epilogue option
 * of ste_gemm applies to the fp32 accumulators unchanged.  q_out/q_scales (optional, N % 128
 * == 0): the final values also leave MX-fp8 quantised ([M][N] e4m3, [M][N/32] E8M0), the input
 * of the next MX-fp8 GEMM; args->C may then be NULL (no bf16/fp32 copy). */
int ste_gemm_mx8(const ste_gemm_args* args, const void* a_scales, const void* b_scales, void* q_out, void* q_scales,
                 void* stream);
/* Host-only plan query of ste_gemm_mx8 (no launch): 1 = the persistent 8-phase MX kernel
 * (>= 240 output tiles, a compile-time epilogue, each operand's fp8 bytes M·lda and N·ldb below
 * 4 GiB because its DMA sources are 32-bit offsets), 0 = the single-stage kernel (64-bit
 * addressing, any shape).  q_out: whether an MX-fp8 output copy is requested. */
int ste_gemm_mx8_kernel(const ste_gemm_args* args, int q_out);
/* Plan thresholds (process-wide, host-only): the fewest 256x256 output tiles for which ste_gemm
 * plans the persistent 8-phase bf16 kernel and ste_gemm_mx8 the 8-phase MX one (both 240 by
 * default: about one wave of 256 CUs).  A value <= 0 leaves that threshold unchanged; the previous
 * values are returned through prev_bf16 / prev_mx8 (either may be NULL).  Parity tests lower them
 * so that a B <= 4 batch runs the same kernel instantiations as the b = 64 bench step; the planned
 * kernels accept any tile count (partial edge tiles take their guarded epilogue). */
int ste_gemm_plan_min_tiles(int bf16_tiles, int mx8_tiles, int* prev_bf16, int* prev_mx8);
/* bf16 x [rows][K] (row stride ldx) -> e4m3 q [rows][K] and E8M0 scales [rows][K/32]:
 * scale 2^e, e = ceil(log2(amax/448)) per 32-element block (no saturation; zero blocks 2^-127). */
int ste_mx8_quant(const void* x, int64_t ldx, int rows, int K, void* q, void* scales, void* stream);

/* ------------------------------------------------------------- LayerNorm --
 * Replaces nn.LayerNorm forward/backward (every LN of both encoders and the
 * heads: tf:…wav2vec2_bert…:122,169,181,381-394; tf:…xlm_roberta…:64,333,389;
 * ref:training/trainer_unfreeze.py:97,475,477,244).
 * Row-wise over `cols`; fp32 statistics saved as mean/rstd [rows].
 * Forward options: row_scale (multiply output rows, e.g. the conformer conv
 * module's masked_fill, tf:…wav2vec2_bert…:194-196), post-activation (swish:
 * conv module's depthwise LN + activation, :209-211), fp32 and/or bf16 outputs,
 * dropout on the output (XLM-R embeddings, tf:…xlm_roberta…:119-120).
 */
typedef struct {
  int rows, cols;
  const void* x; int64_t ldx; int x_bf16;
  const float* gamma; const float* beta; float eps;
  float* y; int64_t ldy;            /* fp32 output (optional) */
  void* yb; int64_t ldyb;           /* bf16 output (optional) */
  float* mean; float* rstd;         /* saved statistics (required) */
  const float* row_scale;           /* optional */
  int act;                          /* STE_ACT_NONE or STE_ACT_SWISH */
  float drop_p; uint64_t seed;      /* dropout on the output (index row*cols+col) */
  void* q8; void* q8s; int64_t ldq8; /* MX-fp8 output (optional, cols % 128 == 0): e4m3 [rows][ldq8]
                                        + E8M0 [rows][cols/32], the input of ste_gemm_mx8 */
  void* ylo; int64_t ldylo;         /* bf16 low half bf16(y - bf16(y)) (optional): with yb, the
                                       [hi | lo] split image of y (see ste_split_bf16) */
} ste_ln_fwd_args;
int ste_layernorm_fwd(const ste_ln_fwd_args* a, void* stream);

/* Backward: g = dy (fp32 or bf16; times row_scale; through swish' if act==SWISH,
 * recomputing the pre-activation from x/mean/rstd), dx = LN'(g) (+ dres),
 * dgamma/dbeta/dsum += column sums (optional).  Outputs: dx fp32 (optional),
 * dxb = bf16(dx * dropmask(drop_seed) * out_scale) (optional).
 * Column sums: with a workspace (ws, >= ste_layernorm_bwd_ws_floats(rows, cols) floats, ws_floats
 * its size) every block writes its partials there and a second launch adds them in a fixed
 * order — run-to-run deterministic, no same-address atomics; ws = NULL: fp32 atomics.
 * With a workspace the final add is a plain read-modify-write: dgamma, dbeta and dsum must not
 * alias each other, and no other launch may accumulate into them concurrently (one stream at a
 * time); a workspace may be reused by later launches on the same stream, not shared across
 * streams (nor between the two LayerNorms of a pair call). */
typedef struct {
  int rows, cols;
  const void* dy; int64_t lddy; int dy_bf16;
  const void* x; int64_t ldx; int x_bf16;
  const float* mean; const float* rstd;
  const float* gamma; const float* beta;
  const float* row_scale;
  int act;
  const float* dres; int64_t lddres;
  float* dx; int64_t lddx;
  void* dxb; int64_t lddxb;
  float* dgamma; float* dbeta;
  float drop_p; uint64_t seed; float out_scale;   /* dropout/scale applied to the dxb copy only */
  float in_drop_p; uint64_t in_seed;              /* forward output dropout to undo on dy */
  const float* out_row_scale;                     /* multiplies the dxb copy rows (optional) */
  float* dsum;                                    /* += column sums of the dxb values (fp32, optional):
                                                     the bias gradient of the Linear feeding this residual */
  float* ws; int64_t ws_floats;                   /* column-partial workspace (optional, see above) */
} ste_ln_bwd_args;
int ste_layernorm_bwd(const ste_ln_bwd_args* a, void* stream);
/* workspace floats ste_layernorm_bwd / _bwd_pair need for deterministic column sums */
int64_t ste_layernorm_bwd_ws_floats(int rows, int cols);

/* Two chained LayerNorms in one pass over the rows (a Conformer layer's final_layer_norm and
 * the next layer's ffn1_layer_norm, tf:…wav2vec2_bert…:381-394, 359-362): forward
 * y2 = LN_b(LN_a(x)) with LN_a's output (which a must also write, a->y) kept in registers for
 * LN_b (b->x is not read); backward in reverse: b's input gradient, in registers, is a's dy
 * (a->dy is not read; b->dx optional).  cols <= 1024; every other option per LN as above. */
int ste_layernorm_fwd_pair(const ste_ln_fwd_args* a, const ste_ln_fwd_args* b, void* stream);
int ste_layernorm_bwd_pair(const ste_ln_bwd_args* a, const ste_ln_bwd_args* b, void* stream);

/* ------------------------------------------------------------- Attention --
 * Multi-head self-attention core, softmax(QKᵀ·scale + relbias + mask)·V, fused
 * (scores never reach HBM).  Replaces:
 *   audio: Wav2Vec2BertSelfAttention relative_key path,
 *          tf:…wav2vec2_bert…:285-327 (bias[l,r] = q_l·E[clamp(r-l,-left,right)+left]·scale)
 *   text:  XLM-R SDPA attention with key-padding mask and probs dropout,
 *          tf:…xlm_roberta…:186-250.
 * q/k/v/o are bf16 [B*T, *] with row strides ldq/ldk/ldv/ldo; head h uses
 * columns h*64..h*64+63 (head_dim fixed at 64).  key_mask [B*T] (nonzero = valid)
 * may be NULL.  rel_E [left+right+1, 64] bf16 may be NULL (no relative bias); windows of up to
 * 80 bins (left + right + 1 <= 80; STE_ERR_SHAPE beyond).
 * lse [B*H*T] fp32 is saved for backward.
 */
typedef struct {
  int B, T, H;
  const void* q; int64_t ldq;
  const void* k; int64_t ldk;
  const void* v; int64_t ldv;
  void* o; int64_t ldo;
  float* lse;
  const int32_t* key_mask;
  const void* rel_E; int rel_left, rel_right;
  float scale;
  float drop_p; uint64_t seed;
  /* backward */
  const void* dout; int64_t lddo;
  void* dq; int64_t lddq;
  void* dk; int64_t lddk;
  void* dv; int64_t lddv;
  float* delta;       /* workspace [B*H*T] */
  float* dE;          /* fp32 [left+right+1, 64], accumulated in a fixed order (may be NULL) */
  float* gwork;       /* workspace [B*H*T*80] fp32, required when dE != NULL */
  /* optional low half of O (bf16, row stride ldolo): the forward (whose PV product runs on
   * P split into bf16 hi + lo halves, so O is ~fp32-accurate) writes bf16(O - bf16(O)), and
   * the backward forms delta = rowsum(dO·(O + O_lo)) from it, i.e. from the ~fp32 output.
   * With near-uniform attention O ≈ mean(V) and dS = P(dP - delta) is a small difference of
   * large terms, so a delta from the bf16-rounded O alone is the dominant error of dQ/dK/dE. */
  void* o_lo; int64_t ldolo;
  /* a query row whose every key is masked: 0 = uniform weights over the sequence (an additive
   * finfo.min mask, the eager attention of w2v-bert, tf:…wav2vec2_bert…:306-327); 1 = zero weights,
   * zero output and zero gradients (torch SDPA's fully-masked-row rule, which the XLM-R SDPA path
   * of the reference's transformers takes, tf:…xlm_roberta…:186-250).  The forward saves the row's
   * LSE as -inf (uniform) / +inf (zero) for the backward. */
  int zero_masked_rows;
} ste_attn_args;
int ste_attention_fwd(const ste_attn_args* a, void* stream);
/* fp32 forward of the text encoder's attention (the precise text forward, see ste_split_bf16):
 * q/k/v fp32 (row strides ld*, head h at columns h*64..), rel_E must be NULL; o32 fp32 [B*T, ldo32]
 * (optional) receives O; a->o / a->o_lo (bf16, optional) its hi / lo halves and a->lse the LSE, in the
 * conventions of ste_attention_fwd, so ste_attention_bwd runs on bf16 copies of q/k/v. */
int ste_attention_fwd_f32(const ste_attn_args* a, float* o32, int64_t ldo32, void* stream);
int ste_attention_bwd(const ste_attn_args* a, void* stream);
/* fp32 backward of ste_attention_fwd_f32 (the precise text backward; replaces the autograd of
 * tf:…xlm_roberta…:186-250 as trainer_unfreeze.py:1093 `loss.backward()` runs it): q/k/v and dout fp32,
 * o / o_lo the forward's bf16 hi / lo halves of O (delta = dout·(o + o_lo)), lse as saved, the
 * forward's key_mask / drop_p / seed / zero_masked_rows; writes dq / dk / dv fp32 (row strides
 * lddq / lddk / lddv; head h at columns h*64..).  rel_E must be NULL; delta, dE, gwork unused.
 * Run-to-run deterministic (no atomics). */
int ste_attention_bwd_f32(const ste_attn_args* a, void* stream);

/* ----------------------------------------------- Conformer conv module core --
 * GLU over channels then causal depthwise conv (left pad K-1), no bias.
 * Replaces tf:…wav2vec2_bert…:198-207 (glu, F.pad(K-1,0), depthwise_conv).
 * pre: bf16 [B*T, 2C]; w: fp32 [C, K]; out: bf16 [B*T, C].
 * Backward: dout bf16 [B*T, C] -> dpre bf16 [B*T, 2C]; dw fp32 [C,K] += (optional; with ws
 * of ste_glu_dwconv_bwd_ws_floats floats the per-block partials are summed in a fixed order,
 * run-to-run deterministic; ws = NULL: fp32 atomics).
 */
int ste_glu_dwconv_fwd(const void* pre, const float* w, void* out, int B, int T, int C, int K, void* stream);
int ste_glu_dwconv_bwd(const void* pre, const float* w, const void* dout, void* dpre, float* dw,
                       int B, int T, int C, int K, float* ws, int64_t ws_floats, void* stream);
int64_t ste_glu_dwconv_bwd_ws_floats(int B, int T, int C, int K);

/* ------------------------------------------------------------------ fbank --
 * Batched Kaldi-style log-mel fbank + per-utterance CMVN + stride-2 stacking:
 * the arithmetic of SeamlessM4TFeatureExtractor.__call__
 * (tf:models/seamless_m4t/feature_extraction_seamless_m4t.py:112-138,140-301,
 * tf:audio_utils.py:809-1017) fused with ref:training/trainer_unfreeze.py:880-921
 * (custom_collate_fn padding).  wav fp32 [B, ld_wav]; lengths int32 [B].
 * feats fp32 [B, Tmax, 160]; mask int64 [B, Tmax]; work fp32 >= B*Fmax*80 + B*160 with
 * Fmax = 2*Tmax (log-mel + per-clip CMVN statistics; the constant tables are compile-time data,
 * so the call keeps no device state and is re-entrant and graph-capturable).  mask_mode 0: collate semantics (1 for t < T_b);
 * mask_mode 1: extractor semantics (0 for a padded odd frame).
 */
int ste_fbank(const float* wav, int64_t ld_wav, const int32_t* lengths, int B, int Tmax, float pad_value,
              float* feats, int64_t* mask, int mask_mode, float* work, void* stream);

/* ------------------------------------------------------------------ heads --
 * AttentivePooling (ref:training/trainer_unfreeze.py:171-211) after its first
 * Linear+tanh has run through ste_gemm: score = t·w2 + b2, masked softmax over
 * the sequence (-1e9 fill), pooled = Σ w·h.
 * t bf16 [B*L, Hh]; h bf16 [B*L, H]; mask int32 [B*L] (NULL = all valid);
 * outputs: weights fp32 [B*L], pooled fp32 [B,H] and bf16 [B,H] (optional).
 */
int ste_attn_pool_fwd(const void* t, const float* w2, const float* b2, const void* h, const int32_t* mask,
                      int B, int L, int Hh, int H, float* weights, float* pooled, void* pooled_bf16,
                      void* stream);
/* Backward: dpooled fp32 [B,H] -> dh fp32 [B*L,H] (+=), dt bf16 [B*L,Hh]
 * (= dscore*w2*(1-t^2): the gradient at the scorer's first Linear output, tanh'
 * included), optional dt_lo bf16 [B*L,Hh] = bf16(dt - bf16(dt)) (the low half, for a
 * two-pass weight-gradient GEMM), dw2 fp32 [Hh] (+=), db2 fp32 [1] (+=), db1 fp32 [Hh] (+=,
 * the first Linear's bias gradient Σ_l dt_l summed in fp32; may be NULL).
 * work: fp32 scratch of ste_attn_pool_bwd_work_floats(B, L, Hh) floats (dscore [B*L], then
 * per-row-chunk column-sum partials, then the per-sample db2 terms; every sum in a fixed order).  Hh <= 1024.  mask: the forward's int32 [B*L] mask or
 * NULL; masked positions get no score gradient (masked_fill's backward, ref:199-200).  Replaces the
 * autograd of ref:184-211. */
int ste_attn_pool_bwd_work_floats(int B, int L, int Hh);
int ste_attn_pool_bwd(const void* t, const float* w2, const void* h, const float* weights, const float* dpooled,
                      const int32_t* mask, int B, int L, int Hh, int H, float* dh, void* dt, void* dt_lo, float* dw2,
                      float* db2,
                      float* db1, float* work, void* stream);
/* The same pooling on fp32 states (t fp32 [B*L, Hh] from ste_gemm_f32, h fp32 [B*L, H]; dt fp32,
 * no low half): the text side, whose positive and corrupted transcripts' pooled vectors are
 * differenced by the loss gradient (see ste_gemm_f32). */
int ste_attn_pool_fwd_f32(const float* t, const float* w2, const float* b2, const float* h, const int32_t* mask,
                          int B, int L, int Hh, int H, float* weights, float* pooled, void* pooled_bf16, void* stream);
int ste_attn_pool_bwd_f32(const float* t, const float* w2, const float* h, const float* weights, const float* dpooled,
                          const int32_t* mask, int B, int L, int Hh, int H, float* dh, float* dt, float* dw2,
                          float* db2, float* db1, float* work, void* stream);

/* Pooling without the scorer, use_attentive_pooling=False
 * (ref:training/trainer_unfreeze.py:578-580 text `last_hidden_state[:, 0, :]`, :621-636 audio
 * masked mean `sum(h*m)/clamp(sum(m), 1e-9)`): h bf16 [B*L, H]; mask int32 [B*L] (NULL = all
 * valid); cls != 0 selects row 0 of each sample. Outputs: weights fp32 [B*L] (the pooling
 * weights, read by the backward), pooled fp32 [B,H] and bf16 [B,H] (optional). */
int ste_mean_pool_fwd(const void* h, const int32_t* mask, int B, int L, int H, int cls, float* weights, float* pooled,
                      void* pooled_bf16, void* stream);
/* The same on fp32 states h [B*L, H]. */
int ste_mean_pool_fwd_f32(const float* h, const int32_t* mask, int B, int L, int H, int cls, float* weights,
                          float* pooled, void* pooled_bf16, void* stream);
/* Backward of any fixed-weight pooling: dh fp32 [B*L,H] += weights[b,l] * dpooled fp32 [B,H]. */
int ste_weighted_pool_bwd(const float* weights, const float* dpooled, int B, int L, int H, float* dh, void* stream);

/* CrossModalAttention with a single query vector per sample
 * (ref:training/trainer_unfreeze.py:125-168 called with x.unsqueeze(1) at :653-667):
 * q fp32 [B,P]; k,v bf16 [B*S, P] (row stride ldkv); mask int32 [B*S] (NULL = all);
 * nh heads of P/nh; softmax(q·kᵀ·scale, masked -1e9), dropout, ·v -> out fp32 [B,P].
 * probs fp32 [B*nh*S] saved for backward. */
int ste_xattn1_fwd(const float* q, const void* k, const void* v, int64_t ldkv, const int32_t* mask, int B, int S,
                   int P, int nh, float scale, float drop_p, uint64_t seed, float* probs, float* out, void* stream);
/* backward: mask = the forward's key mask (NULL = none); masked keys get no score gradient
 * (masked_fill's backward, ref:148-153) — only visible for an all-masked sample */
int ste_xattn1_bwd(const float* q, const void* k, const void* v, int64_t ldkv, const float* probs, const float* dout,
                   const int32_t* mask, int B, int S, int P, int nh, float scale, float drop_p, uint64_t seed,
                   float* dq, float* dk, float* dv, int64_t lddkv, void* stream);  /* dk/dv: fp32, += */
/* nq (1 or 2) query sets sharing one K/V (the positive and corrupted transcripts' text->audio
 * calls, ref:training/trainer_unfreeze.py:525-542): query qi of sample b is row qi*B+b of q / out /
 * dout / dq and of probs [(qi*B+b)*nh + head]*S; query set qi drops with seed_qi, exactly as an
 * xattn1 call on that set alone.  dk/dv are accumulated once for both sets.  P/nh % 8 == 0,
 * ldkv % 8 == 0, k/v/out/dq/dk/dv 16-B aligned. */
int ste_xattn_fwd(const float* q, const void* k, const void* v, int64_t ldkv, const int32_t* mask, int B, int S, int P,
                  int nh, int nq, float scale, float drop_p, uint64_t seed0, uint64_t seed1, float* probs, float* out,
                  void* stream);
int ste_xattn_bwd(const float* q, const void* k, const void* v, int64_t ldkv, const float* probs, const float* dout,
                  const int32_t* mask, int B, int S, int P, int nh, int nq, float scale, float drop_p,
                  uint64_t seed0, uint64_t seed1, float* dq, float* dk, float* dv, int64_t lddkv, void* stream);
/* As ste_xattn_bwd, but dk/dv are bf16 and WRITTEN (not accumulated), and colsum_part fp32
 * [B, 2P] receives per-sample column sums of dk (cols [0,P)) and dv (cols [P,2P)) in fp32, for the
 * key/value bias gradient; lddkv % 8 == 0. */
int ste_xattn_bwd_bf16(const float* q, const void* k, const void* v, int64_t ldkv, const float* probs,
                       const float* dout, const int32_t* mask, int B, int S, int P, int nh, int nq, float scale,
                       float drop_p,
                       uint64_t seed0, uint64_t seed1, float* dq, void* dk, void* dv, int64_t lddkv,
                       float* colsum_part, void* stream);

/* WordLevelAlignmentModule attention core (ref:training/trainer_unfreeze.py:214-310, the
 * nn.MultiheadAttention(P, nh=4, batch_first) of :237-242 with key_padding_mask, probs
 * dropout): q bf16 [B*L, ldq], kv bf16 [B*T, ldkv] = [K | V] (K cols h*d, V cols P+h*d),
 * kmask int32 [B*T] (0 = padded key), probs fp32 [B,nh,L,T] saved, out bf16 [B*L, ldo].
 * Backward: dout bf16 -> dq bf16 [B*L, lddq], dkv fp32 [B*T, lddkv] (written), dsbuf
 * fp32 [B,nh,L,T] workspace. */
int ste_align_attn_fwd(const void* q, int64_t ldq, const void* kv, int64_t ldkv, const int32_t* kmask, int B, int L,
                       int T, int P, int nh, float drop_p, uint64_t seed, float* probs, void* out, int64_t ldo,
                       void* stream);
int ste_align_attn_bwd(const void* q, int64_t ldq, const void* kv, int64_t ldkv, const float* probs,
                       const void* dout, int64_t lddo, int B, int L, int T, int P, int nh, float drop_p,
                       uint64_t seed, float* dsbuf, void* dq, int64_t lddq, float* dkv, int64_t lddkv, void* stream);
/* Backward of a Linear(K -> 1) + activation pair: out[m][k] = a[m]*w[k]*act'(z[m][k]) (bf16),
 * dw[k] += Σ_m a[m] z[m][k], db += Σ_m a[m]  (z = the activation OUTPUT for RELU/TANH). */
int ste_rank1_bwd(const float* a, const float* w, const void* z, int M, int K, int act, void* out, float* dw,
                  float* db, void* stream);

/* ------------------------------------------------------------------- loss --
 * F.normalize(p=2, dim=1, eps=1e-12) rows (ref:training/trainer_unfreeze.py:561-563). */
int ste_l2norm_fwd(const float* x, int rows, int cols, float* y, float* norms, void* stream);
int ste_l2norm_bwd(const float* y, const float* norms, const float* dy, int rows, int cols, float* dx,
                   void* stream);
/* Batch similarity matrix S = A·[Tpos;Tneg]ᵀ in exact fp32 on the f32 MFMA
 * (v_mfma_f32_32x32x2_f32): a [B,P], t [2B,P] -> S [B,2B].  s_pos = diag(S[:, :B]),
 * s_neg = diag(S[:, B:]) reproduce ref:training/trainer_unfreeze.py:1073-1074. */
int ste_similarity(const float* a, const float* t, int B, int NT, int P, float* S, void* stream);
/* AlignmentAwareInfoNCE (ref:training/trainer_unfreeze.py:702-742):
 * loss = mean_i softplus((s_neg-s_pos)/tau) * (1 - aw*sigmoid(mean_l align[i,l]))
 *        + gamma*mean_i relu(s_neg).  s_pos/s_neg are read from S's diagonals
 * (ldS = row stride, pos at column i, neg at column off_neg+i); align may be NULL.
 * Backward writes ds_pos, ds_neg [B] and dalign [B*L] (optional), scaled by gscale. */
int ste_pair_loss_fwd(const float* S, int64_t ldS, int off_neg, const float* align, int B, int L, float tau,
                      float aw, float gamma, float* s_pos, float* s_neg, float* loss, void* stream);
int ste_pair_loss_bwd(const float* s_pos, const float* s_neg, const float* align, int B, int L, float tau,
                      float aw, float gamma, const float* gscale, float* ds_pos, float* ds_neg, float* dalign,
                      void* stream);

/* ------------------------------------- data-parallel global similarity --
 * north_star: "an RCCL all-gather of embeddings ... before the similarity matmul".  After the
 * all-gather, S_g = A_g·[Tpos_g;Tneg_g]ᵀ (ste_similarity, [NB, 2NB]).
 * ste_pair_metrics: per row i of S [NB rows, ldS], accumulates into acc fp64[6]:
 *   Σ sigmoid(S[i][i]/τ), Σ sigmoid(S[i][off_neg+i]/τ) (ref to_human_readable :924-939, the
 *   clean / corrupt similarities train_epoch reports :1120-1161), Σ [s_pos > s_neg],
 *   Σ [argmax_{j<NB} S[i][j] == i] (in-batch top-1 retrieval), row count, and
 *   loss_w·Σ_r losses[r] (the ranks' batch losses, e.g. x local batch; losses may be NULL).
 * ste_inbatch_ce: optional in-batch-negative InfoNCE (weight 0 = the reference's loss, D1):
 *   local rows i < B of S (ldS) over NB global clean transcripts, target row0+i:
 *   loss[0] += weight/B Σ CE_i (loss-scale gscale (optional) multiplies dS only);
 *   dS[i][j] = weight·gs/B·(softmax_j − δ_{j,row0+i})/τ.
 * ste_rowmat_f32: out[r][p] += Σ_c X[r*sxr + c*sxc]·Y[c*P + p]  (R rows, P % 4 == 0). */
int ste_pair_metrics(const float* S, int64_t ldS, int NB, int off_neg, float tau, const float* losses, int nloss,
                     float loss_w, double* acc, void* stream);
int ste_inbatch_ce(const float* S, int64_t ldS, int B, int NB, int row0, float tau, float weight, const float* gscale,
                   float* loss, float* dS, int64_t lddS, void* stream);
int ste_rowmat_f32(const float* X, int64_t sxr, int64_t sxc, const float* Y, int R, int C, int P, float* out,
                   void* stream);
/* Gradients of s_pos[i] = <a_i, tp_i>, s_neg[i] = <a_i, tn_i> (the diagonals of S). */
int ste_pair_sim_bwd(const float* a, const float* tp, const float* tn, const float* ds_pos, const float* ds_neg,
                     int B, int P, float* da, float* dtp, float* dtn, void* stream);

/* --------------------------------------------------------------- embedding --
 * XLMRobertaEmbeddings (tf:…xlm_roberta…:75-121,142-155): position ids
 * cumsum(ids!=pad)*(ids!=pad)+pad, word+pos+type(0) gather.  Output fp32 sum
 * [B*L, D] (LayerNorm runs through ste_layernorm_fwd).  pos_ids int32 [B*L] saved. */
int ste_text_embed_fwd(const int64_t* ids, int B, int L, int D, int pad_idx, const float* word, const float* pos,
                       const float* type0, float* out, int32_t* pos_ids, void* stream);
/* Backward (nn.Embedding padding_idx rows get no gradient): dword / dpos rows += the sum of the
 * token rows carrying that id, in row order (one writer per table row, no atomics); dtype0 +=
 * the column sum of every row, ordered through ws (ste_text_embed_bwd_ws_floats floats; NULL:
 * atomics).  D % 4 == 0, D <= 1024.  Run-to-run deterministic with ws. */
int ste_text_embed_bwd(const int64_t* ids, const int32_t* pos_ids, const float* dout, int B, int L, int D,
                       int pad_idx, float* dword, float* dpos, float* dtype0, float* ws, int64_t ws_floats,
                       void* stream);
int64_t ste_text_embed_bwd_ws_floats(int B, int L, int D);

/* Row-sparse exchange of the word-embedding gradient between data-parallel ranks
 * (replaces all-reducing the dense 250,002 x 768 table that
 * ref:training/trainer_unfreeze.py:1084-1117 leaves to a single GPU).
 * ste_rows_extract: unique non-pad ids of ids[n] -> out_ids[cap] (-1 = empty slot),
 *   rows[cap, D] = grad[id] and grad[id] = 0.  flags int32 [vocab] must be zero on entry
 *   and is zero again on exit.  cap >= number of unique ids (e.g. n).
 * ste_rows_accumulate: grad[ids[s]] += scale * rows[s] for ids[s] >= 0 (unique ids). */
int ste_rows_extract(const int64_t* ids, int n, int pad_idx, float* grad, int D, int32_t* flags,
                     int32_t* out_ids, float* rows, int cap, int32_t* count, void* stream);
int ste_rows_accumulate(float* grad, int D, const int32_t* ids, const float* rows, int cap, float scale,
                        void* stream);

/* ------------------------------------------------------------- optimizer --
 * torch.nn.utils.clip_grad_norm_ + torch.optim.AdamW.step
 * (ref:training/trainer_unfreeze.py:1108-1110, groups :1487-1511).
 * ste_sumsq accumulates Σg² of n fp32 values into *acc in fp64: with part (double[2048]) the
 * per-block sums are added in block order (deterministic), part = NULL: fp64 atomics.
 * ste_adamw: reads clip coefficient min(1, max_norm/(sqrt(*sumsq)+1e-6)) on device
 * when sumsq != NULL, then decoupled-decay AdamW; writes bf16 shadow if non-NULL. */
int ste_sumsq(const float* g, int64_t n, double* acc, double* part, void* stream);
int ste_adamw(float* p, const float* g, float* m, float* v, void* p_bf16, int64_t n, float lr, float beta1,
              float beta2, float eps, float wd, int step, const double* sumsq, float max_norm, void* stream);

/* ------------------------------------------------------------ elementwise -- */
/* Split-bf16 operand image: y [rows][nblk*K] bf16 (nblk 1-3) gets nblk copies of x [rows][K] fp32,
 * copy i the high half bf16(x) or, when bit i of lo_mask is set, the low half bf16(x - bf16(x)).
 * ste_gemm on A = [x_hi | x_lo] (nblk 2, mask 2) and B = [W | W] (the bf16 weight twice, K' = 2K)
 * computes X·W_bf16ᵀ with the activations to ~16 mantissa bits: the text encoder's precise
 * forward (every XLM-R Linear, tf:…xlm_roberta…:186-398).  The weight's own rounding is shared by
 * the positive and corrupted transcripts, so it is not differenced by the loss gradient; the
 * activations' is.  nblk 3 ([hi|lo|hi]·[hi|hi|lo]) adds the weight's low half. */
int ste_split_bf16(const float* x, int64_t ldx, int64_t rows, int K, void* y, int nblk, int lo_mask, void* stream);
int ste_cast_f32_bf16(const float* x, void* y, int64_t n, void* stream);
/* y = alpha*x + beta*y over strided fp32 rows (gradient accumulation of head branches). */
int ste_axpby2d(float* y, int64_t ldy, const float* x, int64_t ldx, int64_t rows, int cols, float alpha, float beta,
                void* stream);
/* strided 2-D copy of 2- or 4-byte elements (concatenations feeding fusion GEMMs). */
int ste_copy2d(void* y, int64_t ldy, const void* x, int64_t ldx, int64_t rows, int cols, int elem_bytes,
               void* stream);
/* SpecAugment time masking of the audio encoder input (tf:…wav2vec2_bert…:944-988, training mode):
 * forward x[r,:] = embed for rows with spec[r] != 0 and valid[r] != 0 (x fp32 [rows, cols], row
 * stride ld; spec int32 [rows]; valid = the frame mask as float); backward dembed += Σ dx[r,:]
 * over the same rows (dembed may be NULL; with ws of ste_spec_mask_bwd_ws_floats floats the
 * per-block sums are added in a fixed order, ws = NULL: fp32 atomics) and dx[r,:] = 0. */
int ste_spec_mask_fwd(float* x, int64_t ld, const int32_t* spec, const float* valid, const float* embed,
                      int64_t rows, int cols, void* stream);
int ste_spec_mask_bwd(float* dx, int64_t ld, const int32_t* spec, const float* valid, float* dembed,
                      int64_t rows, int cols, float* ws, int64_t ws_floats, void* stream);
int64_t ste_spec_mask_bwd_ws_floats(int64_t rows, int cols);
/* y[c, r] = x[r, c] for 2-byte elements (row strides ldx >= cols, ldy >= rows, in elements).
 * Builds the k-contiguous copies Wᵀ [in, out] of the nn.Linear weights that the input-gradient
 * GEMMs dX = dY·W read as their KC operand (replaces reading W k-major in the backward of
 * every encoder Linear: tf:…wav2vec2_bert…:119-226, tf:…xlm_roberta…:186-398). */
int ste_transpose16(void* y, int64_t ldy, const void* x, int64_t ldx, int64_t rows, int cols, void* stream);
/* out[c] += Σ_r x[r, c] over a row-major [rows, cols] fp32/bf16 matrix (bias gradients): with ws
 * (>= ste_colsum_ws_floats(rows, cols) floats) one partial row per 512-row chunk, added in chunk
 * order (run-to-run deterministic); ws = NULL: fp32 atomics. */
int ste_colsum(const void* x, int is_bf16, int64_t rows, int cols, int64_t ld, float* out, float* ws,
               int64_t ws_floats, void* stream);
int64_t ste_colsum_ws_floats(int64_t rows, int cols);
/* out[b·cols + c] += Σ_{r < rows} part[(b·rows + r)·cols + c], summed in a fixed order (the
 * ordered second pass of every deterministic column sum: GEMM bias gradients, ste_colsum, the
 * depthwise-conv and SpecAugment-embedding gradients, the pooling scorer bias). */
int ste_rowsum_ordered(const float* part, int64_t rows, int cols, int batch, float* out, void* stream);
/* y[r, c] = x[r, c] * scale[r]  (fp32, row stride ld) */
int ste_scale_rows(float* x, const float* scale, int64_t rows, int cols, int64_t ld, void* stream);
int ste_mask_i64_to_f32(const int64_t* m, float* f, int32_t* i32, int64_t n, void* stream);

/* ------------------------------------------- wav2vec2 raw-waveform front end --
 * EnhancedAudioTextModel(audio_model_name="facebook/wav2vec2-base"),
 * whose encode_audio (ref:training/trainer_unfreeze.py:587-641) hands raw 16 kHz samples to
 * transformers' Wav2Vec2Model (tf:models/wav2vec2/modeling_wav2vec2.py:1244-1375).  Activations
 * are time-major [B*T, C]; the strided Conv1d layers and the grouped positional conv are
 * ste_gemm launches on strided views (see csrc/w2v2.hip), these entries are the rest.
 *
 * conv0 (C_in = 1, no bias; :302-323): y fp32 [B*T0, C] = Σ_j w0[c, j]·wave[b, S0·t + j]
 *   (w0 [C, K0], K0 <= 16, S0 <= 8, S0·(T0-1) + K0 <= N). */
int ste_w2v_conv0_fwd(const float* wave, int64_t ldw, const float* w0, int B, int N, int T0, int C, int K0, int S0,
                      float* y, void* stream);
/* GroupNorm(num_groups = C) over time per (b, c) (biased variance, eps) + affine + GELU:
 * h bf16 [B*T0, C]; mean/rstd fp32 [B*C] are kept for the backward.  C % 4 == 0, C <= 1024.
 * work: fp32 scratch of ste_w2v_gn_work(B, T0, C, K0) floats (fp64 partial sums per 512-row
 * chunk; deterministic, no atomics), shared by the forward (K0 = 1) and the backward. */
int64_t ste_w2v_gn_work(int B, int T0, int C, int K0);
int ste_w2v_gn_fwd(const float* y, const float* gamma, const float* beta, int B, int T0, int C, float eps,
                   float* mean, float* rstd, void* h, float* work, int64_t work_floats, void* stream);
/* Backward of conv0 + GroupNorm + GELU given dh = dL/dh fp32 [B*T0, C]: dgamma/dbeta/dw0 +=
 * (each may be NULL). */
int ste_w2v_gn_bwd(const float* dh, const float* y, const float* mean, const float* rstd, const float* gamma,
                   const float* beta, const float* wave, int64_t ldw, int B, int N, int T0, int C, int K0, int S0,
                   float* dgamma, float* dbeta, float* dw0, float* work, int64_t work_floats, void* stream);
/* out[i] += Σ_s part[s·n + i] (per-clip weight-gradient slabs of the strided conv GEMMs). */
int ste_w2v_slab_sum(float* out, const float* part, int64_t n, int S, void* stream);
/* col2im of a strided Conv1d input gradient: out[b, ti, c] = gelu'(z[b,ti,c]) ·
 * Σ_{s·to + j = ti} dcol[b·To + to, j·C + c] (dcol fp32 row stride ldd; z bf16 or NULL for no
 * activation; out bf16 if out_bf16 else fp32; [B*Ti, C]).  k = s = 1 applies gelu' alone. */
int ste_w2v_conv_fold(const float* dcol, int64_t ldd, const void* z, int B, int Ti, int To, int C, int k, int s,
                      void* out, int out_bf16, void* stream);
/* [A][P][Q] -> [A][Q][P]: bf16 copy (conv weights [Co][Ci][k] -> the GEMM's [Co][k][Ci]), or with
 * fp32_accumulate an fp32 += (the weight gradient back into the [Co][Ci][k] layout). */
int ste_w2v_perm12(const void* src, void* dst, int A, int P, int Q, int fp32_accumulate, void* stream);
/* Positional conv (weight-normed Conv1d(D, D, K, padding K/2, groups G) + SamePad + GELU,
 * :326-379).  pos_pack: x fp32 [B*T, D] -> bf16 [G][B*Tp + K][D/G], Tp = T + K - 1, row b·Tp + u
 * holding x[b, u - padl] (zero outside [0, T)); the forward GEMM reads it with row stride D/G.
 * pos_elem: mode 0 out = src + gelu(cpad + bias); mode 1 out = src·gelu'(cpad + bias); mode 2
 * out = (src + cpad)·maskf[row] (maskf may be NULL); cpad fp32 rows b·Tp + t, src/out [B*T, D]. */
int ste_w2v_pos_pack(const float* x, int B, int T, int D, int G, int K, int padl, void* out, void* stream);
int ste_w2v_pos_elem(int mode, const float* cpad, const float* bias, const float* src, const float* maskf, int B,
                     int T, int D, int Tp, float* out, void* stream);
/* weight_norm(dim=2) (nn.utils.parametrizations.weight_norm): v fp32 [D][Cg][K], g fp32 [K];
 * writes norms[K] and the GEMM operands wr bf16 [G][Cg co][K][Cg ci] (forward) and wf bf16
 * [G][Cg ci][K][Cg co] (taps reversed, the input gradient).  Backward from dW in the wr layout
 * (fp32): dg[j] += s_j/n_j, dv += (g_j/n_j)·dW - (g_j s_j/n_j³)·v, s_j = Σ dW·v. */
int ste_w2v_wnorm_fwd(const float* v, const float* g, int D, int Cg, int K, float* norms, void* wr, void* wf,
                      void* stream);
int ste_w2v_wnorm_bwd(const float* dwr, const float* v, const float* g, const float* norms, int D, int Cg, int K,
                      float* dv, float* dg, void* stream);
/* Frame mask of the conv stack (:997-1036): per clip L = Σ mask[b, :] (N if mask is NULL) pushed
 * through floor((L - k)/s) + 1 per layer; maskf/mask32 [B*Tf] = t < L (either may be NULL).
 * kernels/strides are HOST arrays of nconv <= 16 entries. */
int ste_w2v_frame_mask(const int64_t* mask, int B, int N, int Tf, int nconv, const int* kernels, const int* strides,
                       float* maskf, int32_t* mask32, void* stream);
/* Wav2Vec2FeatureExtractor do_normalize: out[b, n] = (x - mean)/sqrt(var + 1e-7) over the first
 * lengths[b] samples (population variance; lengths NULL = N), pad after. */
int ste_w2v_wave_norm(const float* wave, int64_t ldw, const int32_t* lengths, int B, int N, float pad, float* out,
                      void* stream);
/* x[r, c] *= keep(seed, r·N + c)/(1-p) (the GEMM epilogue's dropout index) · maskf[r] (NULL = 1):
 * backward of an output dropout + row mask, in place on a contiguous fp32 [M, N]. */
int ste_w2v_drop_rows(float* x, int M, int N, float p, uint64_t seed, const float* maskf, void* stream);

const char* ste_version(void);

#ifdef __cplusplus
}
#endif
#endif /* STE_H_ */

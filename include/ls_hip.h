/*
 * ls_hip.h -- C-ABI of the MI355X (gfx950) kernel library libls_hip.so for the
 * LatentSync inference denoising hot path.
 *
 * The reference has no FFI on this path: its swap points are
 * the duck-typed Python objects injected into LipsyncPipeline.__init__
 * (latentsync/pipelines/lipsync_pipeline.py:49-124).  This library sits UNDER
 * those objects; the host package latentsync_amd binds it with ctypes.  Every
 * entry point below names the reference interface whose arithmetic it replaces.
 *
 * Conventions
 *   - All tensors are caller-allocated device buffers (plain pointers); no entry
 *     point allocates, frees or synchronises, so every call can be captured into
 *     a hipGraph.  `stream` is a hipStream_t (NULL = default stream).
 *   - Activations are "pixel-major" (NHWC): frames are folded into the image
 *     index exactly like InflatedConv3d's "b c f h w -> (b f) c h w"
 *     (latentsync/models/resnet.py:10-18); element (img, y, x, c) lives at
 *     ((img*H + y)*W + x)*ld + c.  Storage type is bf16 (uint16_t bit pattern)
 *     unless a field says fp32.
 *   - Return value: 0 = LS_OK, otherwise an ls_status; ls_last_error() returns
 *     a thread-local message for the last failure.
 */
#ifndef LS_HIP_H
#define LS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LS_ABI_VERSION 13

typedef enum {
  LS_OK = 0,
  LS_ERR_INVALID = 1,  /* bad shape / alignment / unsupported combination */
  LS_ERR_LAUNCH = 2,   /* hipLaunchKernel / hipGetLastError failure       */
  LS_ERR_WORKSPACE = 3 /* workspace missing or too small                   */
} ls_status;

enum { LS_ACT_NONE = 0, LS_ACT_GEGLU = 1, LS_ACT_GELU = 2, LS_ACT_SILU = 3 };

/*
 * Fused implicit-GEMM convolution / linear layer on bf16 MFMA
 * (v_mfma_f32_16x16x32_bf16), fp32 accumulate.
 *
 *   Y[m, n] = epilogue( sum_k A[m, k] * Wp[n, k] )
 *
 * A is never materialised: row m is an output pixel (img, yo, xo); column
 * k reads input channel ci of the tap's source pixel -- k = tap*Cin + ci, or for
 * ksize 3 with Cin % 64 == 0 (ABI 10) k = (ci/64)*576 + tap*64 + ci%64 -- from x1
 * (ci < C1) or x2 (ci >= C1, the fused torch.cat of the up blocks,
 * unet_blocks.py:624,745).  Optional prologue per element (fused GroupNorm
 * apply + SiLU of ResnetBlock3D, resnet.py:185-186 / 207-213):
 *   a = x * aff_scale[s, ci] + aff_shift[s, ci]; if (silu_in) a = silu(a)
 * with s = img / imgs_per_sample.  Zero padding is applied after the prologue.
 * ksize 1 = linear / 1x1 conv (Transformer proj_in/out, q/k/v/out, FF, shortcut);
 * ksize 3 = InflatedConv3d 3x3 (conv1/2, conv_in/out, samplers).
 * stride 2 + pad 1 = Downsample3D (resnet.py:89), stride 2 + pad 0 = the SD-VAE
 * downsampler after F.pad(0,1,0,1); upsample = nearest x2 fused into the
 * gather (Upsample3D, resnet.py:53-73).
 *
 * Wp is the packed weight [N][K]: K = ksize*ksize*Cin rounded up to 64, in the same
 * k order: tap-major, except ksize 3 with Cin % 64 == 0, which is channel-chunk-major
 * (the 9 taps of a 64-channel chunk consecutive; see latentsync_amd/packing.py).
 * Epilogue, in this order:
 *   if (ln_rowstats)  acc = rstd[m] * (acc - mean[m] * ln_colsum[n])
 *       -- LayerNorm of the A rows folded into the GEMM: with Wp = W * gamma
 *       (per input column), bias = b + W beta and ln_colsum[n] = sum_k Wp[n, k],
 *       this equals W LN(x) + b exactly in real arithmetic (BasicTransformerBlock
 *       norm1/2/3 -> to_q|k|v / to_q / ff.net.0, attention.py:145-199;
 *       TemporalTransformerBlock norms -> q|k|v / FF, motion_module.py:240-313);
 *       ln_rowstats = (mean, rstd) fp32 pairs per row from ls_row_stats
 *   v = acc + bias[n] + rowvec[((m / rows_per_vec) % rowvec_mod) * rowvec_ld + n]
 *       (temb add, resnet.py:190-205; W pe of the motion positional encoding;
 *        rowvec_mod 0 = no modulo)
 *   v = (v + res[m, n]) * out_scale                      (residual, resnet.py:221)
 *   act: GEGLU pairs packed columns (32b+i, 32b+16+i) -> out col 16b+i,
 *        out = h * gelu_erf(g) (diffusers GEGLU); GELU (whisper MLP); SiLU.
 * split_k > 1 needs `workspace` of split_k*M*N fp32 (ls_conv_workspace_bytes).
 */
typedef struct {
  const uint16_t* x1; const uint16_t* x2;
  int32_t C1, C2;            /* channels read from x1 / x2 (C2 = 0: no concat) */
  int32_t ld1, ld2;          /* pixel pitch (elements) of x1 / x2             */
  int32_t n_img, H, W;       /* input images / resolution (ksize 1: H=1, W=rows) */
  int32_t Ho, Wo;            /* output resolution                              */
  int32_t ksize, stride, pad, upsample;
  const float* aff_scale; const float* aff_shift; int32_t imgs_per_sample; int32_t silu_in;
  const uint16_t* w; int32_t K; int32_t N;
  const float* bias;
  const float* rowvec; int32_t rows_per_vec; int32_t rowvec_ld; /* rowvec_ld 0 = N */
  const uint16_t* res; int32_t ldr; float out_scale;
  int32_t act;
  void* y; int32_t ldy; int32_t y_f32;
  int32_t split_k;           /* 0 = choose automatically                       */
  void* workspace; size_t workspace_bytes;
  const float* ln_rowstats;  /* NULL or (mean, rstd) per A row (ksize 1 only)  */
  const float* ln_colsum;    /* [N] column sums of Wp (with ln_rowstats)       */
  int32_t rowvec_mod;        /* 0 = none                                       */
  float* row_stats_out;      /* NULL or fp32 [M][2] (mean, rstd) of each output row (ksize 1,
                                LayerNorm statistics for the next folded GEMM; the row-block
                                kernel emits them from its epilogue, other paths run
                                ls_row_stats on y)                                  */
  float row_stats_eps;       /* LayerNorm eps of row_stats_out (0 = 1e-5)        */
  float* gn_colsum_out;      /* NULL or fp32 [M / LS_GN_SLOT_ROWS][2][N]: per 128-row slot and
                                output column, the sum and the sum of squares of the stored
                                bf16 values (GroupNorm statistics of y for
                                ls_groupnorm_colsum; M % 128 == 0, bf16 output, no GEGLU).
                                The tiled kernels emit them from their epilogue; the other
                                paths (split-K, row-block, small tiles) read y once more. */
} ls_conv_desc;

#define LS_GN_SLOT_ROWS 128

int ls_conv2d(const ls_conv_desc* d, void* stream);
/* Which kernel family ls_conv2d would run for d: 0 = tiled DMA GEMM, 1 = row-block
 * GEMM (K = 320 / 640 linears; also takes the GroupNorm affine prologue on its
 * register-resident A rows), 2 = register-staged tiled GEMM (affine prologue
 * elsewhere -- callers materialise the affine with ls_groupnorm_apply instead),
 * 3 = halo-tile 3x3 conv (ABI 12: 3x3 / stride 1 / pad 1 (or a nearest-x2 upsample without an
 * input affine, round 6), Cin % 64 == 0, W in {16, 32,
 * 64} or a multiple of 64, N % 160 or % 128 == 0; takes the GroupNorm affine + SiLU on
 * its input, once per pixel, and the dual-source concat), -1 = invalid descriptor.
 * Host-only, no launch. */
int ls_conv_path(const ls_conv_desc* d);
size_t ls_conv_workspace_bytes(const ls_conv_desc* d);

/*
 * GroupNorm statistics -> per-(sample, channel) affine for the consumer's
 * prologue.  Replaces nn.GroupNorm of ResnetBlock3D (5-D: stats span all frames
 * of a sample, resnet.py:140,164; unet.py:236), Transformer3DModel.norm and
 * TemporalTransformer3DModel.norm (4-D per frame, attention.py:51,
 * motion_module.py:101) and the SD-VAE GroupNorms.
 * Input: n_samples * pix_per_sample pixels of C = C1 + C2 channels (x2 = concat).
 * Output: scale[s, c] = gamma[c] * rstd[s, g]; shift[s, c] = beta[c] - mean[s, g] * scale.
 * One launch: the last-arriving block of a sample merges the split partials.
 * workspace >= ls_groupnorm_workspace_bytes(); its first 4 KiB are arrival
 * counters that must be zero before the first call (each call re-arms them).
 */
int ls_groupnorm(const uint16_t* x1, const uint16_t* x2, int32_t C1, int32_t C2, int32_t n_samples,
                 int64_t pix_per_sample, int32_t groups, float eps, const float* gamma, const float* beta,
                 float* scale, float* shift, void* workspace, size_t workspace_bytes, void* stream);
size_t ls_groupnorm_workspace_bytes(int32_t n_samples, int32_t groups);

/*
 * GroupNorm statistics from producer column sums (ls_conv_desc.gn_colsum_out or
 * ls_gn_colsum): the same affine as ls_groupnorm without reading the activation
 * again.  cs1 / cs2: [n_samples * pix_per_sample / 128][2][C1 | C2] of x1 / x2;
 * pix_per_sample % LS_GN_SLOT_ROWS == 0.  Slot sums are merged in fp64 per
 * (sample, group); var = E[x^2] - mean^2 (the fp32 slot sums bound the relative
 * variance error by ~1e-7 * (1 + mean^2 / var)).
 */
int ls_groupnorm_colsum(const float* cs1, const float* cs2, int32_t C1, int32_t C2, int32_t n_samples,
                        int64_t pix_per_sample, int32_t groups, float eps, const float* gamma, const float* beta,
                        float* scale, float* shift, void* stream);

/* The column sums of an existing bf16 [M][ldy] tensor (first N columns) by a read
 * pass: out [M / 128][2][N] as ls_conv_desc.gn_colsum_out. */
int ls_gn_colsum(const uint16_t* y, int64_t ldy, int64_t M, int32_t N, float* out, void* stream);

/* Materialised GroupNorm(+SiLU) apply over an optional channel concat
 * (x1 | x2) -> y [n_pix][C1 + C2]: the input of a 3x3 conv, whose gather would
 * otherwise recompute the affine + SiLU once per tap and per N-tile. */
int ls_groupnorm_apply(const uint16_t* x1, const uint16_t* x2, int32_t C1, int32_t C2, int64_t n_pix,
                       int64_t pix_per_sample, const float* scale, const float* shift, int32_t silu, uint16_t* y,
                       void* stream);

/*
 * LayerNorm over the last dim (nn.LayerNorm of BasicTransformerBlock
 * attention.py:145,157,172 and TemporalTransformerBlock motion_module.py:195,201;
 * whisper LayerNorm model.py:29-31).  Optional fused temporal positional
 * encoding add (VersatileAttention pos_encoder, motion_module.py:267-268):
 *   y[r, c] += pe[(r / pe_rows_per_frame) % pe_frames, c]   (pe fp32 [len][C]).
 * x rows are ldx elements apart (ldx >= C, multiple of 8); y is dense [rows][C].
 */
int ls_layernorm(const uint16_t* x, int64_t ldx, int64_t rows, int32_t C, float eps, const float* gamma,
                 const float* beta, const float* pe, int32_t pe_rows_per_frame, int32_t pe_frames, uint16_t* y,
                 void* stream);

/* Per-row LayerNorm statistics (mean, rstd = 1/sqrt(var + eps)) fp32 pairs of
 * x [rows][C] (row pitch ldx): the producer side of the LayerNorm -> linear fold
 * (ls_conv_desc.ln_rowstats). */
int ls_row_stats(const uint16_t* x, int64_t ldx, int64_t rows, int32_t C, float eps, float* stats, void* stream);

/*
 * Multi-head attention softmax(Q K^T * scale) V on MFMA with LDS-staged K/V
 * tiles (F.scaled_dot_product_attention of Attention.forward attention.py:271,
 * VersatileAttention motion_module.py:300, whisper qkv_attention model.py:88-100,
 * SD-VAE mid attention).  Element (b, h, i, d) of T in {q,k,v,o} is at
 *   T + (b / z2)*T_sb1 + (b % z2)*T_sb2 + i*T_si + h*T_sh + d
 * so spatial (rows = tokens), temporal ("(b f) s c -> (b s) f c") and audio
 * cross-attention (Nk = 50) are strided views of the projection outputs.
 * head_dim <= 512.
 */
typedef struct {
  const uint16_t* q; const uint16_t* k; const uint16_t* v; uint16_t* o;
  int64_t q_sb1, q_sb2, q_si, q_sh;
  int64_t k_sb1, k_sb2, k_si, k_sh;
  int64_t v_sb1, v_sb2, v_si, v_sh;
  int64_t o_sb1, o_sb2, o_si, o_sh;
  int32_t batch, z2, heads, nq, nk, head_dim;
  float scale;
} ls_attn_desc;

int ls_attention(const ls_attn_desc* d, void* stream);

/*
 * The same attention with the P V product in fp8 (BASELINE.json configs[4], "fp8 MFMA
 * attention"; replaces the same SDPA call, attention.py:271): QK^T and the softmax as
 * ls_attention (bf16 MFMA, fp32), P and V in OCP e4m3 on the block-scaled MFMA
 * v_mfma_scale_f32_16x16x128_f8f6f4.  V is quantised by a pre-pass into `workspace`
 * with one e8m0 scale per (head dim, 128-key tile) -- block scaling, the tile's max
 * mapped into [128, 256), the same scale for all four 32-key MX blocks of a tile; P (<= 2^8 by the kernel's rescale threshold) uses scale 1 and the
 * row sums come from the same e4m3 P.  Two launches (quantise, attend), capturable.
 * head_dim 40 or 80 (the UNet's 64^2 / 32^2 levels); q/k/v rows 16-B aligned, o rows 8-B aligned.
 * Workspace: ls_attention_fp8_workspace_bytes(d) (0 = unsupported head_dim), 16-B aligned;
 * its layout is documented in ls_attn.hip (the tests read it back).
 */
size_t ls_attention_fp8_workspace_bytes(const ls_attn_desc* d);
int ls_attention_fp8(const ls_attn_desc* d, void* workspace, size_t workspace_bytes, void* stream);

/*
 * The motion module's temporal self-attention fused with its input side: replaces, per
 * VersatileAttention block (latentsync/models/motion_module.py:203-218 and :262-313),
 *   LayerNorm(h) -> "(b f) s c -> (b s) f c" + pe[:f] -> to_q / to_k / to_v -> SDPA over
 *   the f frames (8 heads) -> "(b s) f c -> (b f) s c"
 * writing the attention output o (before to_out).  The q|k|v projections never reach HBM.
 *   x, o   : (n_samples * F * S) rows of C bf16, row (b*F + f)*S + s, pitches ldx / ldo
 *   gamma  : fp32 [C], the LayerNorm weight;  bpe: fp32 [16][C], LayerNorm bias + pe row f
 *   w      : bf16 [3C][C] packed per 80-column group g and 16-channel tile t = 0..4: q rows
 *            80g+16t..+15 scaled by log2(e)/sqrt(C/8), then the same k rows, then v rows
 *            (latentsync_amd/ops.py pack_temporal)
 * C = 320 (d 40) or 640 (d 80), heads = 8, 1 <= F <= 16, S % 16 == 0 (C = 320) or S % 8 == 0
 * (C = 640), 16-B aligned pointers, pitches % 8 == 0.
 */
typedef struct {
  const uint16_t* x;
  int32_t ldx;
  const float* gamma;
  const float* bpe;
  const uint16_t* w;
  uint16_t* o;
  int32_t ldo;
  int32_t C, heads, n_samples, F, S;
  float eps;
} ls_tattn_desc;

int ls_temporal_attention(const ls_tattn_desc* d, void* stream);

/*
 * FeedForward of a BasicTransformerBlock / TemporalTransformerBlock with its LayerNorm and
 * residual, one launch (ABI 11; diffusers FeedForward(dim, "geglu"), attention.py:174-199
 * norm3 + ff, motion_module.py:240-313 ff_norm + ff):
 *   y = x + W2 (h * gelu_erf(g)) + b2,  [h | g] = W1 LN(x) + b1
 * x, y: bf16 rows [M][ldx] / [M][ldy]; ln_rowstats: (mean, rstd) fp32 pairs of the x rows
 * (the producing GEMM's row_stats_out); w1: bf16 [2*inner][C], the GEGLU rows interleaved
 * in 16-row blocks (packing.geglu_interleave) with LayerNorm gamma folded in (W1 * gamma),
 * b1: fp32 [2*inner] = b1 + W1 beta in the same order; w2: bf16 W2 [C][inner] re-packed
 * per 32-column chunk (packing.pack_ff_w2: [inner/32][C][32], columns permuted and 16-B
 * pieces swizzled to the kernel's register layout); b2: fp32 [C].  C = 320, inner = 1280
 * (the 32x32 level) only.  The 4C-wide GEGLU intermediate never reaches memory.
 */
typedef struct {
  const void* x;
  const float* ln_rowstats;
  const void* w1;
  const float* b1;
  const void* w2;
  const float* b2;
  void* y;
  int64_t M;
  int32_t ldx, ldy, C, inner;
} ls_ff_desc;

int ls_feedforward(const ls_ff_desc* d, void* stream);

/*
 * The 32x32-level tail of a Transformer3DModel block / motion module in ONE launch (ABI
 * 13): the attention branch's out-projection + residual, the LayerNorm, the GEGLU
 * FeedForward + residual and proj_out + the block input, with the GroupNorm column sums
 * of the result (replaces attention.py:174-199 attn2.to_out + norm3 + ff and :110-118
 * proj_out; motion_module.py:262-313 the last to_out + ff_norm + ff and :126-151 proj_out):
 *   h2 = o Wo^T + bo + h1,  y = h2 + W2 (h * gelu_erf(g)) + b2 with [h | g] = W1 LN(h2) + b1,
 *   z  = y Wp^T + bp + xb
 * Rows: o, h1, xb, z bf16 [M][ld*] (M % 128 == 0).  LN statistics are computed in the
 * kernel over the bf16-rounded h2 (biased variance, eps).  Weights (packing.pack_ff_chain):
 * wo, wp bf16 [C/32][C][32] k-step images (wp and w1 with each 32-wide k block permuted to
 * the register order of pack_ff_w2, wo in natural order; 16-B pieces swizzled as w2); w1
 * bf16 [2*inner][C] (GEGLU rows interleaved, LN gamma folded), b1 = b1 + W1 beta; w2 as
 * ls_feedforward; bo, b2, bp fp32 [C].  cs_out: NULL or fp32 [M/128][2][C] column sums
 * (Σz, Σz²) of the stored z per 128-row slot (ls_conv_desc.gn_colsum_out's layout).
 * C = 320, inner = 1280 only.  h2 and y never reach memory.
 */
typedef struct {
  const void* o;
  const void* wo;
  const float* bo;
  const void* h1;
  const void* w1;
  const float* b1;
  const void* w2;
  const float* b2;
  const void* wp;
  const float* bp;
  const void* xb;
  void* z;
  float* cs_out;
  int64_t M;
  int32_t ldo, ldh, ldxb, ldz, C, inner;
  float eps;
} ls_ff_chain_desc;

int ls_ff_chain(const ls_ff_chain_desc* d, void* stream);

/*
 * The audio cross-attention branch of a BasicTransformerBlock, one launch (ABI 12;
 * attention.py:174-199 norm2 + attn2, Attention.forward :250-280 with the Whisper chunks
 * as encoder_hidden_states; replaces the LN-folded to_q GEMM + ls_attention + the
 * to_out GEMM with its residual):
 *   y = x + Wo softmax((Wq LN(x) + bq) K^T / sqrt(d)) V + bo
 * and stats_out = (mean, rstd) of the stored y rows (eps; norm3's LayerNorm fold).
 * x, y: bf16 rows [M][ldx] / [M][ldy], hw rows per image (a multiple of 128, M a multiple
 * of hw); ln_rowstats: (mean, rstd) of the x rows; kv: bf16 [M / hw * L][ldkv] rows of
 * to_k | to_v of the image's L audio tokens (L <= 64); wq / bq: packing.pack_xattn_q
 * (per head 48 rows with LayerNorm gamma / beta and log2(e) / sqrt(d) folded, k-images
 * swizzled); wo: packing.pack_xattn_wo (columns permuted to the kernel's k-slot order,
 * padding slots zero); bo: fp32 [C].  C = 320, 8 heads (the 32x32 level) only.
 */
typedef struct {
  const void* x;
  const float* ln_rowstats;
  const void* wq;
  const float* bq;
  const void* kv;
  const void* wo;
  const float* bo;
  void* y;
  float* stats_out;
  int64_t M;
  int32_t ldx, ldy, ldkv, C, heads, L, hw;
  float eps;
} ls_xattn_desc;

int ls_cross_attention_block(const ls_xattn_desc* d, void* stream);

/*
 * Small-M linear in fp32: y[m, n] = sum_k act(x[m, k]) * W[n, k] + bias[n]
 * (x fp32, W bf16 [N][K], 0 < M <= 1024, K <= 2048, K % 8 == 0); pre-activation SiLU optional.  TimestepEmbedding
 * (unet.py:382) and the batched time_emb_proj of every ResnetBlock3D
 * (resnet.py:190-194).
 */
int ls_small_linear(const float* x, int32_t M, int32_t K, const uint16_t* w, const float* bias, int32_t N,
                    int32_t silu_in, float* y, void* stream);

/* diffusers Timesteps(320, flip_sin_to_cos, shift) (unet.py:95,376): t read from
 * timesteps[*step] (device int32 array + device step index), out fp32 [B][dim]. */
int ls_timestep_embed(const int32_t* timesteps, const int32_t* step, int32_t B, int32_t dim, int32_t flip,
                      float shift, float* out, void* stream);

/* The same embedding for B fp32 timesteps, one per sample (ABI 13): the reference's
 * forward accepts a python float and a per-sample timestep vector, broadcasting it over
 * the batch (unet.py:361-376); ts device fp32 [B], out fp32 [B][dim]. */
int ls_timestep_embed_f32(const float* ts, int32_t B, int32_t dim, int32_t flip, float shift, float* out,
                          void* stream);

/*
 * CFG combine + DDIMScheduler.step (eta = 0) fused, then re-packs the next UNet
 * input (lipsync_pipeline.py:540-562).  eps: UNet output bf16 NHWC [Bu*P][ld_eps]
 * (4 used channels); lat fp32 [P][4] updated in place; coef fp32 table
 * [n_steps][4] = {sqrt(a_t), sqrt(1-a_t), sqrt(a_prev), sqrt(1-a_prev)} read at
 * *step; then *step += 1 (single thread).  When guidance > 1 the batch halves are
 * (uncond, audio).  unet_in (bf16 NHWC [Bu*P][ld_in]) receives the new latents in
 * channels 0..3 of every batch copy.
 */
int ls_ddim_cfg_step(const uint16_t* eps, int32_t ld_eps, int32_t Bu, int64_t P, float guidance, float* lat,
                     const float* coef, int32_t* step, uint16_t* unet_in, int32_t ld_in, void* stream);

/* Pixel prep (ImageProcessor.preprocess_fixed_mask_image image_processor.py:145-152):
 * faces uint8 NCHW [F][3][R][R]; mask fp32 [R][R] (1 = keep);
 * pix / masked bf16 NHWC [F][R][R][ld] (channels 3..ld-1 zeroed). */
int ls_prep_pixels(const uint8_t* faces, int32_t F, int32_t R, const float* mask, uint16_t* pix, uint16_t* masked,
                   int32_t ld, void* stream);

/* DiagonalGaussianDistribution.sample + (z - shift) * scaling (lipsync_pipeline.py:296-297):
 * moments fp32 NHWC [P][ld_m] (mean = ch 0..3, logvar = ch 4..7), eps fp32 [P][4];
 * writes bf16 into dst[P][ld_dst] at channel offset c_off. */
int ls_vae_sample(const float* moments, int32_t ld_m, const float* eps, int64_t P, float scaling, float shift,
                  uint16_t* dst, int32_t ld_dst, int32_t c_off, void* stream);

/* Builds the constant channels of the UNet input for a window
 * (lipsync_pipeline.py:517-549): ch 4 = nearest-resized keep-mask (prepare_mask_latents
 * :290), ch 5..8 masked-image latents, ch 9..12 reference latents (both already
 * written by ls_vae_sample into `cond` [P][16]); replicated into Bu copies of
 * unet_in [Bu][P][ld_in] together with the initial latents lat fp32 [P][4]. */
int ls_pack_unet_input(const float* lat, const uint16_t* cond, const float* mask, int32_t F, int32_t R, int32_t h,
                       int32_t Bu, uint16_t* unet_in, int32_t ld_in, void* stream);

/* decode_latents prep (lipsync_pipeline.py:146-147): z = lat / scaling + shift,
 * lat fp32 [P][4] -> bf16 NHWC [P][ld]. */
int ls_scale_latents(const float* lat, int64_t P, float inv_scaling, float shift, uint16_t* z, int32_t ld,
                     void* stream);

/* paste_surrounding_pixels_back + pixel_values_to_images (lipsync_pipeline.py:327-341):
 * out = dec * (1 - keep) + pix * keep; dec / pix bf16 NHWC [F][R][R][ld*];
 * out_nchw fp32 [F][3][R][R] (may be NULL), out_u8 uint8 [F][R][R][3] (may be NULL). */
int ls_paste_back(const uint16_t* dec, int32_t ld_dec, const uint16_t* pix, int32_t ld_pix, const float* mask,
                  int32_t F, int32_t R, float* out_nchw, uint8_t* out_u8, void* stream);

/* y[r, c] = x[r, c] + table[r % table_rows, c] (table fp32 [table_rows][C]): the
 * whisper positional-embedding add (whisper/model.py:155). */
int ls_add_rows(const uint16_t* x, int64_t rows, int32_t C, int32_t ldx, const float* table, int32_t table_rows,
                uint16_t* y, int32_t ldy, void* stream);

/* Tuning / A-B switches for ls_conv2d (process-wide, host side only):
 * key 1 = force the register-staged kernel (1) instead of the LDS-DMA one;
 * key 2 = force tile 0 auto, 1 128x128, 2 128x64, 3 64x64, 4 128x32; key 3 = split-K with key 2;
 * key 4 = ablation (1 skip MFMA, 2 skip operand DMA, 4 skip the output store, 8 the general epilogue
 * arithmetic; timing only); key 5 = DMA K-tile depth 32 or 64;
 * key 6 = row-block GEMM on / off; key 7 = its K = 640 instances on / off; key 8 = halo-tile 3x3
 * conv on / off (ABI 12); key 9 = d = 40 self attention on the 32x32x16 kernel (ABI 12);
 * key 10 = 256x128 3-stage tile for the short-K linears; key 11 = register-staged operand loads in
 * the tiled GEMM; key 12 = halo pieces over the read pixels only (default on); key 13 = 128-channel
 * halo tiles where 160 also divides N; key 14 = 1x1 GEMM with A straight into registers.  Keys 10, 11,
 * 13, 14 are measured-slower A/B options; key 15 = K = 640 row-block GEMM with two
 * 16-row fragments per wave (256-row blocks; default on); key 16 = 128-column halo tiles on 16 x 8
 * patches, two blocks per CU, for Cin <= 256 (default on; off: 16 x 16, one block per CU);
 * key 17 = ls_ff_chain rows per wave: 1 = 16 rows (default), 2 = 32 rows, one wave per SIMD
 * (measured slower; diagnostics build only); key 18 = nearest-x2 upsample convs on the halo-tile
 * kernel (default on; off: the tiled gather); key 19 = the narrow 16-column halo tile for 3x3 convs
 * with N = 8 / 16 (the VAE's conv_out with conv_norm_out + SiLU fused; default on; off: the tiled
 * 128 x 32 GEMM); key 20 = the K = 640 residual linears on the row-block GEMM (default off: the
 * tiled 128 x 160 kernel). */
int ls_set_tuning(int32_t key, int32_t value);

/* Diagnostics: workgroups per CU the runtime can co-schedule for a GEMM kernel
 * instance (hipOccupancyMaxActiveBlocksPerMultiprocessor with its dynamic LDS):
 * which 1 = 128x160 DMA tile, 2 = 256x256 8-wave tile, 3 = 128x128 DMA tile. */
int ls_gemm_occupancy(int32_t which);

/* Whisper log-mel spectrogram (whisper/audio.py:92-125: torch.stft n_fft 400, hop
 * 160, periodic Hann, centre/reflect padding, last frame dropped, |X|^2, mel
 * filterbank, log10 clamp 1e-10, clip-global max-8 floor, (x + 4) / 4).
 * audio fp32 [n_samples] (16 kHz mono), filters fp32 [n_mels][201];
 * out bf16 [t_pad][n_mels] frame-major, T = n_samples / 160 frames, zero for
 * T <= t < t_pad (the transcribe segment pad, whisper/audio.py pad_or_trim).
 * Workspace: ls_log_mel_workspace_bytes. */
size_t ls_log_mel_workspace_bytes(int64_t n_samples, int32_t n_mels);
int ls_log_mel(const float* audio, int64_t n_samples, const float* filters, int32_t n_mels, int64_t t_pad,
               uint16_t* out, void* workspace, size_t workspace_bytes, void* stream);

/* Audio2Feature.feature2chunks / get_sliced_feature (audio2feature.py:24-49, 85-100):
 * feat bf16 rows [T][layers][C] with row stride ld_row; chunk i, row j =
 * feat[clamp(int(i * 50 / fps) - 2 * left + j / layers, 0, T - 1)][j % layers];
 * out [n_chunks][(left + right + 1) * 2 * layers][C], bf16 or fp32 (out_f32). */
int ls_audio_chunks(const uint16_t* feat, int64_t ld_row, int32_t T, int32_t layers, int32_t C, int32_t n_chunks,
                    double fps, int32_t left, int32_t right, void* out, int32_t out_f32, void* stream);

/* ---- paste-back warp (restore_video), SURVEY.md §8(f) row 1 ---------------------- */

/* torchvision resize(face, (out_h, out_w), antialias=True) (aten _upsample_bilinear2d_aa)
 * followed by (x / 2 + 0.5).clamp(0, 1) * 255 -> uint8, as LipsyncPipeline.restore_video
 * does per face (lipsync_pipeline.py:348-354).  faces fp32 NCHW [N][3][in_h][in_w];
 * out uint8 HWC [N][out_h][out_w][3]. */
int ls_face_resize_u8(const float* faces, int32_t N, int32_t in_h, int32_t in_w, int32_t out_h, int32_t out_w,
                      uint8_t* out, void* stream);

/* Constant tables of the warp (OpenCV initInterTab2D Lanczos4 fixed-point coefficients,
 * getGaussianKernel(2 w + 1, 0) for w = 0..w_edge_max), computed on the host and copied
 * into the caller's device buffer `tables` of ls_restore_tables_bytes(w_edge_max) bytes.
 * Synchronises `stream` (initialisation only; not capturable). */
size_t ls_restore_tables_bytes(int32_t w_edge_max);
int ls_restore_init_tables(void* tables, int32_t w_edge_max, void* stream);

/* AlignRestore.restore_img (affine_transform.py:85-115, upscale_factor 1) for N frames,
 * in place: frames uint8 [N][H][W][3]; faces uint8 [N][fh][fw][3] (the resized faces);
 * warp fp64 [N][6] = the frame->face matrix cv2.warpAffine iterates with (the inverse of
 * invertAffineTransform(affine_matrix), in warpAffine's own operation order);
 * roi int32 [N][4] (x0, y0, x1, y1), 16-byte aligned: the frame box outside which the
 * soft mask is 0 (width <= roi_w, height <= roi_h); w_edge_max bounds
 * int(sqrt(mask area)) // 20 and must not exceed the tables' bound.
 * Per pixel of the ROI: warpAffine(ones) bilinear -> 2x2 erode -> area (fp64) ->
 * (2 w_edge)^2 erode -> (2 w_edge + 1)^2 Gaussian (BORDER_REFLECT_101) -> soft;
 * frame = trunc(soft * mask_e * lanczos4(face) + (1 - soft) * frame).
 * Workspace: ls_restore_workspace_bytes(N, roi_h, roi_w). */
size_t ls_restore_workspace_bytes(int32_t N, int32_t roi_h, int32_t roi_w);
int ls_restore_frames(uint8_t* frames, int32_t N, int32_t H, int32_t W, const uint8_t* faces, int32_t fh, int32_t fw,
                      const double* warp, const int32_t* roi, int32_t roi_h, int32_t roi_w, int32_t w_edge_max,
                      const void* tables, void* workspace, size_t workspace_bytes, void* stream);

/* ---- face-alignment ingest + mask resize, SURVEY.md §8(f) row 2 / §8(a) a3 ----------- */

/* cv2.resize(img, (dst_w, dst_h), interpolation=INTER_LANCZOS4) for N uint8 HWC images
 * with C (1..4) interleaved channels: load_fixed_mask's mask.png resize
 * (image_processor.py:31-36) and the aligned face's resize to the resolution
 * (image_processor.py:141).  OpenCV's generic resize path (resize.cpp resizeGeneric_
 * with HResizeLanczos4 / VResizeLanczos4: int16 coefficients saturate_cast(c * 2048),
 * taps clamped to the image, (sum + 2^21) >> 22); dst_h == src_h and dst_w == src_w is
 * a copy, as in cv::resize.  The per-axis tables are built on the host and copied into
 * `workspace` (ls_resize_lanczos4_workspace_bytes): this call synchronises `stream`
 * (one-off preprocessing; not capturable). */
size_t ls_resize_lanczos4_workspace_bytes(int32_t dst_h, int32_t dst_w);
int ls_resize_lanczos4_u8(const uint8_t* src, int32_t N, int32_t src_h, int32_t src_w, int32_t C, uint8_t* dst,
                          int32_t dst_h, int32_t dst_w, void* workspace, size_t workspace_bytes, void* stream);

/* AlignRestore.align_warp_face (affine_transform.py:53-70): cv2.warpAffine(frame, M,
 * (out_w, out_h), INTER_LANCZOS4, BORDER_CONSTANT, border_value) for N uint8 RGB
 * frames [N][H][W][3] -> out [N][out_h][out_w][3].  warp fp64 [N][6] is the
 * dst->src matrix warpAffine iterates with (the inverse of M, in warpAffine's own
 * operation order); tables = the buffer of ls_restore_init_tables (its Lanczos-4
 * table). */
int ls_align_warp_u8(const uint8_t* frames, int32_t N, int32_t H, int32_t W, const double* warp, int32_t out_h,
                     int32_t out_w, int32_t border_value, const void* tables, uint8_t* out, void* stream);

int ls_abi_version(void);
const char* ls_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* LS_HIP_H */

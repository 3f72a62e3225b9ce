/* libpdm — MI355X (gfx950) HIP implementation of the Panoptic-Diffusion sampling hot path.
 *
 * C ABI only: plain pointers, sizes and a hipStream_t (passed as void*).  All device buffers are owned
 * by the caller (torch tensors on the Python side); a pdm_uvit handle stores configuration and the
 * device addresses of the caller-owned packed weights, nothing else.  Every entry point is
 * stream-ordered and asynchronous; it returns 0 on success or a non-zero status, with the message in
 * pdm_last_error() (thread-local).  No entry point allocates, frees or synchronises, so all of them can
 * be captured into a HIP graph.
 *
 * The reference has no FFI: its boundary is Python.  Each entry point below names
 * the reference call it replaces; the Python package panopticdiffusionmodels_amd keeps the reference
 * signatures above it (get_nnet / nnet(...) / NoiseScheduleVP / DPM_Solver.sample / decode).
 */
#ifndef PDM_H
#define PDM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PDM_OK 0
#define PDM_ERR_ARG 1     /* invalid argument / unsupported shape (Python: ValueError) */
#define PDM_ERR_HIP 2     /* HIP runtime error (Python: RuntimeError) */
#define PDM_ERR_STATE 3   /* missing weight / not prepared (Python: RuntimeError) */

#define PDM_F32 0
#define PDM_BF16 1
#define PDM_FP8 2     /* OCP e4m3 bytes (MXFP8 data) */
#define PDM_E8M0 3    /* MXFP8 block-scale dwords: [K/128][rows], byte j of (kt, r) = exponent of block kt*4 + j */

/* GEMM epilogues */
#define PDM_EPI_BF16 0   /* out_bf16 = A W^T + b */
#define PDM_EPI_GELU 1   /* out_bf16 = gelu_erf(A W^T + b) */
#define PDM_EPI_F32 2    /* out_f32 (+)= A W^T + b, optional bf16 copy into out_bf16 */

const char* pdm_last_error(void);
int pdm_version(void);
int pdm_device_arch(char* buf, int len);
/* Tile-policy overrides for A/B measurement (0 = automatic; the default everywhere).
 *   GEMM: 1 = 128x128, 2 = 256x256 BK32 ring, 3 = 256x256 BK64 ring, 4 = 256x256 8-phase staggered,
 *         5 / 6 / 7 = 256x256 LDS-DMA descriptor kernel (schedules 0 / 1 / 2; 7 is the automatic choice for
 *         N >= 256 where 11 does not apply), 8 = its 256x128 half-N tile, 9 = a 512x128 tall tile (both N <= 128,
 *         bf16 / fp32 epilogues), 11 = the persistent 256x256 kernel (schedule 2 run across tiles; bf16 / GELU /
 *         bf16-residual epilogues, K >= 256: the automatic choice where it applies, else 7)
 *   attention: 1 = streamed K/V per 64-query block, 2 / 3 = head-resident K/V with 2 / 3 query tiles per wave,
 *              4 = head-resident v2 (Dh 64), 7 = head-resident Dh 72 (64 + 8 split); 5/6, 8/9 = their load-only /
 *              math-only timing variants (wrong results); 11 = persistent head-resident Dh 64 with the next head's
 *              K/V streamed in during the last pass (12 / 13 its load-only / math-only timing variants); 14 = the
 *              same for Dh 72 (15 / 16 timing variants) */
/* GEMM tile-order knob: raster = row panels per tile group inside an XCD's tile range (0 = row-major);
 * dbg_tile0 bit 0 stages every tile's operands from tile (0, 0); bit 1 lets a bf16 GEMM run with no output (mainloop +
 * LDS staging only); bit 4 skips every 256-tile epilogue -- timing experiments, results are wrong; bit 7 (tests):
 * a stream-K tail never takes its predecessor's hand-off and recomputes the tile (results unchanged) */
int pdm_set_gemm_tuning(int raster, int dbg_tile0);
int pdm_set_gemm_algo(int algo);
/* stream-K policy of the persistent GEMM (the last, partly filled wave of 256 x 256 tiles spread over all CUs as
 * K-step ranges; results bit-identical to whole tiles): 0 off (default: measured slower at every U-ViT shape,
 * DESIGN.md §4c), 1 auto (where the last wave is < 97 % full), 2 wherever it applies; + 4: standalone pdm_gemm calls
 * take it too.  The flag blocks and the 64 MiB fp32 slab are library-owned, one set per (device, stream), allocated
 * on first use outside a stream capture (a forward captured without one keeps whole tiles) */
int pdm_set_gemm_sk(int mode);
/* number of stream-K GEMM launches issued by this process so far (host-side count) */
long long pdm_gemm_sk_launches(void);
/* stream-K diagnostics gathered while pdm_set_gemm_tuning bit 8 is set: out3 = {tails run, hand-offs not taken,
 * summed poll time in 10 ns ticks}; reading clears them (synchronises the device) */
int pdm_gemm_sk_stats(unsigned long long* out3);
/* diagnostics of -DPDM_G8S_SEG builds (tools/g8s_seg.py): shader cycles per persistent-GEMM main-loop segment summed
 * over workgroups -- wave 0 [0..11] and wave 4 [12..23] (phase A: fragment reads, refill issue, vmcnt wait, barrier,
 * MFMAs, barrier; phase B: the same) -- and the workgroup count [24]; reading clears them.  Zeros in production builds
 * (a measurement hook with no reference counterpart) */
int pdm_gemm_seg_stats(unsigned long long* out25);
int pdm_set_attention_algo(int algo);

/* ---- network handle: libs/uvit.py:138-230 UViT, libs/uvit_t2i.py:258-525 UViT (t2i) -------------- */
typedef struct pdm_uvit pdm_uvit;

typedef struct pdm_uvit_cfg {
  int img_size, patch_size, in_chans, embed_dim, depth, num_heads;
  int mlp_hidden;          /* int(embed_dim * mlp_ratio) */
  int num_classes;         /* <= 0: unconditional (no label token) */
  int conv;                /* final 3x3 conv present (applied by pdm_stage_epilogue, not by forward) */
  int skip;                /* long skips present */
  int qkv_bias;
  int mlp_time_embed;      /* must be 0 (all reference configs) */
  /* t2i (libs/uvit_t2i.py) */
  int t2i;
  int clip_dim, num_clip_token;
  int separate, enable_panoptic, num_panoptic_class;
  /* 1: MXFP8 block linears (BASELINE configs[4] "fp8 MFMA"; class-conditional / unconditional U-ViT only,
   * embed_dim and mlp hidden multiples of 128).  attn.qkv / attn.proj / mlp.fc1 / mlp.fc2 weights are then
   * PDM_FP8 [out][in] with a "<key>_scale" PDM_E8M0 [in/128][out] companion (qkv / fc1: quantised after the
   * norm fold); every activation feeding them is MXFP8, written by the epilogue that produces it.  Everything
   * else (skip_linear, whose output replaces the residual stream, attention, heads) stays as in the bf16 path.
   * The residual-stream operands of the LayerNorm-fused Linears are MXFP8 of x minus its 256-column group means
   * and those Linears also take "<key minus .weight>.ln_gcol" bf16 [out][16] (pdm_gemm_args.ln_gcol). */
  int fp8;
  /* with fp8: which block Linears are MXFP8, bit 0 attn.qkv, 1 attn.proj, 2 mlp.fc1, 3 mlp.fc2; 0 = all four.
   * Supported: 0 / 0xF, and 0xB (mlp.fc1 in bf16: the forward error of the H/4 net drops from 6.9e-2 to
   * 5.0e-2 rel-L2, tools/fp8_ablation.py).  A bf16 Linear's weight is registered as in the bf16 path. */
  int fp8_linears;
  /* residual stream precision between blocks, for every forward (class-conditional, t2i, MXFP8).  0 (default):
   * bf16 -- a performance choice, NOT the reference's numerics: under autocast the reference's x stays fp32
   * through the in-blocks and the mid-block (x + pos_embed promotes it, libs/uvit.py:212) and is half precision
   * (fp16) only after each out-block's skip_linear; 1: fp32 throughout (closer to the reference: L/2 forward
   * 5.7e-3 vs 7.5e-3 rel-L2 to the fp32 oracle). */
  int residual_fp32;
} pdm_uvit_cfg;

/* replaces utils.get_nnet (utils.py:291-299) + UViT.__init__ (libs/uvit.py:139-195) */
int pdm_uvit_create(const pdm_uvit_cfg* cfg, pdm_uvit** out);
int pdm_uvit_destroy(pdm_uvit* h);
/* replaces load_state_dict (eval_ldm_discrete.py:46): register the device address of one packed weight
 * under its reference state_dict key.  Linear weights bf16 [out, in]; everything
 * else fp32.  decoder_pred(.mask).weight is bf16 padded to a multiple of 16 rows.  attn.qkv (weight,
 * ln_colsum, ln_bias) is norm1-folded and its q rows (0 .. embed_dim) are scaled by Dh^-0.5 * log2(e), the
 * softmax scale in base 2 (libs/uvit.py:64,73): the attention kernels then exponentiate the scores directly. */
int pdm_uvit_set_param(pdm_uvit* h, const char* name, const void* dev_ptr, int dtype, long long numel);
/* enumerate the keys the handle expects (name, dtype, element count) */
int pdm_uvit_param_count(const pdm_uvit* h);
int pdm_uvit_param_info(const pdm_uvit* h, int i, char* name, int len, int* dtype, long long* numel);
/* checks every required key is registered with the expected dtype / size */
int pdm_uvit_validate(pdm_uvit* h);
int pdm_uvit_workspace_size(const pdm_uvit* h, int rows, size_t* bytes);

/* replaces UViT.forward (libs/uvit.py:201-230) up to and including unpatchify: writes the pre-final-conv
 * output eps_pre [rows, C, H, W] fp32.  x [rows, C, H, W] fp32, t [rows] fp32 (as the net receives it),
 * y [rows] int64 or NULL.  The final conv (if any) + CFG are applied by pdm_stage_epilogue. */
int pdm_uvit_forward(pdm_uvit* h, const float* x, const float* t, const int64_t* y, float* eps_pre, int rows,
                     void* workspace, size_t workspace_bytes, void* stream);

/* replaces UViT(t2i).forward (libs/uvit_t2i.py:378-525).  context [rows, num_clip_token, clip_dim] fp32,
 * mask_token [rows, K, H, W] fp32 or NULL.  Writes eps_pre [rows, C, H, W] and (if mask_token and not
 * use_ground_truth) mask_pre [rows, K, H, W] (pre-final-conv, pre-tanh). */
int pdm_uvit_t2i_forward(pdm_uvit* h, const float* x, const float* t, const float* context,
                         const float* mask_token, int use_ground_truth, float* eps_pre, float* mask_pre,
                         int rows, void* workspace, size_t workspace_bytes, void* stream);

/* Profiling hook (bench.py roofline): when enabled with max_launches > 0, every GEMM launch of the
 * following forwards is bracketed by HIP events recorded on the launch stream (events are created here,
 * the only entry points that create resources; profile_read synchronises on them).  profile_read returns,
 * for the most recent forward, each GEMM's duration (ms) and algorithmic FLOPs (2 M N K). */
int pdm_uvit_profile(pdm_uvit* h, int max_launches);
int pdm_uvit_profile_read(pdm_uvit* h, float* ms, double* flops, int cap, int* n);

/* ---- solver / guidance epilogue ------------------------------------------------------------------
 * final_layer conv3x3 (libs/uvit.py:183,229) + CFG combine (eval_ldm_discrete.py:77, eval_ldm.py:71,
 * train_t2i_discrete.py:429-431) + optional tanh (libs/uvit_t2i.py:513) + the DPM-Solver stage
 * arithmetic (dpm_solver_pp.py:310-328 x0 conversion, 420-829 linear combinations).  Per element:
 *   act(v) = tanh(v) if act_tanh else v   (per call, before the combine: libs/uvit_t2i.py:513 then 429)
 *   e = act(conv(pre[b])) (conv skipped if conv_w == NULL)
 *   if has_uncond: e += cfg_scale * (e - act(conv(pre[b+B])))
 *   m = ax * xin + ae * e   (xin may be NULL -> m = ae * e);   m_out = m (if not NULL)
 *   x_out = cm * m + sum_i c[i] * T[i]   (if not NULL; also copied to x_out2 / x_out3 when not NULL:
 *   the next model input is written straight into both CFG halves of the batched input)            */
typedef struct pdm_stage_epilogue_args {
  const float* pre;
  const float* conv_w; const float* conv_b;
  int B, C, H, W;
  int has_uncond; float cfg_scale;
  int act_tanh;
  const float* xin; float ax, ae;
  float* m_out;
  int n_terms; const float* T[6]; float c[6]; float cm;
  float* x_out; float* x_out2; float* x_out3;
} pdm_stage_epilogue_args;
int pdm_stage_epilogue(const pdm_stage_epilogue_args* a, void* stream);

/* out = sum_i c[i] * T[i], n fp32 elements (generic DPM_Solver update path, dpm_solver_pytorch.py:301-432) */
int pdm_lincomb(float* out, int n_terms, const float* const* T, const float* c, long long n, void* stream);

/* ---- individual kernels (exposed for parity tests and the generic Python path) -------------------- */
/* nn.Linear on bf16 rows: libs/uvit.py:61-63,117; libs/timm.py:101-104.  W [N][K] bf16. */
int pdm_gemm_bf16(const void* A1, int lda1, const void* A2, int lda2, int K1, const void* W, const float* bias,
                  int M, int N, int K, int epi, void* out_bf16, int ldo, float* out_f32, int ldr, int accumulate,
                  void* stream);
/* Fused LayerNorm GEMM (libs/uvit.py:100,103 norm1 -> qkv, norm2 -> fc1).  Producer (epi = fp32, stats_out
 * non-null): per row and 256-column group t, (sum, M2 about the group mean) of the stored fp32 values ->
 * stats_out[row][ceil(N/256)][2].  Consumer (epi = bf16 / GELU, ln_stats non-null): A = bf16(x) un-normalised,
 * W = W_ref * diag(norm.weight), ln_colsum[n] = sum_k W[n][k], bias = W_ref norm.bias (+ b_ref):
 *   out = rstd * (A W^T - mean * ln_colsum) + bias,  mean / rstd merged from the row's ceil(K/256) partials. */
int pdm_gemm_bf16_ln(const void* A, int lda, const void* W, const float* bias, int M, int N, int K, int epi,
                     void* out_bf16, int ldo, float* out_f32, int ldr, int accumulate, float* stats_out,
                     const float* ln_stats, const float* ln_colsum, float ln_eps, void* stream);
/* LayerNorm partials of fp32 rows (as above) + optional bf16 copy xb [rows][D] */
int pdm_rowstats(const float* x, int ldx, int rows, int D, void* xb, float* stats, void* stream);
/* General GEMM entry (every operand / epilogue option of the kernels; the fixed-signature entries above are
 * shorthands).  fp8 != 0: A1 / W are MXFP8 e4m3 bytes with E8M0 block-scale dwords a_scale [K/128][a_scale_ld]
 * / w_scale [K/128][w_scale_ld] (byte j of dword (kt, row) scales K block kt*4 + j, 32 elements), computed on
 * v_mfma_scale_f32_16x16x128_f8f6f4.  out_fp8 != NULL: the epilogue also writes its stored values in MXFP8
 * (e4m3 [M][ldo8] + scales [N/128][out_scale_ld], exponent ceil(log2(amax/448)) per 32 columns).  LayerNorm
 * producer / consumer fields as pdm_gemm_bf16_ln. */
typedef struct pdm_gemm_args {
  const void* A1; int lda1;
  const void* A2; int lda2; int K1;
  const void* W; int ldw;
  const float* bias;
  int M, N, K;
  void* out_bf16; int ldo;
  float* out_f32; int ldr; int accumulate;
  float* stats_out;
  const float* ln_stats; const float* ln_colsum; float ln_eps;
  int fp8;
  const unsigned* a_scale; int a_scale_ld;
  const unsigned* w_scale; int w_scale_ld;
  void* out_fp8; int ldo8;
  unsigned* out_scale; int out_scale_ld;
  /* group-centred MXFP8 LayerNorm operands.  mx_center (fp32 epilogue with stats_out and out_fp8): the MXFP8
   * copy holds x - mu_t, mu_t = stats_out's sum / width of the row's 256-column group t.  ln_gcol (fp8
   * consumer with ln_stats): A holds such a centred copy; ln_gcol [N][16] bf16 = per column n the group sums
   * c_t[n] = sum_{k in group t} W[n][k] of the dequantised weight as bf16 pairs (hi at [t], lo at [8 + t]);
   *   out = rstd * (A W^T + sum_t (mu_t - mean) c_t) + bias   (ln_colsum then unused) */
  int mx_center;
  const void* ln_gcol;
  /* epi = 3 (residual on a bf16 stream): out_bf16 = bf16(A W^T + bias (+ res_in when accumulate)), LayerNorm
   * partials of the rounded values to stats_out; res_in [M][ldri] bf16 may alias out_bf16 */
  const void* res_in; int ldri;
  /* epi = 2 with accumulate: the fp32 residual is read from res_f32 [M][ldrf] instead of out_f32 (out of place:
   * out_f32 = res_f32 + A W^T + bias); null = in place */
  const float* res_f32; int ldrf;
  /* row gather of A1: row m of the product reads A1 row (m / a_rows_per_group) * a_group_stride + m %
   * a_rows_per_group (0: contiguous) -- the t2i injection reads the image rows of the mask-stream output */
  int a_rows_per_group; int a_group_stride;
  /* epi = 3: second output of the rounded rows at out2 row (m / out2_rows_per_group) * out2_group_stride + m %
   * out2_rows_per_group (stride ldo) and, with stats_out, their LayerNorm partials at the same row of stats_out2
   * (libs/uvit_t2i.py:426/443/459: the new x straight into the image half of the next mask-stream input) */
  void* out2; int out2_rows_per_group; int out2_group_stride;
  float* stats_out2;
} pdm_gemm_args;
int pdm_gemm(const pdm_gemm_args* a, int epi, void* stream);
/* Two GEMMs with the same epilogue, N, K and strides (different operands, rows and outputs) as ONE grouped launch of
 * the persistent kernel where it takes both (the t2i image- and mask-stream Linears of a layer), else the two
 * launches in order; results identical to two pdm_gemm calls either way. */
int pdm_gemm_pair(const pdm_gemm_args* a, const pdm_gemm_args* b, int epi, void* stream);
/* sizeof(pdm_gemm_args) as compiled into the library (binding layout check) */
int pdm_gemm_args_size(void);
/* Implicit-GEMM conv3x3 (stride 1, pad 1) on NHWC bf16 input [B, H>>up, W>>up, Cin] (up = 1: the nearest-x2
 * upsample of libs/autoencoder.py:35-50 folded into the addressing); Wt [N][9*Cin] in (ky, kx, ci) order;
 * output rows = output pixels (b, y, x), N channels (libs/autoencoder.py ResnetBlock conv1/conv2, Upsample.conv) */
int pdm_gemm_conv3x3_bf16(const void* in, int B, int H, int W, int Cin, int up, const void* Wt, const float* bias,
                          int N, int epi, void* out_bf16, float* out_f32, int accumulate, void* stream);
/* batch independent GEMMs (operand strides in elements; the decoder AttnBlock's q k^T and p v, autoencoder.py:177-188) */
int pdm_gemm_batched_bf16(const void* A, int lda, long long sA, const void* W, int ldw, long long sW,
                          const float* bias, int M, int N, int K, int batch, int epi, void* out_bf16, int ldo,
                          long long sO, float* out_f32, int ldr, long long sR, int accumulate, void* stream);
/* nn.LayerNorm (libs/uvit.py:100,103,180): fp32 rows -> bf16 rows */
int pdm_layernorm(const float* x, int ldx, const float* gamma, const float* beta, void* y, int ldy, int rows, int D,
                  float eps, void* stream);
/* Attention core (libs/uvit.py:66-92 minus the two Linears): packed qkv bf16 -> bf16 */
int pdm_attention(const void* qkv, int ldq, void* out, int ldo, int B, int L, int H, int Dh, float scale,
                  void* stream);
/* the same with q already multiplied by Dh^-0.5 * log2(e) (what the U-ViT forward's qkv GEMM produces: its
 * attn.qkv q rows are packed pre-scaled), so the softmax is taken as exp2 of the scores directly */
int pdm_attention_log2(const void* qkv, int ldq, void* out, int ldo, int B, int L, int H, int Dh, void* stream);
/* fp32 -> bf16 conversion (round to nearest even); n == 0 is a no-op (null pointers allowed) */
int pdm_f32_to_bf16(const float* x, void* y, long long n, void* stream);
/* MXFP8 quantisation of rows x [rows][ldx] (dtype PDM_F32 or PDM_BF16, K % 32 == 0) -> e4m3 q [rows][ldq] and
 * E8M0 scale dwords s [ceil(K/128)][s_ld >= rows]: exponent ceil(log2(amax/448)) per 32 columns, RNE data (the
 * quantiser of every MXFP8-emitting epilogue; in the fp8 forward it turns the attention output into the
 * attn.proj operand) */
int pdm_mx_quantize(const void* x, int dtype, int ldx, int rows, int K, void* q, int ldq, unsigned* s, int s_ld,
                    void* stream);

/* ---------------------------------------------------------------------------------------------------
 * KL-f8 decoder: FrozenAutoencoderKL.decode (libs/autoencoder.py:446-450) = z / scale_factor ->
 * post_quant_conv -> Decoder.forward (libs/autoencoder.py:303-409).  Weights are registered under the
 * reference state_dict keys with these repacks (done by libs/autoencoder.py on the Python side):
 *   3x3 convs (except decoder.conv_in): bf16 [Cout][3][3][Cin]   (ky, kx, ci order)
 *   decoder.conv_out: as above, padded to 4 output rows (bias padded to 4)
 *   mid.attn_1.{q,k,v}: packed into "decoder.mid.attn_1.qkv.weight" bf16 [3C][C] + ".qkv.bias" f32 [3C]
 *   proj_out / nin_shortcut (1x1): bf16 [Cout][Cin]
 *   post_quant_conv, decoder.conv_in, norms, biases: fp32 in the reference layout
 * Input z: fp32 [B, 4, h, w] (NCHW); output: fp32 [B, out_ch, 8h, 8w] (NCHW), not clamped. */
typedef struct pdm_decoder pdm_decoder;

typedef struct pdm_decoder_cfg {
  int ch;              /* 128 */
  int ch_mult[4];      /* (1, 2, 4, 4) */
  int num_levels;      /* len(ch_mult) */
  int num_res_blocks;  /* 2 (the up path runs num_res_blocks + 1 blocks per level) */
  int z_channels;      /* 4 */
  int out_ch;          /* 3 */
  int latent_size;     /* h = w of z: 32 (256x256 images) or 64 (512x512) */
  float scale_factor;  /* 0.18215 (libs/autoencoder.py:419) */
} pdm_decoder_cfg;

int pdm_decoder_create(const pdm_decoder_cfg* cfg, pdm_decoder** out);
int pdm_decoder_destroy(pdm_decoder* d);
int pdm_decoder_param_count(const pdm_decoder* d);
int pdm_decoder_param_info(const pdm_decoder* d, int i, char* name, int len, int* dtype, long long* numel);
int pdm_decoder_set_param(pdm_decoder* d, const char* name, const void* dev_ptr, int dtype, long long numel);
int pdm_decoder_workspace_size(const pdm_decoder* d, int batch, size_t* bytes);
int pdm_decoder_decode(pdm_decoder* d, const float* z, float* img, int batch, void* workspace,
                       size_t workspace_bytes, void* stream);
/* GroupNorm statistics from the producing convolution / linear epilogues (default 1); 0 = a separate statistics
 * pass over every GroupNorm input (A/B and parity tests).  Process-wide; not thread-safe against a running decode. */
int pdm_decoder_set_gn_fusion(int on);

/* ---- output stage (utils.sample2dir, utils.py:561-640) ------------------------------------------
 * Decoded images fp32 [B, C, H, W] -> uint8 [B, H, W, C]: unpreprocess (datasets.py:104-108) followed by
 * torchvision save_image's quantisation (v * 255 + 0.5, clamp, truncate), bit-exact. */
int pdm_images_to_u8(const float* img, uint8_t* out, int B, int C, int H, int W, void* stream);
/* Analog-bit masks fp32 [B, nbits, H, W] -> ids int32 [B, H, W] = bits2int(pred_mask > 0) (utils.py:490-518)
 * and/or colour-mapped uint8 [B, H, W, 3] = colormap[id] (utils.py:532-543; colormap int32 [256][3]).
 * Either output may be NULL (not both). */
int pdm_mask_bits_to_rgb(const float* bits, int nbits, const int32_t* colormap, int32_t* ids, uint8_t* rgb, int B,
                         int H, int W, void* stream);

/* ---- CLIP text encoder: the t2i conditioning producer (libs/clip.py:13-38 FrozenCLIPEmbedder.encode =
 * transformers CLIPTextModel(input_ids).last_hidden_state, openai/clip-vit-large-patch14) -------------
 * Input: token ids int64 [B, L] (L <= max_position; the reference pads to 77 with padding="max_length");
 * output: fp32 [B, L, width].  Weights under the CLIPTextModel state_dict keys (without "text_model."), with:
 *   encoder.layers.i.self_attn.{q,k,v}_proj packed into ".self_attn.qkv.weight" bf16 [3W][W] and
 *   layer_norm1 / layer_norm2 folded into qkv / mlp.fc1 like the U-ViT blocks: ".weight" = bf16(W diag(gamma)),
 *   ".ln_colsum" f32 = row sums of that bf16 weight, ".ln_bias" f32 = W beta + b;
 *   out_proj / fc2: bf16 [N][K] + f32 bias; embeddings and final_layer_norm: fp32 in the reference layout. */
typedef struct pdm_clip pdm_clip;

typedef struct pdm_clip_cfg {
  int vocab;         /* 49408 */
  int width;         /* 768 */
  int layers;        /* 12 */
  int heads;         /* 12 (head dim 64; 32 also supported) */
  int mlp_hidden;    /* 3072 */
  int max_position;  /* 77 (<= 128) */
  float eps;         /* 1e-5 */
} pdm_clip_cfg;

int pdm_clip_create(const pdm_clip_cfg* cfg, pdm_clip** out);
int pdm_clip_destroy(pdm_clip* c);
int pdm_clip_param_count(const pdm_clip* c);
int pdm_clip_param_info(const pdm_clip* c, int i, char* name, int len, int* dtype, long long* numel);
int pdm_clip_set_param(pdm_clip* c, const char* name, const void* dev_ptr, int dtype, long long numel);
int pdm_clip_workspace_size(const pdm_clip* c, int batch, size_t* bytes);
int pdm_clip_encode(pdm_clip* c, const int64_t* ids, int batch, int L, float* out, void* workspace,
                    size_t workspace_bytes, void* stream);

/* ---- training step: LSimple (sde.py:270-279, train_ldm_discrete.py:87-90) + AdamW + EMA (train_ldm_discrete.py:
 * 159-175, utils.py:308-345) of the class-conditional / unconditional U-ViT (libs/uvit.py) and of the panoptic t2i
 * U-ViT (libs/uvit_t2i.py, separate streams: train_t2i_discrete.py:148-224, 466-473); head dim 64 (<= 608 tokens per
 * stream) or 72 (U-ViT-H, <= 415), mlp_time_embed = False ----------------------------------------------------------------------------------
 * All parameters live in one caller-owned flat fp32 buffer; pdm_train_param_info gives each reference state_dict
 * key its element offset and count (256-B aligned, ordered head / out-blocks last..first / mid / in-blocks
 * last..first / embeddings, so each block's gradients are one contiguous range).  The caller also owns a gradient
 * buffer of the same size and layout, two bf16 buffers (the working copy, n_params elements, and the transposed
 * block Linear weights, n_wt elements) and, for the optimizer, moments m, v and the EMA copy (n_params each). */
typedef struct pdm_trainer pdm_trainer;
int pdm_train_create(const pdm_uvit_cfg* cfg, pdm_trainer** out);
int pdm_train_destroy(pdm_trainer* t);
int pdm_train_param_count(const pdm_trainer* t);
int pdm_train_param_info(const pdm_trainer* t, int i, char* name, int len, long long* offset, long long* numel);
int pdm_train_sizes(const pdm_trainer* t, long long* n_params, long long* n_wt);
int pdm_train_set_buffers(pdm_trainer* t, float* params, float* grads, void* wb, void* wt);
/* bf16 working copies from the fp32 parameters (after loading them; pdm_train_adamw refreshes them itself) */
int pdm_train_refresh(pdm_trainer* t, void* stream);
int pdm_train_workspace_size(const pdm_trainer* t, int rows, size_t* bytes);
/* replaces loss = LSimple(...); loss.mean().backward() for one batch of `rows` samples: xt [rows, C, H, W] the noised
 * input, tvals [rows] the timesteps as the net receives them (n, or t * 999 for the ScoreModel), y [rows] int64 labels
 * (NULL for an unconditional net), target [rows, C, H, W] the noise.  Writes loss[rows] = mos(target - nnet(xt)) and
 * into the gradient buffer d(gscale * sum(loss)) / d(params) (gscale = 1 / rows: loss.mean()).  The forward keeps
 * its activations in the workspace (bf16 GEMM operands, fp32 residual stream). */
int pdm_train_step(pdm_trainer* t, const float* xt, const float* tvals, const int64_t* y, const float* target,
                   float* loss, int rows, float gscale, void* workspace, size_t workspace_bytes, void* stream);
/* the t2i step (a trainer created from a t2i cfg): LSimple's panoptic branch with mask_token = mask_n
 * (train_t2i_discrete.py:155-171) -- xt [rows, C, H, W] noised latent, tvals [rows] timesteps, context [rows, nctx,
 * clip_dim] CLIP tokens, mask_token [rows, K, H, W] the noised analog bits, target the latent noise, mask_target
 * [rows, K, H, W] the analog bits (int2bits * 2 - 1).  Writes loss[rows] = mos(target - eps_pred), loss_mask[rows] =
 * mos(mask_pred - mask_target) and d(gscale * sum(loss + loss_mask)) / d(params) (train_t2i_discrete.py:468-473
 * backpropagates loss_eps.mean() + loss_mask.mean()). */
int pdm_train_step_t2i(pdm_trainer* t, const float* xt, const float* tvals, const float* context,
                       const float* mask_token, const float* target, const float* mask_target, float* loss,
                       float* loss_mask, int rows, float gscale, void* workspace, size_t workspace_bytes, void* stream);
/* torch.optim.AdamW step `step` (>= 1, bias corrections 1 - beta^step) over every parameter with the gradient buffer
 * (plus grads2, same layout, when not NULL: the second lane's gradients of a batch split over two handles), then
 * ema = ema_rate * ema + (1 - ema_rate) * params (utils.ema; ema may be NULL) and the bf16 copies */
int pdm_train_adamw(pdm_trainer* t, float* m, float* v, float* ema, const float* grads2, float lr, float beta1,
                    float beta2, float eps, float weight_decay, int step, float ema_rate, void* stream);
/* the backward kernels on their own (parity tests).  pdm_wgrad: C[n][k] (+)= sum_m A[m][n] B[m][k] (bf16 A [M][lda],
 * B [M][ldb], fp32 C [N][ldc]; scratch for split-reduction partials, may be NULL).  pdm_attention_backward: softmax
 * attention over packed qkv [B*L][3*H*Dh] with output o [B*L][H*Dh] and its gradient dout -> dqkv (Dh 64, L <= 608;
 * Dh 72, L <= 415).
 * pdm_layernorm_backward: nn.LayerNorm(D) over fp32 rows x, dh the output gradient (fp32, or bf16 if dh_bf16) ->
 * dx (+= if accumulate), optional bf16 copy dxb, dgamma, dbeta (written); scratch >= (4 ceil(rows/4) + 1) 8 D bytes
 * is plenty. */
/* dW tile policy (0 = automatic: 256 x 128 for n >= 256, else 128 x 128; 128 / 256 force one, A/B timing) */
int pdm_set_wgrad_tile(int tile);
int pdm_wgrad(const void* A, int lda, const void* B, int ldb, float* C, int ldc, int M, int N, int K, int accumulate,
              float* scratch, size_t scratch_bytes, void* stream);
int pdm_attention_backward(const void* qkv, const void* o, const void* dout, void* dqkv, int B, int L, int H, int Dh,
                           void* stream);
int pdm_layernorm_backward(const float* x, const void* dh, int dh_bf16, const float* gamma, float* dx, void* dxb,
                           float* dgamma, float* dbeta, int rows, int D, int accumulate, float* scratch,
                           size_t scratch_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PDM_H */

// Internal launcher declarations shared by the kernels and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <stddef.h>
#include <stdint.h>

namespace pdm {

typedef __bf16 bf16;

// EPI_RES: the residual epilogue of EPI_F32 on a bf16 residual stream: out_bf16 = bf16(acc + bias (+ res_in))
enum { EPI_BF16 = 0, EPI_GELU = 1, EPI_F32 = 2, EPI_RES = 3 };

struct GemmArgs {
  const bf16* A1; int lda1;   // A[:, 0:K1]
  const bf16* A2; int lda2;   // A[:, K1:K] (may be null when K1 == K)
  int K1;
  const bf16* W;              // [N][K] row-major (nn.Linear weight)
  const float* bias;          // [N] or null
  int M, N, K;
  bf16* out_bf16; int ldo;    // EPI_BF16 / EPI_GELU output, or optional bf16 copy for EPI_F32
  float* out_f32; int ldr;    // EPI_F32 output (residual stream)
  int accumulate;             // EPI_F32: out_f32 += result (residual add) instead of =; EPI_RES: add res_in
  int a_rows_per_group;       // >0: A1 row m is read from (m / rpg) * a_group_stride + m % rpg
  int a_group_stride;
  int ldw;                    // W row stride (0 -> K)
  int batch;                  // >1: blockIdx.y selects A1 + z*sA, W + z*sW, out_bf16 + z*sO, out_f32 + z*sR
  long long sA, sW, sO, sR;
  // implicit-GEMM conv3x3 (stride 1, pad 1) over an NHWC bf16 A1 [B, Hs, Ws, convC]: row m = output pixel
  // (b, y, x) of an convH x convW grid, K = 9 * convC in (ky, kx, ci) order, padded taps read `zero`.
  int conv, convH, convW, convC, conv_up;   // conv_up: source is the nearest-x2 upsample (Hs = H/2)
  const bf16* zero;           // >= 256 zero bytes
  // LayerNorm fusion (norm1 -> qkv, norm2 -> fc1: libs/uvit.py:100,103,115-120), see ln_partials below.
  //  producer (EPI_F32 with stats_out): per stored row m and 256-column group t = n / 256 writes the group's
  //    (sum, M2 about the group mean) of the final fp32 values to stats_out[(m * stats_ld + t) * 2 + {0,1}]
  //  consumer (EPI_BF16 / EPI_GELU with ln_stats): A holds bf16(x) un-normalised, W = W_ref * diag(gamma),
  //    out[m, n] = rstd_m * (acc - mean_m * ln_colsum[n]) + bias[n]   (bias = W_ref beta (+ b_ref))
  //    with mean_m / rstd_m merged from the ln_D-column row's partials (Chan), eps ln_eps
  float* stats_out; int stats_ld;
  const float* ln_stats; int ln_ld; int ln_D; float ln_eps; const float* ln_colsum;
  // MXFP8 (OCP e4m3 data + one E8M0 scale per 32 consecutive K elements, the block-scaled MFMA
  // v_mfma_scale_f32_16x16x128_f8f6f4): fp8 != 0 -> A1 [M][lda1] and W [N][ldw] are e4m3 bytes (split-K, conv
  // and row gather unsupported) and a_scale / w_scale hold the E8M0 exponents as dwords
  // [K/128][a_scale_ld >= M] / [K/128][w_scale_ld >= N], byte j of dword (kt, row) = block kt*4 + j.
  int fp8;
  const unsigned* a_scale; int a_scale_ld;
  const unsigned* w_scale; int w_scale_ld;
  // MXFP8 output (any epilogue): the stored values (the bf16 / GELU result, or the fp32 residual row) also
  // quantised to e4m3 [M][ldo8] with E8M0 scales [N/128][out_scale_ld >= M] in the layout above (scale
  // 2^ceil(log2(amax/448)) per 32 columns, so no element saturates)
  unsigned char* out_fp8; int ldo8;
  unsigned* out_scale; int out_scale_ld;
  // Group-centred MXFP8 LayerNorm operands (the fp8 forward's norm1 -> qkv / norm2 -> fc1).  e4m3 keeps 3
  // mantissa bits of every element, so quantising the RAW residual row x loses the LayerNorm's signal
  // x - mean once |mean| >> std.  Instead:
  //  producer (EPI_F32 with stats_out, out_fp8 and mx_center): the MXFP8 copy holds x - mu_t, mu_t = the mean of
  //    the row's 256-column group t, i.e. exactly stats_out's sum / group width
  //  consumer (fp8, EPI_BF16 / EPI_GELU with ln_stats and ln_gcol): A = MX(x - mu_t); ln_gcol [N][16] bf16 holds
  //    per output column n the group sums c_t[n] = sum_{k in group t} W[n][k] of the dequantised weight as a
  //    bf16 pair (hi [0..7], lo [8..15], t < 8, zero padded), and
  //      out[m, n] = rstd_m * (acc + sum_t (mu_t - mean_m) * c_t[n]) + bias[n]
  //    where the rank-ceil(K/256) correction runs as one extra bf16 MFMA per accumulator with the split
  //    products hi*hi + hi*lo + lo*hi (fp32-level accuracy) and ln_colsum is unused
  int mx_center;
  const bf16* ln_gcol;
  // EPI_RES residual input [M][ldri] bf16 (may alias out_bf16: each element is read before it is written, by
  // the same thread)
  const bf16* res_in; int ldri;
  // EPI_RES second output (the 256-tile epilogue): the rounded row m is also stored at out2 row
  // (m / out2_rpg) * out2_gs + m % out2_rpg (stride ldo) and, with stats_out, its partials at the same row of
  // stats_out2 (stride stats_ld) -- the t2i injection writes the new image tokens x straight into the image half of
  // the next mask-stream input cat(x, m) (libs/uvit_t2i.py:426, 443, 459)
  bf16* out2; int out2_rpg, out2_gs;
  float* stats_out2;
  // EPI_F32 with accumulate: the residual is read from res_f32 [M][ldrf] instead of out_f32 (out of place:
  // out_f32 = res_f32 + A W^T + bias; the training forward keeps every block's input and output streams)
  const float* res_f32; int ldrf;
  // tuning knobs (set by gemm_launch): raster = row panels per tile group inside an XCD's range (0: row-major);
  // dbg_tile0 = stage every tile's operands from tile (0, 0) (timing experiments only: wrong results)
  int raster, dbg_tile0;
  // EPI_GELU activation: 0 = exact-erf GELU (nn.GELU, libs/timm.py:102), 1 = quick GELU x * sigmoid(1.702 x)
  // (the CLIP text encoder's hidden_act, transformers CLIPMLP)
  int act;
  // stream-K state of the persistent kernel (gemm.hip gemm8s_body SK = 1), both or neither: sk_flags >= 256 zeroed
  // words owned by THIS launch (one per workgroup: "head slab published"), sk_slab >= 256 x 64 Ki floats (one fp32
  // 256 x 256 accumulator tile per workgroup).  Null: whole tiles only.
  unsigned* sk_flags;
  float* sk_slab;
  // GroupNorm partials of the stored tile (the decoder's GroupNorm(32) inputs, libs/autoencoder.py Normalize): with
  // gn_part the 256-tile epilogues (gemm8d, gemm8t; EPI_F32 / EPI_BF16) write, per 256-row chunk of an image of gn_P
  // rows and per group of gn_cpg = N / 32 columns, the fp64 (sum, sum of squares) of the stored values to
  // gn_part[((b * gn_P / 256 + chunk) * 32 + g) * 2 + {0,1}] -- gn_partial_kernel's layout with 256-pixel chunks
  double* gn_part; int gn_P, gn_cpg;
};
void gemm_set_tuning(int raster, int dbg_tile0);
// stream-K policy: 0 off (default), 1 auto (where the last wave of tiles is < 97 % full), 2 wherever it applies
void gemm_set_sk(int mode);
int gemm_get_sk();
long long gemm_sk_launches();
int gemm_sk_stats(unsigned long long* out3);
int gemm_seg_stats(unsigned long long* out25);
// whether gemm_launch(p, epi) runs an epilogue that writes p.gn_part (the decoder falls back to gn_partial_kernel)
bool gemm_gn_fusable(const GemmArgs& p, int epi);
constexpr int SK_FLAG_WORDS = 256;                       // flags per launch
constexpr long long SK_SLAB_BYTES = 256LL * 65536 * 4;   // 64 MiB

// Row partials of the fused LayerNorm: X fp32 [rows, D] -> stats [rows, ceil(D/256)] (sum, M2) per 256-column
// group (+ optional bf16 copy xb [rows, D], + optional MXFP8 copy xq / xs in the GemmArgs A-operand layout).  Used where no GEMM epilogue produced them (token assembly, the
// t2i mask-stream refresh, and behind the 128-tile GEMM policy).
// The MXFP8 copy is group-centred (x - mu_t, GemmArgs::mx_center) when center != 0.
hipError_t rowstats_launch(const float* x, int ldx, int rows, int D, bf16* xb, int ldb, float* stats, int stats_ld,
                           hipStream_t stream, unsigned char* xq = nullptr, int ldq = 0, unsigned* xs = nullptr,
                           int xs_ld = 0, int center = 0);

// the same partials of bf16 rows (a bf16 residual stream: EPI_RES outputs)
hipError_t rowstats_bf16_launch(const bf16* x, int ldx, int rows, int D, float* stats, int stats_ld, hipStream_t stream);

const char* gemm_check(const GemmArgs& p, int epi);
hipError_t gemm_launch(const GemmArgs& p, int epi, hipStream_t stream);
// whether gemm_launch_pair runs the two problems as one grouped persistent launch (else two gemm_launch calls)
bool gemm_pair_groups(const GemmArgs& a, const GemmArgs& b, int epi);
// two GEMMs of the same N / K / epilogue / strides as one persistent launch when the kernel can take both (t2i image-
// and mask-stream Linears of a layer); otherwise the two launches of gemm_launch, in order
hipError_t gemm_launch_pair(const GemmArgs& a, const GemmArgs& b, int epi, hipStream_t stream);
void gemm_set_algo(int algo);

// LayerNorm over the last dim of fp32 rows -> bf16.  Row r of the output is row
// (r / rows_per_group) * group_stride + row_offset + (r % rows_per_group) of the input.
struct LayerNormArgs {
  const float* x; int ldx;
  const bf16* xb;             // bf16 input rows instead of x (the bf16 residual stream), same ldx
  const float* gamma; const float* beta;
  bf16* y; int ldy;
  int rows, D;
  int rows_per_group, group_stride, row_offset;   // row gather (final norm over patch tokens only)
  float eps;
  const float* add;           // optional fp32 rows added after the affine (gathered like x, with add_* below)
  const bf16* addb;           // the same rows in bf16 (the bf16 residual stream), instead of add
  int add_ld, add_group_stride, add_row_offset;
};
const char* layernorm_check(const LayerNormArgs& p);
hipError_t layernorm_launch(const LayerNormArgs& p, hipStream_t stream);

// Fused multi-head attention over a packed qkv buffer [B*L, 3*D] (layout (3, H, Dh) per token, as
// libs/uvit.py:71 rearranges it) -> out [B*L, D] (layout (H, Dh)).  No mask; softmax scale Dh^-1/2.
struct AttentionArgs {
  const bf16* qkv; int ldq;   // row stride of qkv (elements)
  bf16* out; int ldo;
  int B, L, H, Dh;
  float scale;
  int q_log2;                 // q already multiplied by scale * log2(e) (the U-ViT qkv weights are packed so)
};
const char* attention_check(const AttentionArgs& p);
hipError_t attention_launch(const AttentionArgs& p, hipStream_t stream);
void attention_set_algo(int algo);

// Token assembly (libs/uvit.py:201-212, libs/uvit_t2i.py:382-409):
// out[b, row] for the sequence [label?][time][context x n_ctx?][patches] + pos_embed, fp32.
struct AssembleArgs {
  const float* img;           // [B, C, Himg, Wimg]
  int C, Himg, Wimg, p;
  const float* patch_w;       // [D, C*p*p] fp32
  const float* patch_b;       // [D]
  const float* t;             // [B] timesteps (already scaled as the net receives them)
  const float* time_emb;      // optional precomputed time tokens [B, D] (mlp_time_embed); null -> sinusoid
  const int64_t* y;           // [B] labels or null
  const float* label_emb;     // [num_classes, D]
  const float* ctx_tokens;    // [B, n_ctx, D] already embedded context tokens, or null
  int n_ctx;
  const float* pos;           // [L_pos, D]; rows used = tokens of this sequence
  float* out; int ld_out;     // [B, L_total, D] with row stride ld_out (elements)
  int B, D, L_total;          // tokens per sample written
  int row0_patch;             // index of the first patch token
  int time_row;               // index of the time token (-1: none)
  int label_row;              // index of the label token (-1: none)
  int ctx_row;                // index of the first context token (-1: none)
};
const char* assemble_check(const AssembleArgs& p);
hipError_t assemble_launch(const AssembleArgs& p, hipStream_t stream);

// decoder_pred (D -> P = p*p*C, bias) on bf16 patch rows + unpatchify scatter to NCHW fp32
// (libs/uvit.py:182,225-228 and unpatchify 46-51; column order (p1, p2, C)).
struct HeadArgs {
  const bf16* x; int ldx;     // token (b, i) is row b * in_group_stride + in_row_offset + i, N = (H/p)*(W/p)
  int in_group_stride, in_row_offset;
  const bf16* W;              // [P_pad][D] (rows >= P are zero)
  const float* bias;          // [P]
  float* out;                 // [B, C, H, W]
  int B, D, C, p, Himg, Wimg, P, P_pad;
  int act_tanh;               // apply tanh after (used for no-conv mask heads only)
};
const char* head_check(const HeadArgs& p);
hipError_t head_launch(const HeadArgs& p, hipStream_t stream);

// Final 3x3 conv (optional) + classifier-free guidance + solver stage epilogue, fp32, [B, C, H, W].
//   e   = conv(pre[b])            (identity if w == null)
//   if act_tanh: e = tanh(e)              (per call, before the CFG combine)
//   if uncond: e = e + s * (e - act(conv(pre[b + B])))
//   m   = ax * xin + ae * e        (x0 conversion for data prediction; ax = 0, ae = 1 for noise)
//   m_out = m (if non-null);  x_out = sum_i c_i * T_i + cm * m  (if non-null)
struct EpilogueArgs {
  const float* pre;           // [B or 2B, C, H, W]
  const float* w; const float* bias;   // conv [C, C, 3, 3], [C]
  int B, C, Himg, Wimg;
  int has_uncond; float cfg_scale;
  int act_tanh;
  const float* xin; float ax, ae;
  float* m_out;
  int n_terms; const float* T[6]; float c[6]; float cm;
  float* x_out; float* x_out2; float* x_out3;   // x_out2/3: optional duplicate destinations
};
const char* epilogue_check(const EpilogueArgs& p);
hipError_t epilogue_launch(const EpilogueArgs& p, hipStream_t stream);

// records `msg` as pdm_last_error() (capi.hip) and returns `code`
int set_error(int code, const std::string& msg);

hipError_t cast_bf16_launch(const float* x, bf16* y, long long n, hipStream_t stream);

// MXFP8 copy of fp32 (dtype 0) / bf16 (dtype 1) rows x [rows][ldx] -> e4m3 q [rows][ldq] + E8M0 scale dwords
// s [K/128][s_ld] (GemmArgs A-operand layout); hipErrorInvalidValue on a bad shape / stride / alignment
hipError_t mxq_launch(const void* x, int dtype, int ldx, int rows, int K, unsigned char* q, int ldq, unsigned* s,
                      int s_ld, hipStream_t stream);

// out = sum_i c_i * T_i over n elements (fp32); used by the generic solver path.
hipError_t lincomb_launch(float* out, int n_terms, const float* const* T, const float* c, long long n, hipStream_t stream);

// Strided row copy fp32: dst[r*ldd + j] = src[r*lds + j], j < D, r < rows (t2i mask stream concat); row r of a
// group of rows_per_group is row (r / rpg) * group_stride + r % rpg on either side.  Optionally a second row
// (dst2 / src2, D2 floats, same row mapping) in the same launch: the row's LayerNorm partials.
hipError_t rowcopy_launch(float* dst, int ldd, const float* src, int lds, int rows, int D, int rows_per_group,
                          int dst_group_stride, int src_group_stride, hipStream_t stream, float* dst2 = nullptr,
                          int ldd2 = 0, const float* src2 = nullptr, int lds2 = 0, int D2 = 0);

}  // namespace pdm

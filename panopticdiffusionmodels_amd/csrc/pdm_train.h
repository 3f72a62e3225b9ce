// Internal declarations of the training-step kernels (train_kernels.hip) used by the trainer driver (train.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "pdm_kernels.h"

namespace pdm {

// dW[n][k] (+)= sum_m A[m][n] B[m][k]: A = dY [M][lda >= N], B = X [M][ldb >= K] (bf16, row-major over the reduction
// rows m; optional row gather m -> (m / rpg) * gs + off + m % rpg), C fp32 [N][ldc].  wgrad_launch splits the
// reduction into fp32 partials in `part` (compact [split][N][K]) summed by a second kernel when that fills the chip.
struct WgradArgs {
  const bf16* A; int lda; int a_rpg, a_gs, a_off;
  const bf16* B; int ldb; int b_rpg, b_gs, b_off;
  float* C; int ldc; long long sC;
  int M, N, K;
  int mchunk;        // set by wgrad_launch
  int accumulate;
  // optional: the bias gradient sum_m A[m][n] -> bias_out[n] (+= with bias_acc), from the A tiles the dW GEMM stages
  // anyway (one MFMA against a ones fragment per A fragment in the k0 == 0 column of tiles); sB: partial stride
  float* bias_out; int bias_acc; long long sB;
};
const char* wgrad_check(const WgradArgs& p);
extern int g_wgrad_tile;   // 0 = automatic tile, 128 / 256 = forced n-tile (timing A/B)
hipError_t wgrad_launch(const WgradArgs& p, float* part, size_t part_bytes, hipStream_t stream);

// dst[c] (+)= sum_r x[gather(r)][c] over `rows` rows of `ncols` columns (bias / pos_embed gradients)
hipError_t colsum_launch(const void* x, int is_bf16, int ld, int rows, int ncols, int rpg, int gs, int off, float* dst,
                         int accumulate, float* part, size_t part_bytes, hipStream_t stream);

// LayerNorm backward over rows of x (fp32 [.][ldx], gathered like the forward), dh = gradient of the LN output
// ([rows][lddh], fp32 or bf16, NOT gathered); dx [.][lddx] (=, or += with accumulate) at the gathered rows, optional
// bf16 copy dxb (same layout); dgamma / dbeta (=, or += with accumulate_params).  part: scratch.
struct LnBwdArgs {
  const float* x; int ldx;
  int lddh;
  const float* gamma;
  float* dx; int lddx; bf16* dxb;
  int rows, D, rpg, gs, off;
  float eps;
  int accumulate, accumulate_params;
  float* part; size_t part_bytes;
};
hipError_t ln_bwd_launch(const LnBwdArgs& p, const void* dh, int dh_bf16, float* dgamma, float* dbeta,
                         hipStream_t stream);

// exact-erf GELU forward (u -> g) and backward (dg <- dg * gelu'(u)), bf16, n % 8 == 0
hipError_t gelu_fwd_launch(const bf16* u, bf16* g, long long n, hipStream_t stream);
hipError_t gelu_bwd_launch(bf16* dg, const bf16* u, long long n, hipStream_t stream);

// softmax attention backward over the forward's packed qkv [B*L][ldq] ((3, H, 64) columns), its output o [B*L][ldo]
// ((H, 64) columns) and the output gradient dout [B*L][lddo] -> dqkv [B*L][lddq] in the qkv column layout
struct AttnBwdArgs {
  const bf16* qkv; int ldq;
  const bf16* o; int ldo;
  const bf16* dout; int lddo;
  bf16* dqkv; int lddq;
  int B, L, H, Dh;
  float scale;
};
const char* attn_bwd_check(const AttnBwdArgs& p);
hipError_t attn_bwd_launch(const AttnBwdArgs& p, hipStream_t stream);

// LSimple: loss[b] = mean (target - pred)^2 over `per` elements, dpred = d(gscale * sum_b loss[b]) / dpred; with
// tanh_bwd, pred = tanh(u) and dpred is the gradient w.r.t. u (the t2i mask head's loss_mask)
hipError_t lsimple_launch(const float* pred, const float* target, float* loss, float* dpred, int B, int per,
                          float gscale, hipStream_t stream, int tanh_bwd = 0);

// final_layer conv3x3 backward (NCHW fp32): din (data gradient), dw [C][C][3][3] and db [C] (written, not added)
hipError_t conv3x3_bwd_launch(const float* dout, const float* in, const float* w, float* din, float* dw, float* db,
                              int B, int C, int H, int W, hipStream_t stream);

// decoder_pred + unpatchify backward
struct HeadBwdArgs {
  const float* dpre;   // [B, C, Himg, Wimg] gradient of the head output (pre final conv)
  const float* W;      // [P][D] fp32 decoder_pred.weight
  bf16* dtok;          // [B*N][P_pad] gradient of the decoder_pred output (bf16, zero padded)
  float* dx;           // [B*N][D] gradient of the normalised patch tokens
  int B, D, C, p, Himg, Wimg, P, P_pad;
};
hipError_t head_bwd_launch(const HeadBwdArgs& p, hipStream_t stream);

// PatchEmbed operand: pv [B*N][ldp] bf16, k = (c, p1, p2) of the conv weight flatten, zero padded to ldp
hipError_t patchify_launch(const float* img, bf16* pv, int B, int C, int H, int W, int p, int ldp, hipStream_t stream);
// dlab[y[b]] += dx[b * L + row]
hipError_t label_scatter_launch(const float* dx, int L, int row, int D, const int64_t* y, float* dlab, int B,
                                hipStream_t stream);
// dst[gd(r)] (+)= src[gs(r)], dstb[gd(r)] = bf16(dst[gd(r)]) over `rows` rows of D fp32 (D % 4 == 0); row gather
// g(r) = (r / rpg) * gs + off + r % rpg, rpg 0 = contiguous
hipError_t rows_add_cast_launch(float* dst, bf16* dstb, int drpg, int dgs, int doff, const float* src, int srpg, int sgs,
                                int soff, int rows, int D, int accumulate, hipStream_t stream);
// dx (+)= add (add may be null), dxb = bf16(dx); n % 4 == 0
hipError_t add_cast_launch(float* dx, const float* add, bf16* dxb, long long n, hipStream_t stream);
// W fp32 [N][K] -> W^T bf16 [K][N]
hipError_t transpose_bf16_launch(const float* w, bf16* wt, int N, int K, hipStream_t stream);

struct AdamWArgs {
  float* p; const float* g; const float* g2; float* m; float* v; float* ema; bf16* pb;   // g2: optional second lane
  float lr, wd, b1, b2, eps, step_size, inv_sqrt_bc2, ema_rate;
};
hipError_t adamw_launch(const AdamWArgs& a, long long n, hipStream_t stream);

}  // namespace pdm

// C ABI of the LSimple training step (include/pdm.h "training") and its driver: the
// class-conditional / unconditional U-ViT (libs/uvit.py) forward with every activation the backward needs kept
// resident in HBM (no recomputation: at L/2 with 128 images per GPU they take ~25 GB of the 288 GB, where the
// reference needs use_checkpoint=True), the LSimple loss, the backward and the AdamW + EMA update.
//
// Parameters live in ONE caller-owned flat fp32 buffer (offsets from pdm_train_param_info, each 256-B aligned, in
// backward order: head, out-blocks last to first, mid, in-blocks last to first, embeddings, so every block's
// gradients are one contiguous range for a bucketed all-reduce), with a same-offset fp32 gradient buffer, a bf16
// working copy of everything (the forward's GEMM weights) and a bf16 transposed copy of every block Linear weight
// (W^T [in][out]: the dX GEMMs of the backward run on the forward's GEMM kernels as A = dY against W^T).
// Like the forward drivers (capi.hip) a step is a fixed sequence of stream-ordered launches on caller memory.
//
// The panoptic t2i network (libs/uvit_t2i.py with separate=True, enable_panoptic=True: train_t2i_discrete.py LSimple
// with mask_token = mask_n) runs the same blocks on two token streams -- the image stream x ([time, context, patches],
// Lx tokens) and the mask stream mx = cat(x, m) (Lm = Lx + patches tokens) -- with the mask block output's image rows
// added back into x through the layer's zero conv; its loss is loss_eps + loss_mask (mos of the tanh mask head against
// the analog bits).  Parameters the forward never uses (zero_convs.{even}, mask_embed_0) sit after every used one and
// are left out of the AdamW range, as torch.optim skips parameters without gradients.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/pdm.h"
#include "pdm_kernels.h"
#include "pdm_train.h"

using pdm::bf16;

namespace {

#define TR_HIP(call)                                                                                         \
  do {                                                                                                       \
    hipError_t e_ = (call);                                                                                  \
    if (e_ != hipSuccess) return pdm::set_error(PDM_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define TR_CHECK(msg_expr)                                 \
  do {                                                     \
    const char* m_ = (msg_expr);                           \
    if (m_) return pdm::set_error(PDM_ERR_ARG, m_);        \
  } while (0)
#define TR_TRY(x)          \
  do {                     \
    int r_ = (x);          \
    if (r_) return r_;     \
  } while (0)

size_t aup(size_t x, size_t a) { return (x + a - 1) / a * a; }

enum { KIND_F32 = 0, KIND_LINEAR = 1, KIND_HEAD = 2 };

struct TParam {
  std::string name;
  long long off, numel, alloc;
  int kind, N, K;
  long long wt_off;
};

constexpr size_t PART_BYTES = 64ull << 20;   // fp32 partial sums (split-K weight gradients, column sums, LN params)

}  // namespace

struct pdm_trainer {
  pdm_uvit_cfg cfg;
  int D = 0, H = 0, Dh = 0, Hid = 0, C = 0, p = 0, img = 0, n_patch = 0, extras = 0, L = 0, P = 0, P_pad = 0;
  int Kp = 0, Kp_pad = 0, depth = 0, nhalf = 0, nb = 0;
  // t2i: mask-stream tokens Lm, context tokens / width, mask channels K, mask head / patch-vector widths
  bool t2i = false;
  int Lm = 0, nctx = 0, clip = 0, K = 0, PK = 0, PK_pad = 0, Kpm = 0, Kpm_pad = 0;
  long long active = 0;   // AdamW range [0, active): the parameters the forward uses
  std::vector<TParam> params;
  std::map<std::string, int> idx;
  long long total = 0, wt_total = 0;
  float* Pm = nullptr;
  float* G = nullptr;
  bf16* WB = nullptr;
  bf16* WT = nullptr;

  void add(const std::string& name, long long numel, int kind = KIND_F32, int N = 0, int K = 0, long long alloc = 0) {
    TParam t{name, total, numel, alloc ? alloc : numel, kind, N, K, -1};
    if (kind == KIND_LINEAR) {
      t.wt_off = wt_total;
      wt_total += (long long)aup((size_t)numel, 64);
    }
    total += (long long)aup((size_t)t.alloc, 64);
    idx[name] = (int)params.size();
    params.push_back(t);
  }
  const TParam& prm(const std::string& n) const { return params[idx.at(n)]; }
  const float* f(const std::string& n) const { return Pm + prm(n).off; }
  float* g(const std::string& n) const { return G + prm(n).off; }
  const bf16* wb(const std::string& n) const { return WB + prm(n).off; }
  const bf16* wt(const std::string& n) const { return WT + prm(n).wt_off; }
  bool has(const std::string& n) const { return idx.count(n) != 0; }
  // block b of stream s (0: the image / only stream, 1: the t2i mask stream)
  std::string block(int b, int s = 0) const {
    const std::string sfx = s ? "_mask" : "";
    if (b < nhalf) return "in_blocks" + sfx + "." + std::to_string(b);
    if (b == nhalf) return "mid_block" + sfx;
    return "out_blocks" + sfx + "." + std::to_string(b - nhalf - 1);
  }
  bool skip_block(int b) const { return b > nhalf && cfg.skip; }
  int skip_src(int b) const { return 2 * nhalf - b; }   // in-block whose output out-block b concatenates
};

namespace {

// one token stream's saved activations (per block) and long skips
struct SW {
  int L = 0;
  std::vector<float*> X0, X1;             // per block: input (after skip_linear), after the attention residual
  std::vector<bf16*> H1, QKV, ATT, H2, U, Gl, XS;
  std::vector<bf16*> SK;                  // in-block outputs (bf16): the long skips
  std::vector<float*> DSK;                // gradients w.r.t. the long skips
};

struct TWork {
  SW I, Q;   // the image (class-conditional: the only) stream; the t2i mask stream
  float *XF, *XTMP, *PRE, *EPS, *DPRED, *DPRE, *DHN, *DX, *DX2, *PART;
  bf16 *HN, *DTOK, *PV, *DXB, *DXB2, *DH, *DG, *DATT, *DQKV;
  // t2i: per layer the bf16 mask-block output (all Lm rows; in-blocks: the mask long skip), the mask stream's
  // running input / final output and gradients, the context tokens, the mask head
  std::vector<bf16*> MOB;
  float *MXTMP, *MF, *MPRE, *MPRED, *MDPRED, *MDPRE, *DMHN, *DMX, *DMX2, *CTXF, *TMP;
  bf16 *CTXB, *MHN, *MDTOK, *PVM, *DMXB, *DMXB2;
  size_t bytes;
};

TWork tlayout(const pdm_trainer* t, int rows, char* base) {
  TWork w{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off = aup(off + bytes, 256);
    return p;
  };
  const size_t D = t->D, Mp = (size_t)rows * t->n_patch, Hd = t->Hid;
  const size_t img = (size_t)rows * t->C * t->img * t->img;
  auto stream = [&](SW& S, int L, bool own_skips) {
    const size_t M = (size_t)rows * L;
    S.L = L;
    for (int b = 0; b < t->nb; ++b) {
      S.X0.push_back((float*)take(M * D * 4));
      S.X1.push_back((float*)take(M * D * 4));
      S.H1.push_back((bf16*)take(M * D * 2));
      S.QKV.push_back((bf16*)take(M * 3 * D * 2));
      S.ATT.push_back((bf16*)take(M * D * 2));
      S.H2.push_back((bf16*)take(M * D * 2));
      S.U.push_back((bf16*)take(M * Hd * 2));
      S.Gl.push_back((bf16*)take(M * Hd * 2));
      S.XS.push_back(t->skip_block(b) ? (bf16*)take(M * D * 2) : nullptr);
    }
    for (int i = 0; i < t->nhalf; ++i) {
      S.SK.push_back(own_skips ? (bf16*)take(M * D * 2) : nullptr);
      S.DSK.push_back((float*)take(M * D * 4));
    }
  };
  stream(w.I, t->L, true);
  const size_t Mx = (size_t)rows * t->L;
  const size_t Mmax = (size_t)rows * (t->t2i ? t->Lm : t->L);
  w.XF = (float*)take(Mx * D * 4);
  w.XTMP = (float*)take(Mx * D * 4);
  w.HN = (bf16*)take(Mp * D * 2);
  w.PRE = (float*)take(img * 4);
  w.EPS = (float*)take(img * 4);
  w.DPRED = (float*)take(img * 4);
  w.DPRE = (float*)take(img * 4);
  w.DTOK = (bf16*)take(Mp * t->P_pad * 2);
  w.DHN = (float*)take(Mp * D * 4);
  w.PV = (bf16*)take(Mp * t->Kp_pad * 2);
  w.DX = (float*)take(Mx * D * 4);
  w.DX2 = (float*)take(Mx * D * 4);
  w.DXB = (bf16*)take(Mx * D * 2);
  w.DXB2 = (bf16*)take(Mx * D * 2);
  w.DH = (bf16*)take(Mmax * D * 2);
  w.DG = (bf16*)take(Mmax * Hd * 2);
  w.DATT = (bf16*)take(Mmax * D * 2);
  w.DQKV = (bf16*)take(Mmax * 3 * D * 2);
  if (t->t2i) {
    const size_t Mm = (size_t)rows * t->Lm, mimg = (size_t)rows * t->K * t->img * t->img;
    stream(w.Q, t->Lm, false);
    for (int b = 0; b < t->nb; ++b) w.MOB.push_back((bf16*)take(Mm * D * 2));
    for (int i = 0; i < t->nhalf; ++i) w.Q.SK[i] = w.MOB[i];
    w.MXTMP = (float*)take(Mm * D * 4);
    w.MF = (float*)take(Mm * D * 4);
    w.MPRE = (float*)take(mimg * 4);
    w.MPRED = (float*)take(mimg * 4);
    w.MDPRED = (float*)take(mimg * 4);
    w.MDPRE = (float*)take(mimg * 4);
    w.DMHN = (float*)take(Mp * D * 4);
    w.DMX = (float*)take(Mm * D * 4);
    w.DMX2 = (float*)take(Mm * D * 4);
    w.DMXB = (bf16*)take(Mm * D * 2);
    w.DMXB2 = (bf16*)take(Mm * D * 2);
    w.CTXF = (float*)take((size_t)rows * t->nctx * D * 4);
    w.CTXB = (bf16*)take((size_t)rows * t->nctx * t->clip * 2);
    w.TMP = (float*)take(Mx * D * 4);
    w.MHN = (bf16*)take(Mp * D * 2);
    w.MDTOK = (bf16*)take(Mp * t->PK_pad * 2);
    w.PVM = (bf16*)take(Mp * t->Kpm_pad * 2);
  }
  w.PART = (float*)take(PART_BYTES);
  w.bytes = off;
  return w;
}

struct TC {
  const pdm_trainer* t;
  hipStream_t s;
  const TWork* w;
};

int t_gemm(const TC& c, const bf16* A, int lda, const bf16* W, const float* bias, int M, int N, int K, int epi, bf16* ob,
           int ldo, float* of, int ldr, int acc, const bf16* A2 = nullptr, int lda2 = 0, int K1 = 0,
           const float* res = nullptr) {
  pdm::GemmArgs a{};
  a.res_f32 = res; a.ldrf = res ? ldr : 0;   // out-of-place residual: of = res + A W^T + bias
  a.A1 = A; a.lda1 = lda;
  a.A2 = A2; a.lda2 = lda2; a.K1 = A2 ? K1 : K;
  a.W = W; a.bias = bias;
  a.M = M; a.N = N; a.K = K;
  a.out_bf16 = ob; a.ldo = ldo;
  a.out_f32 = of; a.ldr = ldr; a.accumulate = acc;
  TR_CHECK(pdm::gemm_check(a, epi));
  TR_HIP(pdm::gemm_launch(a, epi, c.s));
  return PDM_OK;
}

int t_wgrad(const TC& c, const bf16* A, int lda, int N, const bf16* B, int ldb, int K, int M, float* C, int ldc,
            float* bias = nullptr, int a_rpg = 0, int a_gs = 0, int a_off = 0, int b_rpg = 0, int b_gs = 0,
            int b_off = 0) {
  pdm::WgradArgs a{};
  a.bias_out = bias;   // the bias gradient (column sums of A) fused into the dW GEMM
  a.A = A; a.lda = lda; a.a_rpg = a_rpg; a.a_gs = a_gs; a.a_off = a_off;
  a.b_rpg = b_rpg; a.b_gs = b_gs; a.b_off = b_off;
  a.B = B; a.ldb = ldb;
  a.C = C; a.ldc = ldc;
  a.M = M; a.N = N; a.K = K;
  TR_CHECK(pdm::wgrad_check(a));
  TR_HIP(pdm::wgrad_launch(a, c.w->PART, PART_BYTES, c.s));
  return PDM_OK;
}

int t_colsum(const TC& c, const void* x, int bf, int ld, int rows, int ncols, float* dst, int rpg = 0, int gs = 0,
             int off = 0) {
  TR_HIP(pdm::colsum_launch(x, bf, ld, rows, ncols, rpg, gs, off, dst, 0, c.w->PART, PART_BYTES, c.s));
  return PDM_OK;
}

int t_ln(const TC& c, const float* x, int rows, const float* gamma, const float* beta, bf16* y, int rpg, int gs, int off) {
  pdm::LayerNormArgs a{};
  a.x = x; a.ldx = c.t->D;
  a.gamma = gamma; a.beta = beta;
  a.y = y; a.ldy = c.t->D;
  a.rows = rows; a.D = c.t->D;
  a.rows_per_group = rpg; a.group_stride = gs; a.row_offset = off;
  a.eps = 1e-5f;
  TR_CHECK(pdm::layernorm_check(a));
  TR_HIP(pdm::layernorm_launch(a, c.s));
  return PDM_OK;
}

// LayerNorm backward: dx (+)= ..., dxb = bf16(dx), d gamma / d beta of `norm` written
int t_ln_bwd(const TC& c, const float* x, const void* dh, int dh_bf16, const std::string& norm, float* dx, bf16* dxb,
             int rows, int acc, int rpg = 0, int gs = 0, int off = 0) {
  const pdm_trainer* t = c.t;
  pdm::LnBwdArgs a{};
  a.x = x; a.ldx = t->D; a.lddh = t->D;
  a.gamma = t->f(norm + ".weight");
  a.dx = dx; a.lddx = t->D; a.dxb = dxb;
  a.rows = rows; a.D = t->D; a.rpg = rpg; a.gs = gs; a.off = off;
  a.eps = 1e-5f;
  a.accumulate = acc; a.accumulate_params = 0;
  a.part = c.w->PART; a.part_bytes = PART_BYTES;
  TR_HIP(pdm::ln_bwd_launch(a, dh, dh_bf16, t->g(norm + ".weight"), t->g(norm + ".bias"), c.s));
  return PDM_OK;
}

// one block of stream S (sid 0 image / only stream, 1 t2i mask stream) on its saved-activation buffers; the output
// (fp32, and its bf16 copy when outb) goes where the caller says: the next block's input, a skip_linear operand, ...
int block_fwd(const TC& c, const SW& S, int sid, int b, int rows, float* out, bf16* outb) {
  const pdm_trainer* t = c.t;
  const std::string pre = t->block(b, sid);
  const int D = t->D, M = rows * S.L, Hd = t->Hid;
  float* X0 = S.X0[b];
  float* X1 = S.X1[b];
  if (t->skip_block(b))   // libs/uvit.py:116-117: x = skip_linear(cat([x, skip], -1))
    TR_TRY(t_gemm(c, S.XS[b], D, t->wb(pre + ".skip_linear.weight"), t->f(pre + ".skip_linear.bias"), M, D, 2 * D,
                  pdm::EPI_F32, nullptr, 0, X0, D, 0, S.SK[t->skip_src(b)], D, D));
  TR_TRY(t_ln(c, X0, M, t->f(pre + ".norm1.weight"), t->f(pre + ".norm1.bias"), S.H1[b], M, 0, 0));
  TR_TRY(t_gemm(c, S.H1[b], D, t->wb(pre + ".attn.qkv.weight"),
                t->has(pre + ".attn.qkv.bias") ? t->f(pre + ".attn.qkv.bias") : nullptr, M, 3 * D, D, pdm::EPI_BF16,
                S.QKV[b], 3 * D, nullptr, 0, 0));
  {
    pdm::AttentionArgs a{};
    a.qkv = S.QKV[b]; a.ldq = 3 * D;
    a.out = S.ATT[b]; a.ldo = D;
    a.B = rows; a.L = S.L; a.H = t->H; a.Dh = t->Dh;
    a.scale = 1.0f / sqrtf((float)t->Dh);
    a.q_log2 = 0;
    TR_CHECK(pdm::attention_check(a));
    TR_HIP(pdm::attention_launch(a, c.s));
  }
  // x1 = x0 + proj(attn), out of place (both streams are kept for the LayerNorm backward)
  TR_TRY(t_gemm(c, S.ATT[b], D, t->wb(pre + ".attn.proj.weight"), t->f(pre + ".attn.proj.bias"), M, D, D, pdm::EPI_F32,
                nullptr, 0, X1, D, 1, nullptr, 0, 0, X0));
  TR_TRY(t_ln(c, X1, M, t->f(pre + ".norm2.weight"), t->f(pre + ".norm2.bias"), S.H2[b], M, 0, 0));
  TR_TRY(t_gemm(c, S.H2[b], D, t->wb(pre + ".mlp.fc1.weight"), t->f(pre + ".mlp.fc1.bias"), M, Hd, D, pdm::EPI_BF16,
                S.U[b], Hd, nullptr, 0, 0));
  TR_HIP(pdm::gelu_fwd_launch(S.U[b], S.Gl[b], (long long)M * Hd, c.s));
  TR_TRY(t_gemm(c, S.Gl[b], Hd, t->wb(pre + ".mlp.fc2.weight"), t->f(pre + ".mlp.fc2.bias"), M, D, Hd, pdm::EPI_F32,
                outb, D, out, D, 1, nullptr, 0, 0, X1));
  return PDM_OK;
}

// on entry DX / DXB = gradient w.r.t. the block output; on exit the gradient w.r.t. its input (for an out-block with a
// long skip: w.r.t. the previous block's output; the skip's share goes to S.DSK)
int block_bwd(const TC& c, const SW& S, int sid, int b, int rows, float*& DX, bf16*& DXB, float*& DX2, bf16*& DXB2) {
  const pdm_trainer* t = c.t;
  const TWork& w = *c.w;
  const std::string pre = t->block(b, sid);
  const int D = t->D, M = rows * S.L, Hd = t->Hid;
  // x = x1 + fc2(gelu(fc1(norm2(x1))))
  TR_TRY(t_gemm(c, DXB, D, t->wt(pre + ".mlp.fc2.weight"), nullptr, M, Hd, D, pdm::EPI_BF16, w.DG, Hd, nullptr, 0, 0));
  TR_TRY(t_wgrad(c, DXB, D, D, S.Gl[b], Hd, Hd, M, t->g(pre + ".mlp.fc2.weight"), Hd, t->g(pre + ".mlp.fc2.bias")));
  TR_HIP(pdm::gelu_bwd_launch(w.DG, S.U[b], (long long)M * Hd, c.s));
  TR_TRY(t_gemm(c, w.DG, Hd, t->wt(pre + ".mlp.fc1.weight"), nullptr, M, D, Hd, pdm::EPI_BF16, w.DH, D, nullptr, 0, 0));
  TR_TRY(t_wgrad(c, w.DG, Hd, Hd, S.H2[b], D, D, M, t->g(pre + ".mlp.fc1.weight"), D, t->g(pre + ".mlp.fc1.bias")));
  TR_TRY(t_ln_bwd(c, S.X1[b], w.DH, 1, pre + ".norm2", DX, DXB, M, 1));
  // x1 = x0 + proj(attn(qkv(norm1(x0))))
  TR_TRY(t_gemm(c, DXB, D, t->wt(pre + ".attn.proj.weight"), nullptr, M, D, D, pdm::EPI_BF16, w.DATT, D, nullptr, 0, 0));
  TR_TRY(t_wgrad(c, DXB, D, D, S.ATT[b], D, D, M, t->g(pre + ".attn.proj.weight"), D, t->g(pre + ".attn.proj.bias")));
  {
    pdm::AttnBwdArgs a{};
    a.qkv = S.QKV[b]; a.ldq = 3 * D;
    a.o = S.ATT[b]; a.ldo = D;
    a.dout = w.DATT; a.lddo = D;
    a.dqkv = w.DQKV; a.lddq = 3 * D;
    a.B = rows; a.L = S.L; a.H = t->H; a.Dh = t->Dh;
    a.scale = 1.0f / sqrtf((float)t->Dh);
    TR_CHECK(pdm::attn_bwd_check(a));
    TR_HIP(pdm::attn_bwd_launch(a, c.s));
  }
  TR_TRY(t_gemm(c, w.DQKV, 3 * D, t->wt(pre + ".attn.qkv.weight"), nullptr, M, D, 3 * D, pdm::EPI_BF16, w.DH, D, nullptr,
                0, 0));
  TR_TRY(t_wgrad(c, w.DQKV, 3 * D, 3 * D, S.H1[b], D, D, M, t->g(pre + ".attn.qkv.weight"), D,
                 t->has(pre + ".attn.qkv.bias") ? t->g(pre + ".attn.qkv.bias") : nullptr));
  TR_TRY(t_ln_bwd(c, S.X0[b], w.DH, 1, pre + ".norm1", DX, DXB, M, 1));
  if (t->skip_block(b)) {   // x0 = skip_linear(cat([x_prev, skip]))
    const int j = t->skip_src(b);
    float* gw = t->g(pre + ".skip_linear.weight");
    TR_TRY(t_wgrad(c, DXB, D, D, S.XS[b], D, D, M, gw, 2 * D, t->g(pre + ".skip_linear.bias")));
    TR_TRY(t_wgrad(c, DXB, D, D, S.SK[j], D, D, M, gw + D, 2 * D));
    const bf16* wt = t->wt(pre + ".skip_linear.weight");   // [2D][D]
    TR_TRY(t_gemm(c, DXB, D, wt + (size_t)D * D, nullptr, M, D, D, pdm::EPI_F32, nullptr, 0, S.DSK[j], D, 0));
    TR_TRY(t_gemm(c, DXB, D, wt, nullptr, M, D, D, pdm::EPI_F32, DXB2, D, DX2, D, 0));
    std::swap(DX, DX2);
    std::swap(DXB, DXB2);
  }
  return PDM_OK;
}

// decoder_pred (+ unpatchify) on bf16 token rows x (token (b, i) = row b * gs + i) -> pre [B, C, S, S]
int t_head(const TC& c, const bf16* x, int gs, const std::string& head, int C, int P, int P_pad, float* pre, int rows) {
  const pdm_trainer* t = c.t;
  pdm::HeadArgs a{};
  a.x = x; a.ldx = t->D; a.in_group_stride = gs; a.in_row_offset = 0;
  a.W = t->wb(head + ".weight"); a.bias = t->f(head + ".bias");
  a.out = pre;
  a.B = rows; a.D = t->D; a.C = C; a.p = t->p; a.Himg = t->img; a.Wimg = t->img; a.P = P; a.P_pad = P_pad;
  TR_CHECK(pdm::head_check(a));
  TR_HIP(pdm::head_launch(a, c.s));
  return PDM_OK;
}

// final 3x3 conv (when cfg.conv) and optional tanh: pre -> out
int t_final(const TC& c, const float* pre, const char* conv, int C, int act_tanh, float* out, int rows) {
  const pdm_trainer* t = c.t;
  pdm::EpilogueArgs a{};
  a.pre = pre;
  if (t->cfg.conv) { a.w = t->f(std::string(conv) + ".weight"); a.bias = t->f(std::string(conv) + ".bias"); }
  a.B = rows; a.C = C; a.Himg = t->img; a.Wimg = t->img;
  a.act_tanh = act_tanh;
  a.ae = 1.0f;
  a.m_out = out;
  TR_CHECK(pdm::epilogue_check(a));
  TR_HIP(pdm::epilogue_launch(a, c.s));
  return PDM_OK;
}

// backward of t_head / t_final: dpred (gradient w.r.t. the final output, tanh already applied) -> the conv's weight
// gradients, decoder_pred's (A = dtok against the head input rows x, gathered by gs) and dx fp32 [rows * n_patch][D]
int t_head_bwd(const TC& c, const float* dpred, const float* pre, float* dpre_buf, const char* conv,
               const std::string& head, int C, int P, int P_pad, bf16* dtok, float* dx, const bf16* x, int gs,
               int rows) {
  const pdm_trainer* t = c.t;
  const float* dpre = dpred;
  if (t->cfg.conv) {
    TR_HIP(pdm::conv3x3_bwd_launch(dpred, pre, t->f(std::string(conv) + ".weight"), dpre_buf,
                                   t->g(std::string(conv) + ".weight"), t->g(std::string(conv) + ".bias"), rows, C,
                                   t->img, t->img, c.s));
    dpre = dpre_buf;
  }
  pdm::HeadBwdArgs a{};
  a.dpre = dpre; a.W = t->f(head + ".weight");
  a.dtok = dtok; a.dx = dx;
  a.B = rows; a.D = t->D; a.C = C; a.p = t->p; a.Himg = t->img; a.Wimg = t->img; a.P = P; a.P_pad = P_pad;
  TR_HIP(pdm::head_bwd_launch(a, c.s));
  const int Mp = rows * t->n_patch;
  return t_wgrad(c, dtok, P_pad, P, x, t->D, t->D, Mp, t->g(head + ".weight"), t->D, t->g(head + ".bias"), 0, 0, 0,
                 gs == t->n_patch ? 0 : t->n_patch, gs, 0);
}

int train_step(const TC& c, const float* xt, const float* tv, const int64_t* y, const float* target, float* loss,
               int rows, float gscale) {
  const pdm_trainer* t = c.t;
  const TWork& w = *c.w;
  const SW& I = w.I;
  const int D = t->D, L = t->L, M = rows * L, Mp = rows * t->n_patch;
  const int C = t->C, S = t->img;
  // ---- forward (libs/uvit.py:201-230)
  {
    pdm::AssembleArgs a{};
    a.img = xt; a.C = C; a.Himg = S; a.Wimg = S; a.p = t->p;
    a.patch_w = t->f("patch_embed.proj.weight"); a.patch_b = t->f("patch_embed.proj.bias");
    a.t = tv;
    a.y = y;
    a.label_emb = t->cfg.num_classes > 0 ? t->f("label_emb.weight") : nullptr;
    a.pos = t->f("pos_embed");
    a.out = I.X0[0]; a.ld_out = D;
    a.B = rows; a.D = D; a.L_total = L;
    a.row0_patch = t->extras;
    a.time_row = t->extras - 1;
    a.label_row = t->cfg.num_classes > 0 ? 0 : -1;
    a.ctx_row = -1;
    TR_CHECK(pdm::assemble_check(a));
    TR_HIP(pdm::assemble_launch(a, c.s));
  }
  for (int b = 0; b < t->nb; ++b) {
    // the output is the next block's input, except where the next block starts from skip_linear (its fp32 input is
    // then that GEMM's output; only the bf16 copy XS is its operand)
    const bool last = b == t->nb - 1;
    float* out = last ? w.XF : (t->skip_block(b + 1) ? w.XTMP : I.X0[b + 1]);
    bf16* outb = b < t->nhalf ? I.SK[b] : (!last && t->skip_block(b + 1) ? I.XS[b + 1] : nullptr);
    TR_TRY(block_fwd(c, I, 0, b, rows, out, outb));
  }
  TR_TRY(t_ln(c, w.XF, Mp, t->f("norm.weight"), t->f("norm.bias"), w.HN, t->n_patch, L, t->extras));
  TR_TRY(t_head(c, w.HN, t->n_patch, "decoder_pred", C, t->P, t->P_pad, w.PRE, rows));
  const float* pred = w.PRE;
  if (t->cfg.conv) {
    TR_TRY(t_final(c, w.PRE, "final_layer", C, 0, w.EPS, rows));
    pred = w.EPS;
  }
  const int per = C * S * S;
  TR_HIP(pdm::lsimple_launch(pred, target, loss, w.DPRED, rows, per, gscale, c.s));
  // ---- backward
  TR_TRY(t_head_bwd(c, w.DPRED, w.PRE, w.DPRE, "final_layer", "decoder_pred", C, t->P, t->P_pad, w.DTOK, w.DHN, w.HN,
                    t->n_patch, rows));
  float* DX = w.DX;
  float* DX2 = w.DX2;
  bf16* DXB = w.DXB;
  bf16* DXB2 = w.DXB2;
  TR_HIP(hipMemsetAsync(DX, 0, (size_t)M * D * 4, c.s));
  TR_HIP(hipMemsetAsync(DXB, 0, (size_t)M * D * 2, c.s));
  TR_TRY(t_ln_bwd(c, w.XF, w.DHN, 0, "norm", DX, DXB, Mp, 0, t->n_patch, L, t->extras));
  for (int b = t->nb - 1; b >= 0; --b) {
    TR_TRY(block_bwd(c, I, 0, b, rows, DX, DXB, DX2, DXB2));
    if (b - 1 >= 0 && b - 1 < t->nhalf && t->cfg.skip)   // in-block b-1's output also fed out-block's long skip
      TR_HIP(pdm::add_cast_launch(DX, I.DSK[b - 1], DXB, (long long)M * D, c.s));
  }
  // token assembly: pos_embed, label_emb, patch_embed (time token: no parameters, mlp_time_embed=False)
  TR_TRY(t_colsum(c, DX, 0, L * D, rows, L * D, t->g("pos_embed")));
  if (t->cfg.num_classes > 0) {
    TR_HIP(hipMemsetAsync(t->g("label_emb.weight"), 0, (size_t)t->cfg.num_classes * D * 4, c.s));
    TR_HIP(pdm::label_scatter_launch(DX, L, 0, D, y, t->g("label_emb.weight"), rows, c.s));
  }
  TR_HIP(pdm::patchify_launch(xt, w.PV, rows, C, S, S, t->p, t->Kp_pad, c.s));
  TR_TRY(t_wgrad(c, DXB, D, D, w.PV, t->Kp_pad, t->Kp, Mp, t->g("patch_embed.proj.weight"), t->Kp,
                 t->g("patch_embed.proj.bias"), t->n_patch, L, t->extras));
  return PDM_OK;
}

// bf16 row copy as 4-byte words: rows of D bf16 from src (gather rpg / sgs) to dst (scatter rpg / dgs)
int t_copy_b(const TC& c, bf16* dst, const bf16* src, int rows, int rpg, int dgs, int sgs) {
  const int D = c.t->D;
  TR_HIP(pdm::rowcopy_launch(reinterpret_cast<float*>(dst), D / 2, reinterpret_cast<const float*>(src), D / 2, rows,
                             D / 2, rpg, dgs, sgs, c.s, nullptr, 0, nullptr, 0, 0));
  return PDM_OK;
}

// The panoptic t2i step (train_t2i_discrete.py:148-224 with mask_token = mask_n, use_ground_truth False;
// libs/uvit_t2i.py:380-525 separate=True): loss[b] = mos(eps - eps_pred), loss_m[b] = mos(mask_pred - bits), and
// d(gscale * sum_b (loss[b] + loss_m[b])) / d(params) -- train_t2i_discrete.py:468-473 backpropagates
// loss_eps.mean() + loss_mask.mean().
int train_step_t2i(const TC& c, const float* xt, const float* tv, const float* ctx, const float* mtok, const float* target,
                   const float* mtarget, float* loss, float* loss_m, int rows, float gscale) {
  const pdm_trainer* t = c.t;
  const TWork& w = *c.w;
  const SW& I = w.I;
  const SW& Q = w.Q;
  const int D = t->D, Lx = t->L, Lm = t->Lm, np = t->n_patch, nctx = t->nctx, nh = t->nhalf, nb = t->nb;
  const int Mx = rows * Lx, Mm = rows * Lm, Mp = rows * np;
  const int C = t->C, S = t->img, K = t->K;
  auto zc = [&](int b) { return "zero_convs." + std::to_string(2 * b + 1) + ".conv"; };
  // ---- forward
  // context_embed (387): bf16 copy of the CLIP tokens (also the weight-gradient operand) -> fp32 context tokens
  TR_HIP(pdm::cast_bf16_launch(ctx, w.CTXB, (long long)rows * nctx * t->clip, c.s));
  TR_TRY(t_gemm(c, w.CTXB, t->clip, t->wb("context_embed.weight"), t->f("context_embed.bias"), rows * nctx, D, t->clip,
                pdm::EPI_F32, nullptr, 0, w.CTXF, D, 0));
  {  // x = cat(time, context, patches) + pos_embed (401-405, 408-409)
    pdm::AssembleArgs a{};
    a.img = xt; a.C = C; a.Himg = S; a.Wimg = S; a.p = t->p;
    a.patch_w = t->f("patch_embed.proj.weight"); a.patch_b = t->f("patch_embed.proj.bias");
    a.t = tv; a.ctx_tokens = w.CTXF; a.n_ctx = nctx;
    a.pos = t->f("pos_embed");
    a.out = I.X0[0]; a.ld_out = D; a.B = rows; a.D = D; a.L_total = Lx;
    a.row0_patch = t->extras; a.time_row = 0; a.label_row = -1; a.ctx_row = 1;
    TR_CHECK(pdm::assemble_check(a));
    TR_HIP(pdm::assemble_launch(a, c.s));
  }
  {  // m = mask_embed(mask_token) + pos_embed_mask (390, 406): the mask rows of the first mask-block input
    pdm::AssembleArgs a{};
    a.img = mtok; a.C = K; a.Himg = S; a.Wimg = S; a.p = t->p;
    a.patch_w = t->f("mask_embed.proj.weight"); a.patch_b = t->f("mask_embed.proj.bias");
    a.pos = t->f("pos_embed_mask");
    a.out = Q.X0[0] + (size_t)Lx * D; a.ld_out = D; a.B = rows; a.D = D; a.L_total = Lm;
    a.row0_patch = 0; a.time_row = -1; a.label_row = -1; a.ctx_row = -1;
    TR_CHECK(pdm::assemble_check(a));
    TR_HIP(pdm::assemble_launch(a, c.s));
  }
  for (int b = 0; b < nb; ++b) {
    const bool sk = t->skip_block(b), last = b == nb - 1;
    // mx = cat(x, m) (426, 443, 459): x is the image block's input before its skip_linear; the mask rows are in
    // place (the previous mask block wrote its whole output here, or the assembly)
    const float* xpre = sk ? w.XTMP : I.X0[b];
    float* mpre = sk ? w.MXTMP : Q.X0[b];
    TR_HIP(pdm::rowcopy_launch(mpre, D, xpre, D, Mx, D, Lx, Lm, Lx, c.s, nullptr, 0, nullptr, 0, 0));
    if (sk) {   // bf16 mx: the mask skip_linear operand
      TR_TRY(t_copy_b(c, Q.XS[b], I.XS[b], Mx, Lx, Lm, Lx));
      TR_TRY(t_copy_b(c, Q.XS[b] + (size_t)Lx * D, w.MOB[b - 1] + (size_t)Lx * D, Mp, np, Lm, Lm));
    }
    float* iout = last ? w.XF : (t->skip_block(b + 1) ? w.XTMP : I.X0[b + 1]);
    float* mout = last ? w.MF : (t->skip_block(b + 1) ? w.MXTMP : Q.X0[b + 1]);
    TR_TRY(block_fwd(c, I, 0, b, rows, iout, nullptr));
    TR_TRY(block_fwd(c, Q, 1, b, rows, mout, w.MOB[b]));
    // x += zeroconv(mx[:, :Lx]) (435-436, 452-453, 470-472) in place; its bf16 copy is the long skip (in-blocks) or
    // the next skip_linear operand
    pdm::GemmArgs a{};
    a.A1 = w.MOB[b]; a.lda1 = D; a.K1 = D;
    a.a_rows_per_group = Lx; a.a_group_stride = Lm;
    a.W = t->wb(zc(b) + ".weight"); a.bias = t->f(zc(b) + ".bias");
    a.M = Mx; a.N = D; a.K = D;
    a.out_f32 = iout; a.ldr = D; a.accumulate = 1;
    a.out_bf16 = b < nh ? I.SK[b] : (!last && t->skip_block(b + 1) ? I.XS[b + 1] : nullptr); a.ldo = D;
    TR_CHECK(pdm::gemm_check(a, pdm::EPI_F32));
    TR_HIP(pdm::gemm_launch(a, pdm::EPI_F32, c.s));
  }
  // heads (477-519): noise from norm(x)'s patch tokens; mask = tanh(final_layer_mask(decoder_pred_mask(m))) on the
  // un-normalised last mask rows
  TR_TRY(t_ln(c, w.XF, Mp, t->f("norm.weight"), t->f("norm.bias"), w.HN, np, Lx, t->extras));
  TR_TRY(t_head(c, w.HN, np, "decoder_pred", C, t->P, t->P_pad, w.PRE, rows));
  const float* pred = w.PRE;
  if (t->cfg.conv) {
    TR_TRY(t_final(c, w.PRE, "final_layer", C, 0, w.EPS, rows));
    pred = w.EPS;
  }
  TR_TRY(t_copy_b(c, w.MHN, w.MOB[nb - 1] + (size_t)Lx * D, Mp, np, np, Lm));
  TR_TRY(t_head(c, w.MHN, np, "decoder_pred_mask", K, t->PK, t->PK_pad, w.MPRE, rows));
  TR_TRY(t_final(c, w.MPRE, "final_layer_mask", K, 1, w.MPRED, rows));
  TR_HIP(pdm::lsimple_launch(pred, target, loss, w.DPRED, rows, C * S * S, gscale, c.s));
  TR_HIP(pdm::lsimple_launch(w.MPRED, mtarget, loss_m, w.MDPRED, rows, K * S * S, gscale, c.s, 1));
  // ---- backward
  TR_TRY(t_head_bwd(c, w.DPRED, w.PRE, w.DPRE, "final_layer", "decoder_pred", C, t->P, t->P_pad, w.DTOK, w.DHN, w.HN,
                    np, rows));
  TR_TRY(t_head_bwd(c, w.MDPRED, w.MPRE, w.MDPRE, "final_layer_mask", "decoder_pred_mask", K, t->PK, t->PK_pad,
                    w.MDTOK, w.DMHN, w.MHN, np, rows));
  float* DX = w.DX;
  float* DX2 = w.DX2;
  bf16* DXB = w.DXB;
  bf16* DXB2 = w.DXB2;
  float* DM = w.DMX;
  float* DM2 = w.DMX2;
  bf16* DMB = w.DMXB;
  bf16* DMB2 = w.DMXB2;
  TR_HIP(hipMemsetAsync(DX, 0, (size_t)Mx * D * 4, c.s));
  TR_HIP(hipMemsetAsync(DXB, 0, (size_t)Mx * D * 2, c.s));
  TR_TRY(t_ln_bwd(c, w.XF, w.DHN, 0, "norm", DX, DXB, Mp, 0, np, Lx, t->extras));
  // the mask head's gradient lands on the mask rows of the last mask-block output (its image rows: the injection's)
  TR_HIP(pdm::rows_add_cast_launch(DM, DMB, np, Lm, Lx, w.DMHN, 0, 0, 0, Mp, D, 0, c.s));
  for (int b = nb - 1; b >= 0; --b) {
    const bool skipped = b < nh && t->cfg.skip;   // in-block b's outputs also fed out-block 2 nh - b's long skips
    // DX: gradient w.r.t. x after this layer's injection (incl. its long-skip share)
    if (skipped) TR_HIP(pdm::add_cast_launch(DX, I.DSK[b], DXB, (long long)Mx * D, c.s));
    // injection: d mx_out[:, :Lx] = dx zc.W (the image rows of the mask-output gradient), zc's weight / bias
    TR_TRY(t_gemm(c, DXB, D, t->wt(zc(b) + ".weight"), nullptr, Mx, D, D, pdm::EPI_F32, nullptr, 0, w.TMP, D, 0));
    TR_TRY(t_wgrad(c, DXB, D, D, w.MOB[b], D, D, Mx, t->g(zc(b) + ".weight"), D, t->g(zc(b) + ".bias"), 0, 0, 0, Lx,
                   Lm, 0));
    TR_HIP(pdm::rows_add_cast_launch(DM, DMB, Lx, Lm, 0, w.TMP, 0, 0, 0, Mx, D, 0, c.s));
    if (skipped) TR_HIP(pdm::add_cast_launch(DM, Q.DSK[b], DMB, (long long)Mm * D, c.s));
    TR_TRY(block_bwd(c, Q, 1, b, rows, DM, DMB, DM2, DMB2));
    TR_TRY(block_bwd(c, I, 0, b, rows, DX, DXB, DX2, DXB2));
    // mx = cat(x, m): its image rows' gradient joins x's; its mask rows' stays as the previous mask output's
    TR_HIP(pdm::rows_add_cast_launch(DX, DXB, 0, 0, 0, DM, Lx, Lm, 0, Mx, D, 1, c.s));
  }
  // embeddings: pos_embed, context_embed (rows 1 .. nctx), patch_embed; pos_embed_mask, mask_embed
  TR_TRY(t_colsum(c, DX, 0, Lx * D, rows, Lx * D, t->g("pos_embed")));
  TR_TRY(t_wgrad(c, DXB, D, D, w.CTXB, t->clip, t->clip, rows * nctx, t->g("context_embed.weight"), t->clip,
                 t->g("context_embed.bias"), nctx, Lx, 1));
  TR_HIP(pdm::patchify_launch(xt, w.PV, rows, C, S, S, t->p, t->Kp_pad, c.s));
  TR_TRY(t_wgrad(c, DXB, D, D, w.PV, t->Kp_pad, t->Kp, Mp, t->g("patch_embed.proj.weight"), t->Kp,
                 t->g("patch_embed.proj.bias"), np, Lx, t->extras));
  TR_TRY(t_colsum(c, DM + (size_t)Lx * D, 0, Lm * D, rows, np * D, t->g("pos_embed_mask")));
  TR_HIP(pdm::patchify_launch(mtok, w.PVM, rows, K, S, S, t->p, t->Kpm_pad, c.s));
  TR_TRY(t_wgrad(c, DMB, D, D, w.PVM, t->Kpm_pad, t->Kpm, Mp, t->g("mask_embed.proj.weight"), t->Kpm,
                 t->g("mask_embed.proj.bias"), np, Lm, Lx));
  return PDM_OK;
}

int refresh(pdm_trainer* t, hipStream_t s) {
  TR_HIP(pdm::cast_bf16_launch(t->Pm, t->WB, t->total, s));
  for (const TParam& q : t->params)
    if (q.kind == KIND_LINEAR) TR_HIP(pdm::transpose_bf16_launch(t->Pm + q.off, t->WT + q.wt_off, q.N, q.K, s));
  return PDM_OK;
}

}  // namespace

extern "C" {

int pdm_train_create(const pdm_uvit_cfg* cfg, pdm_trainer** out) {
  if (!cfg || !out) return pdm::set_error(PDM_ERR_ARG, "pdm_train_create: null argument");
  const pdm_uvit_cfg& c = *cfg;
  if (c.fp8) return pdm::set_error(PDM_ERR_ARG, "pdm_train: bf16 U-ViT only");
  if (c.t2i && !(c.separate && c.enable_panoptic))
    return pdm::set_error(PDM_ERR_ARG, "pdm_train: the t2i network trains with separate panoptic streams only");
  if (c.mlp_time_embed) return pdm::set_error(PDM_ERR_ARG, "pdm_train: mlp_time_embed is not supported");
  if (c.embed_dim <= 0 || c.num_heads <= 0 || c.embed_dim % c.num_heads ||
      (c.embed_dim / c.num_heads != 64 && c.embed_dim / c.num_heads != 72))
    return pdm::set_error(PDM_ERR_ARG, "pdm_train: head dim must be 64 or 72 (the attention backward kernel)");
  if (c.embed_dim % 64 || c.mlp_hidden % 64 || c.depth < 2)
    return pdm::set_error(PDM_ERR_ARG, "pdm_train: embed_dim / mlp hidden multiples of 64, depth >= 2");
  if (c.img_size % c.patch_size) return pdm::set_error(PDM_ERR_ARG, "pdm_train: img_size % patch_size != 0");
  pdm_trainer* t = new pdm_trainer();
  t->cfg = c;
  t->D = c.embed_dim; t->H = c.num_heads; t->Dh = c.embed_dim / c.num_heads; t->Hid = c.mlp_hidden;
  t->C = c.in_chans; t->p = c.patch_size; t->img = c.img_size;
  t->n_patch = (c.img_size / c.patch_size) * (c.img_size / c.patch_size);
  t->t2i = c.t2i != 0;
  if (t->t2i) {   // tokens [time, context x nctx, patches] (libs/uvit_t2i.py:401-405); mask stream cat(x, m)
    t->nctx = c.num_clip_token; t->clip = c.clip_dim; t->K = c.num_panoptic_class;
    t->extras = 1 + t->nctx;
  } else {
    t->extras = c.num_classes > 0 ? 2 : 1;
  }
  t->L = t->n_patch + t->extras;
  t->Lm = t->t2i ? t->L + t->n_patch : 0;
  t->P = c.patch_size * c.patch_size * c.in_chans;
  t->P_pad = (t->P + 15) & ~15;
  t->Kp = t->P;
  t->Kp_pad = (t->Kp + 7) & ~7;
  t->PK = c.patch_size * c.patch_size * t->K;
  t->PK_pad = (t->PK + 15) & ~15;
  t->Kpm = t->PK;
  t->Kpm_pad = (t->Kpm + 7) & ~7;
  t->depth = c.depth; t->nhalf = c.depth / 2; t->nb = 2 * t->nhalf + 1;   // in-blocks, mid_block, out-blocks
  const int Lmax = t->t2i ? t->Lm : t->L;
  if (Lmax > (t->Dh == 64 ? 608 : 415) || t->P > 64 || t->P % 4 || (t->t2i && (t->PK > 64 || t->PK % 4 || t->K <= 0 || t->nctx <= 0 ||
                                                          t->clip <= 0 || t->clip % 64))) {
    delete t;
    return pdm::set_error(PDM_ERR_ARG, "pdm_train: tokens per stream <= 608 (head dim 72: 415), p*p*C (and p*p*K) "
                                       "<= 64 and a multiple of 4, clip_dim a multiple of 64");
  }
  const int D = t->D;
  auto add_block = [&](const std::string& pre, bool skip) {
    if (skip) {
      t->add(pre + ".skip_linear.weight", 2LL * D * D, KIND_LINEAR, D, 2 * D);
      t->add(pre + ".skip_linear.bias", D);
    }
    t->add(pre + ".norm1.weight", D);
    t->add(pre + ".norm1.bias", D);
    t->add(pre + ".attn.qkv.weight", 3LL * D * D, KIND_LINEAR, 3 * D, D);
    if (c.qkv_bias) t->add(pre + ".attn.qkv.bias", 3LL * D);
    t->add(pre + ".attn.proj.weight", (long long)D * D, KIND_LINEAR, D, D);
    t->add(pre + ".attn.proj.bias", D);
    t->add(pre + ".norm2.weight", D);
    t->add(pre + ".norm2.bias", D);
    t->add(pre + ".mlp.fc1.weight", (long long)t->Hid * D, KIND_LINEAR, t->Hid, D);
    t->add(pre + ".mlp.fc1.bias", t->Hid);
    t->add(pre + ".mlp.fc2.weight", (long long)D * t->Hid, KIND_LINEAR, D, t->Hid);
    t->add(pre + ".mlp.fc2.bias", D);
  };
  if (c.conv) {
    t->add("final_layer.weight", (long long)t->C * t->C * 9);
    t->add("final_layer.bias", t->C);
  }
  t->add("decoder_pred.weight", (long long)t->P * D, KIND_HEAD, t->P, D, (long long)t->P_pad * D);
  t->add("decoder_pred.bias", t->P);
  if (t->t2i) {
    if (c.conv) {
      t->add("final_layer_mask.weight", (long long)t->K * t->K * 9);
      t->add("final_layer_mask.bias", t->K);
    }
    t->add("decoder_pred_mask.weight", (long long)t->PK * D, KIND_HEAD, t->PK, D, (long long)t->PK_pad * D);
    t->add("decoder_pred_mask.bias", t->PK);
  }
  t->add("norm.weight", D);
  t->add("norm.bias", D);
  for (int b = t->nb - 1; b >= 0; --b) {
    add_block(t->block(b), t->skip_block(b));
    if (t->t2i) {
      add_block(t->block(b, 1), t->skip_block(b));
      const std::string zc = "zero_convs." + std::to_string(2 * b + 1) + ".conv";
      t->add(zc + ".weight", (long long)D * D, KIND_LINEAR, D, D);
      t->add(zc + ".bias", D);
    }
  }
  if (t->t2i) {
    t->add("context_embed.weight", (long long)D * t->clip);
    t->add("context_embed.bias", D);
  }
  if (c.num_classes > 0 && !t->t2i) t->add("label_emb.weight", (long long)c.num_classes * D);
  t->add("pos_embed", (long long)t->L * D);
  t->add("patch_embed.proj.weight", (long long)D * t->Kp);
  t->add("patch_embed.proj.bias", D);
  if (t->t2i) {
    t->add("pos_embed_mask", (long long)t->n_patch * D);
    t->add("mask_embed.proj.weight", (long long)D * t->Kpm);
    t->add("mask_embed.proj.bias", D);
  }
  t->active = t->total;
  if (t->t2i) {   // in the state dict, never used by the forward (uvit_t2i.py:321-324 / 331: commented-out uses)
    for (int i = 0; i < 2 * c.depth + 2; i += 2) {
      const std::string zc = "zero_convs." + std::to_string(i) + ".conv";
      t->add(zc + ".weight", (long long)D * D);
      t->add(zc + ".bias", D);
    }
    t->add("mask_embed_0.proj.weight", (long long)D * t->Kpm);
    t->add("mask_embed_0.proj.bias", D);
  }
  *out = t;
  return PDM_OK;
}

int pdm_train_destroy(pdm_trainer* t) {
  delete t;
  return PDM_OK;
}

int pdm_train_param_count(const pdm_trainer* t) { return t ? (int)t->params.size() : 0; }

int pdm_train_param_info(const pdm_trainer* t, int i, char* name, int len, long long* offset, long long* numel) {
  if (!t || i < 0 || i >= (int)t->params.size()) return pdm::set_error(PDM_ERR_ARG, "pdm_train_param_info: bad index");
  const TParam& q = t->params[i];
  if (name && len > 0) {
    std::strncpy(name, q.name.c_str(), len - 1);
    name[len - 1] = 0;
  }
  if (offset) *offset = q.off;
  if (numel) *numel = q.numel;
  return PDM_OK;
}

int pdm_train_sizes(const pdm_trainer* t, long long* n_params, long long* n_wt) {
  if (!t) return pdm::set_error(PDM_ERR_ARG, "pdm_train_sizes: null handle");
  if (n_params) *n_params = t->total;
  if (n_wt) *n_wt = t->wt_total;
  return PDM_OK;
}

int pdm_train_set_buffers(pdm_trainer* t, float* params, float* grads, void* wb, void* wt) {
  if (!t || !params || !grads || !wb || !wt) return pdm::set_error(PDM_ERR_ARG, "pdm_train_set_buffers: null argument");
  if (((uintptr_t)params | (uintptr_t)grads | (uintptr_t)wb | (uintptr_t)wt) & 255)
    return pdm::set_error(PDM_ERR_ARG, "pdm_train_set_buffers: buffers must be 256-byte aligned");
  t->Pm = params;
  t->G = grads;
  t->WB = static_cast<bf16*>(wb);
  t->WT = static_cast<bf16*>(wt);
  return PDM_OK;
}

int pdm_train_refresh(pdm_trainer* t, void* stream) {
  if (!t || !t->Pm) return pdm::set_error(PDM_ERR_STATE, "pdm_train_refresh: buffers not set");
  return refresh(t, (hipStream_t)stream);
}

int pdm_train_workspace_size(const pdm_trainer* t, int rows, size_t* bytes) {
  if (!t || rows <= 0 || !bytes) return pdm::set_error(PDM_ERR_ARG, "pdm_train_workspace_size: bad argument");
  *bytes = tlayout(t, rows, nullptr).bytes;
  return PDM_OK;
}

int pdm_train_step(pdm_trainer* t, const float* xt, const float* tvals, const int64_t* y, const float* target,
                   float* loss, int rows, float gscale, void* workspace, size_t workspace_bytes, void* stream) {
  if (!t || !t->Pm) return pdm::set_error(PDM_ERR_STATE, "pdm_train_step: buffers not set");
  if (!xt || !tvals || !target || !loss || rows <= 0 || !workspace)
    return pdm::set_error(PDM_ERR_ARG, "pdm_train_step: null argument");
  if (t->t2i) return pdm::set_error(PDM_ERR_ARG, "pdm_train_step: a t2i trainer steps with pdm_train_step_t2i");
  if ((t->cfg.num_classes > 0) != (y != nullptr))
    return pdm::set_error(PDM_ERR_ARG, "pdm_train_step: labels required iff num_classes > 0");
  TWork w = tlayout(t, rows, static_cast<char*>(workspace));
  if (w.bytes > workspace_bytes) return pdm::set_error(PDM_ERR_ARG, "pdm_train_step: workspace too small");
  TC c{t, (hipStream_t)stream, &w};
  return train_step(c, xt, tvals, y, target, loss, rows, gscale);
}

int pdm_train_step_t2i(pdm_trainer* t, const float* xt, const float* tvals, const float* context,
                       const float* mask_token, const float* target, const float* mask_target, float* loss,
                       float* loss_mask, int rows, float gscale, void* workspace, size_t workspace_bytes, void* stream) {
  if (!t || !t->Pm) return pdm::set_error(PDM_ERR_STATE, "pdm_train_step_t2i: buffers not set");
  if (!t->t2i) return pdm::set_error(PDM_ERR_ARG, "pdm_train_step_t2i: not a t2i trainer");
  if (!xt || !tvals || !context || !mask_token || !target || !mask_target || !loss || !loss_mask || rows <= 0 ||
      !workspace)
    return pdm::set_error(PDM_ERR_ARG, "pdm_train_step_t2i: null argument");
  TWork w = tlayout(t, rows, static_cast<char*>(workspace));
  if (w.bytes > workspace_bytes) return pdm::set_error(PDM_ERR_ARG, "pdm_train_step_t2i: workspace too small");
  TC c{t, (hipStream_t)stream, &w};
  return train_step_t2i(c, xt, tvals, context, mask_token, target, mask_target, loss, loss_mask, rows, gscale);
}

int pdm_train_adamw(pdm_trainer* t, float* m, float* v, float* ema, const float* grads2, float lr, float beta1,
                    float beta2, float eps, float weight_decay, int step, float ema_rate, void* stream) {
  if (!t || !t->Pm) return pdm::set_error(PDM_ERR_STATE, "pdm_train_adamw: buffers not set");
  if (!m || !v || step < 1) return pdm::set_error(PDM_ERR_ARG, "pdm_train_adamw: moments missing or step < 1");
  pdm::AdamWArgs a{};
  a.p = t->Pm; a.g = t->G; a.g2 = grads2; a.m = m; a.v = v; a.ema = ema; a.pb = nullptr;
  a.lr = lr; a.wd = weight_decay; a.b1 = beta1; a.b2 = beta2; a.eps = eps;
  const double bc1 = 1.0 - std::pow((double)beta1, step), bc2 = 1.0 - std::pow((double)beta2, step);
  a.step_size = (float)(lr / bc1);
  a.inv_sqrt_bc2 = (float)(1.0 / std::sqrt(bc2));
  a.ema_rate = ema_rate;
  hipStream_t s = (hipStream_t)stream;
  TR_HIP(pdm::adamw_launch(a, t->active, s));
  return refresh(t, s);
}

int pdm_set_wgrad_tile(int tile) {
  if (tile != 0 && tile != 128 && tile != 256) return pdm::set_error(PDM_ERR_ARG, "pdm_set_wgrad_tile: 0, 128 or 256");
  pdm::g_wgrad_tile = tile;
  return PDM_OK;
}

// ---- individual training kernels (parity tests) ----
int pdm_wgrad(const void* A, int lda, const void* B, int ldb, float* C, int ldc, int M, int N, int K, int accumulate,
              float* scratch, size_t scratch_bytes, void* stream) {
  pdm::WgradArgs a{};
  a.A = static_cast<const bf16*>(A); a.lda = lda;
  a.B = static_cast<const bf16*>(B); a.ldb = ldb;
  a.C = C; a.ldc = ldc; a.M = M; a.N = N; a.K = K; a.accumulate = accumulate;
  TR_CHECK(pdm::wgrad_check(a));
  TR_HIP(pdm::wgrad_launch(a, scratch, scratch_bytes, (hipStream_t)stream));
  return PDM_OK;
}

int pdm_attention_backward(const void* qkv, const void* o, const void* dout, void* dqkv, int B, int L, int H, int Dh,
                           void* stream) {
  pdm::AttnBwdArgs a{};
  a.qkv = static_cast<const bf16*>(qkv); a.ldq = 3 * H * Dh;
  a.o = static_cast<const bf16*>(o); a.ldo = H * Dh;
  a.dout = static_cast<const bf16*>(dout); a.lddo = H * Dh;
  a.dqkv = static_cast<bf16*>(dqkv); a.lddq = 3 * H * Dh;
  a.B = B; a.L = L; a.H = H; a.Dh = Dh;
  a.scale = 1.0f / sqrtf((float)Dh);
  TR_CHECK(pdm::attn_bwd_check(a));
  TR_HIP(pdm::attn_bwd_launch(a, (hipStream_t)stream));
  return PDM_OK;
}

int pdm_layernorm_backward(const float* x, const void* dh, int dh_bf16, const float* gamma, float* dx, void* dxb,
                           float* dgamma, float* dbeta, int rows, int D, int accumulate, float* scratch,
                           size_t scratch_bytes, void* stream) {
  pdm::LnBwdArgs a{};
  a.x = x; a.ldx = D; a.lddh = D; a.gamma = gamma;
  a.dx = dx; a.lddx = D; a.dxb = static_cast<bf16*>(dxb);
  a.rows = rows; a.D = D; a.eps = 1e-5f; a.accumulate = accumulate;
  a.part = scratch; a.part_bytes = scratch_bytes;
  TR_HIP(pdm::ln_bwd_launch(a, dh, dh_bf16, dgamma, dbeta, (hipStream_t)stream));
  return PDM_OK;
}

}  // extern "C"

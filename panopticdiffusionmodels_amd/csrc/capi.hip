// C ABI of libpdm (include/pdm.h) and the U-ViT forward drivers.
//
// The drivers restate the layer loops of libs/uvit.py:201-230 and libs/uvit_t2i.py:378-525 as a fixed
// sequence of stream-ordered kernel launches over a caller-owned workspace: no allocation, no host sync,
// so a whole forward (or a whole sampler step) can be captured into a HIP graph.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/pdm.h"
#include "pdm_kernels.h"

using pdm::bf16;

namespace {

thread_local std::string g_err;
bool g_sk_standalone = false;       // pdm_set_gemm_sk bit 2: standalone pdm_gemm calls take stream-K (library state)
constexpr int SK_LAUNCHES = 512;    // stream-K flag blocks per forward workspace (GEMM launches of one forward)

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

}  // namespace

namespace pdm {
int set_error(int code, const std::string& msg) { return fail(code, msg); }
}  // namespace pdm

namespace {

#define PDM_HIP(call)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (call);                                                             \
    if (e_ != hipSuccess) return fail(PDM_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define PDM_TRY(x)           \
  do {                       \
    int r_ = (x);            \
    if (r_) return r_;       \
  } while (0)

#define PDM_CHECK(msg_expr)                          \
  do {                                               \
    const char* m_ = (msg_expr);                     \
    if (m_) return fail(PDM_ERR_ARG, m_);            \
  } while (0)

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct ParamSpec {
  int dtype;
  long long numel;
  const void* ptr = nullptr;
};

}  // namespace

struct pdm_uvit {
  pdm_uvit_cfg cfg;
  int D, H, Dh, Hid, C, p, n_patch, extras, Lx, Lm, P, P_pad, K, PK, PK_pad, depth, nhalf;
  std::vector<std::string> order;
  std::map<std::string, ParamSpec> params;
  // profiling hook: events around every GEMM launch of the last forward (bench roofline)
  mutable std::vector<hipEvent_t> prof_ev;
  mutable std::vector<double> prof_flops;
  mutable int prof_n = 0;
  mutable bool prof_on = false;

  void add(const std::string& name, int dtype, long long numel) {
    order.push_back(name);
    params[name] = ParamSpec{dtype, numel, nullptr};
  }
  const void* ptr(const std::string& name) const {
    auto it = params.find(name);
    return it == params.end() ? nullptr : it->second.ptr;
  }
  const float* f(const std::string& name) const { return static_cast<const float*>(ptr(name)); }
  const bf16* w(const std::string& name) const { return static_cast<const bf16*>(ptr(name)); }

  // norm1 / norm2 are folded into the next Linear (fused LayerNorm, see GemmArgs): the registered
  // attn.qkv.weight / mlp.fc1.weight are W * diag(norm.weight) in bf16, ln_colsum their row sums and ln_bias
  // W norm.bias (+ the Linear's own bias), both fp32 (include/pdm.h)
  // the residual stream is bf16 (cfg.residual_fp32 == 0)
  bool res16() const { return !cfg.residual_fp32; }
  // block Linear `bit` (0 qkv, 1 proj, 2 fc1, 3 fc2) runs in MXFP8 (cfg.fp8 / cfg.fp8_linears)
  bool f8(int bit) const { return cfg.fp8 && (((cfg.fp8_linears ? cfg.fp8_linears : 0xF) >> bit) & 1); }
  // a block Linear's weight [N][K]: bf16, or (MXFP8) e4m3 bytes + "<key>_scale" E8M0 dwords [K/128][N]; an MXFP8
  // LayerNorm consumer (qkv, fc1) also takes the bf16 hi / lo group sums "<lin>.ln_gcol" [N][16]
  void add_lin(const std::string& key, long long N, long long K, int bit, bool ln) {
    if (f8(bit)) {
      add(key, PDM_FP8, N * K);
      add(key + "_scale", PDM_E8M0, K / 128 * N);
      if (ln) add(key.substr(0, key.size() - 7) + ".ln_gcol", PDM_BF16, N * 16);
    } else {
      add(key, PDM_BF16, N * K);
    }
  }
  void add_block(const std::string& pre, bool skip) {
    add_lin(pre + ".attn.qkv.weight", 3LL * D, D, 0, true);
    add(pre + ".attn.qkv.ln_colsum", PDM_F32, 3LL * D);
    add(pre + ".attn.qkv.ln_bias", PDM_F32, 3LL * D);
    add_lin(pre + ".attn.proj.weight", D, D, 1, false);
    add(pre + ".attn.proj.bias", PDM_F32, D);
    add_lin(pre + ".mlp.fc1.weight", Hid, D, 2, true);
    add(pre + ".mlp.fc1.ln_colsum", PDM_F32, Hid);
    add(pre + ".mlp.fc1.ln_bias", PDM_F32, Hid);
    add_lin(pre + ".mlp.fc2.weight", D, Hid, 3, false);
    add(pre + ".mlp.fc2.bias", PDM_F32, D);
    if (skip) {
      add(pre + ".skip_linear.weight", PDM_BF16, 2LL * D * D);   // bf16 in both modes (run_block8)
      add(pre + ".skip_linear.bias", PDM_F32, D);
    }
  }
};

namespace {

// ------------------------------------------------------------------------------------------------
// An MXFP8 matrix in the GemmArgs operand layout: e4m3 rows q [rows][ld] (bytes) and E8M0 scale dwords
// s [K/128][sld].  cols(k0) is the same rows from column k0 on (k0 % 128 == 0).
struct Q8 {
  unsigned char* q = nullptr;
  int ld = 0;
  unsigned* s = nullptr;
  int sld = 0;
  Q8 cols(int k0) const { return Q8{q + k0, ld, s + (size_t)(k0 / 128) * sld, sld}; }
};

// workspace layout
struct Workspace {
  float* X;     // [rows*Lx, D] residual stream (image)
  bf16* XB;     // [rows*Lx, D] bf16 copy of x (qkv / skip_linear A operand)
  bf16* XT;     // [rows*Lmax, D] bf16 copy of the block-internal x (after skip_linear / attention)
  float* ST;    // [rows*Lmax, T] (sum, M2) LayerNorm partials of x at block entry / exit, T = ceil(D/256)
  float* STT;   // [rows*Lmax, T] partials of the block-internal x
  bf16* QKV;    // [rows*Lmax, 3D]
  bf16* ATT;    // [rows*Lmax, D]
  bf16* MLP;    // [rows*Lmax, Hid]
  bf16* SK;     // [nhalf][rows*Lx, D] long-skip activations (image)
  bf16* HEADIN; // [rows*n_patch, D]
  // t2i
  float* CTXF;  // [rows*n_ctx, D] embedded context (fp32)
  bf16* CTXB;   // [rows*n_ctx, clip_dim] bf16 context
  float* MX;    // [rows*Lm, D] mask stream
  bf16* MXB;    // [rows*Lm, D] bf16 copy of the mask-stream block output
  bf16* MXIN;   // [rows*Lm, D] bf16 copy of the mask-stream block input (qkv / skip_linear operand)
  bf16* MB;     // [rows*Lm, D] bf16 mask-stream block input (bf16 residual stream: MX is then only assembly scratch)
  bf16* SKM;    // [nhalf][rows*Lm, D]
  float* STM;   // [rows*Lm, T] LayerNorm partials of the mask stream
  // t2i on the bf16 stream: the image block's own scratch, so it runs in lockstep with the mask block of its layer
  // (every block Linear of the pair one grouped launch, run_block16_pair)
  bf16 *XT2, *QKV2, *ATT2, *MLP2;
  float* STT2;
  // fp8 forward (cfg.fp8): MXFP8 operands of the block Linears, e4m3 rows + E8M0 scale dwords [K/128][rows*Lx]
  Q8 xq;             // block input x (from the token assembly row pass)                 [rows*Lx, D]
  Q8 xtq;            // block-internal x (skip_linear / proj epilogues: qkv / fc1 operand) [rows*Lx, D]
  Q8 atq;            // attention output (proj operand)                                  [rows*Lx, D]
  Q8 mlq;            // GELU(fc1) (fc2 operand)                                          [rows*Lx, Hid]
  size_t bytes;
};

Workspace layout(const pdm_uvit* h, int rows, char* base) {
  Workspace w{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off = align_up(off + bytes, 256);
    return p;
  };
  const size_t D = h->D;
  const size_t Mx = (size_t)rows * h->Lx;
  const bool mask = h->cfg.t2i && h->cfg.separate && h->cfg.enable_panoptic;
  const size_t Mm = mask ? (size_t)rows * h->Lm : 0;
  const size_t Mmax = Mx > Mm ? Mx : Mm;
  const size_t T = (D + 255) / 256;
  const bool f8 = h->cfg.fp8 != 0;   // MXFP8 operands replace XT / MLP; XB / SK stay (bf16 skip_linear)
  w.X = (float*)take(Mx * D * 4);
  w.XB = (bf16*)take(Mx * D * 2);
  if (!f8 || !h->f8(2) || h->res16()) w.XT = (bf16*)take(Mmax * D * 2);   // (fp8: bf16 fc1 operand / bf16 stream)
  w.ST = (float*)take(Mmax * T * 8);
  w.STT = (float*)take(Mmax * T * 8);
  w.QKV = (bf16*)take(Mmax * 3 * D * 2);
  w.ATT = (bf16*)take(Mmax * D * 2);
  if (!f8) w.MLP = (bf16*)take(Mmax * h->Hid * 2);
  w.SK = (bf16*)take((size_t)h->nhalf * Mx * D * 2);
  w.HEADIN = (bf16*)take((size_t)rows * h->n_patch * D * 2);
  if (f8) {
    auto q8 = [&](size_t K) {
      Q8 r;
      r.q = (unsigned char*)take(Mx * K);
      r.ld = (int)K;
      r.s = (unsigned*)take(K / 128 * Mx * 4);
      r.sld = (int)Mx;
      return r;
    };
    w.xq = q8(D);
    w.xtq = q8(D);   // skip_linear output (qkv operand), and proj output (fc1 operand) when fc1 is MXFP8
    w.atq = q8(D);
    w.mlq = q8(h->Hid);
  }
  if (h->cfg.t2i) {
    w.CTXF = (float*)take((size_t)rows * h->cfg.num_clip_token * D * 4);
    w.CTXB = (bf16*)take((size_t)rows * h->cfg.num_clip_token * h->cfg.clip_dim * 2);
  }
  if (mask) {
    if (h->res16()) w.MB = (bf16*)take(Mm * D * 2);
    w.MX = (float*)take(Mm * D * 4);
    w.MXB = (bf16*)take(Mm * D * 2);
    w.MXIN = (bf16*)take(Mm * D * 2);
    w.STM = (float*)take(Mm * T * 8);
    w.SKM = (bf16*)take((size_t)h->nhalf * Mm * D * 2);
    if (h->res16() && !f8) {
      w.XT2 = (bf16*)take(Mx * D * 2);
      w.STT2 = (float*)take(Mx * T * 8);
      w.QKV2 = (bf16*)take(Mx * 3 * D * 2);
      w.ATT2 = (bf16*)take(Mx * D * 2);
      w.MLP2 = (bf16*)take(Mx * h->Hid * 2);
    }
  }
  w.bytes = off;   // (stream-K's flags and slab are library-owned per stream: sk_state)
  return w;
}

// ------------------------------------------------------------------------------------------------
struct Ctx {
  const pdm_uvit* h;
  hipStream_t s;
  // stream-K state of this forward (null: whole-tile GEMMs): flag blocks handed out one per GEMM launch
  unsigned* skf = nullptr;
  float* sks = nullptr;
  int* skn = nullptr;
};

// Stream-K state of the persistent GEMM (pdm::GemmArgs::sk_flags / sk_slab): SK_RING blocks of SK_FLAG_WORDS flag
// words (one block per GEMM launch) + one 64 MiB fp32 accumulator slab reused launch after launch in stream order.
// Owned by the library, one state per (device, stream), allocated on first use -- stream-K is off by default, so no
// forward workspace carries its 64 MiB, every device has its own (a process driving several GPUs), and
// concurrent streams (the sampling lanes) never share a slab.  Never allocated inside a stream capture: a forward
// captured on a stream without a state keeps whole tiles.
constexpr int SK_RING = 4096;
struct SkState {
  unsigned* flags = nullptr;
  float* slab = nullptr;
  int next = 0;   // next free flag block (host order of the launches on this stream); blocks past it are zero
};
static std::mutex g_sk_mu;
static std::map<std::pair<int, hipStream_t>, SkState> g_sk_state;

static int sk_state(hipStream_t s, SkState** out) {
  *out = nullptr;
  int dev = 0;
  PDM_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lock(g_sk_mu);
  auto it = g_sk_state.find({dev, s});
  if (it == g_sk_state.end()) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    PDM_HIP(hipStreamIsCapturing(s, &cs));
    if (cs != hipStreamCaptureStatusNone) return PDM_OK;   // no allocation inside a capture: whole tiles
    SkState st;
    PDM_HIP(hipMalloc(&st.flags, (size_t)SK_RING * pdm::SK_FLAG_WORDS * 4));
    PDM_HIP(hipMalloc(&st.slab, (size_t)pdm::SK_SLAB_BYTES));
    PDM_HIP(hipMemsetAsync(st.flags, 0, (size_t)SK_RING * pdm::SK_FLAG_WORDS * 4, s));
    it = g_sk_state.emplace(std::make_pair(dev, s), st).first;
  }
  *out = &it->second;
  return PDM_OK;
}

// a forward's stream-K state: SK_LAUNCHES flag blocks of the stream's ring, zeroed on the stream first (one memset
// node in a captured graph, so every replay starts from zeroed flags); none while the policy is off (a graph
// captured then keeps whole tiles)
int sk_begin(Ctx& c, int* counter) {
  *counter = 0;
  if (pdm::gemm_get_sk() == 0) return PDM_OK;
  SkState* st = nullptr;
  PDM_TRY(sk_state(c.s, &st));
  if (!st) return PDM_OK;
  if (st->next + SK_LAUNCHES > SK_RING) {   // wrap: the whole ring zeroed, so blocks past `next` stay clean
    PDM_HIP(hipMemsetAsync(st->flags, 0, (size_t)SK_RING * pdm::SK_FLAG_WORDS * 4, c.s));
    st->next = 0;
  }
  unsigned* f = st->flags + (size_t)st->next * pdm::SK_FLAG_WORDS;
  st->next += SK_LAUNCHES;
  PDM_HIP(hipMemsetAsync(f, 0, (size_t)SK_LAUNCHES * pdm::SK_FLAG_WORDS * 4, c.s));
  c.skf = f;
  c.sks = st->slab;
  c.skn = counter;
  return PDM_OK;
}

// fused-LayerNorm operands of one GEMM: partials produced (st_out) or consumed (st_in + colsum)
struct LnIO {
  float* st_out = nullptr;
  const float* st_in = nullptr;
  const float* colsum = nullptr;
};

// checked launch + the profiling hook (HIP events around every GEMM of the forward)
int launch_gemm(const Ctx& c, const pdm::GemmArgs& a, int epi) {
  PDM_CHECK(pdm::gemm_check(a, epi));
  const pdm_uvit* h = c.h;
  const bool prof = h->prof_on && 2 * (h->prof_n + 1) <= (int)h->prof_ev.size();
  pdm::GemmArgs b = a;
  if (c.skf && *c.skn < SK_LAUNCHES) {   // this launch's own zeroed flag block (used only if it takes stream-K)
    b.sk_flags = c.skf + (size_t)(*c.skn)++ * pdm::SK_FLAG_WORDS;
    b.sk_slab = c.sks;
  }
  if (prof) PDM_HIP(hipEventRecord(h->prof_ev[2 * h->prof_n], c.s));
  PDM_HIP(pdm::gemm_launch(b, epi, c.s));
  if (prof) {
    PDM_HIP(hipEventRecord(h->prof_ev[2 * h->prof_n + 1], c.s));
    h->prof_flops[h->prof_n] = 2.0 * a.M * a.N * a.K;
    ++h->prof_n;
  }
  return PDM_OK;
}

int gemm(const Ctx& c, const bf16* A, int lda, const bf16* W, const float* bias, int M, int N, int K, int epi,
         bf16* ob, int ldo, float* of, int ldr, int accumulate, const bf16* A2 = nullptr, int lda2 = 0, int K1 = 0,
         int a_rpg = 0, int a_gs = 0, LnIO ln = LnIO()) {
  pdm::GemmArgs a{};
  const int T = (c.h->D + 255) / 256;
  a.stats_out = ln.st_out; a.stats_ld = T;
  a.ln_stats = ln.st_in; a.ln_ld = T; a.ln_D = K; a.ln_eps = 1e-5f; a.ln_colsum = ln.colsum;
  a.A1 = A; a.lda1 = lda;
  a.A2 = A2; a.lda2 = lda2;
  a.K1 = A2 ? K1 : K;
  a.W = W; a.bias = bias;
  a.M = M; a.N = N; a.K = K;
  a.out_bf16 = ob; a.ldo = ldo;
  a.out_f32 = of; a.ldr = ldr;
  a.accumulate = accumulate;
  a.a_rows_per_group = a_rpg; a.a_group_stride = a_gs;
  return launch_gemm(c, a, epi);
}

// GemmArgs of a bf16 block Linear: the fused-LayerNorm consumer (ln.st_in, bf16 / GELU epilogue) or the bf16 residual
// epilogue (EPI_RES: out = bf16(A W^T + bias (+ res_in)), partials st_out; A2 = the split-K long-skip operand)
pdm::GemmArgs ln_args(const pdm_uvit* h, const bf16* A, const bf16* W, const float* bias, int M, int N, int K, bf16* out,
                      const float* st_in, const float* colsum) {
  pdm::GemmArgs a{};
  const int T = (h->D + 255) / 256;
  a.ln_stats = st_in; a.ln_ld = T; a.ln_D = K; a.ln_eps = 1e-5f; a.ln_colsum = colsum; a.stats_ld = T;
  a.A1 = A; a.lda1 = K; a.K1 = K;
  a.W = W; a.bias = bias;
  a.M = M; a.N = N; a.K = K;
  a.out_bf16 = out; a.ldo = N;
  return a;
}
pdm::GemmArgs res_args(const bf16* A, int lda, const bf16* W, const float* bias, int M, int N, int K, const bf16* res_in,
                       bf16* out, float* st_out, const bf16* A2 = nullptr, int lda2 = 0, int K1 = 0) {
  pdm::GemmArgs a{};
  a.A1 = A; a.lda1 = lda;
  a.A2 = A2; a.lda2 = lda2;
  a.K1 = A2 ? K1 : K;
  a.W = W; a.bias = bias;
  a.M = M; a.N = N; a.K = K;
  a.out_bf16 = out; a.ldo = N;
  a.res_in = res_in; a.ldri = N; a.accumulate = res_in ? 1 : 0;
  a.stats_out = st_out; a.stats_ld = (N + 255) / 256;
  return a;
}

// two GEMMs as one grouped launch where the kernel takes both (pdm::gemm_launch_pair), with the profiling hook
// counting the pair as one launch of their summed FLOPs
int launch_gemm_pair(const Ctx& c, const pdm::GemmArgs& a, const pdm::GemmArgs& b, int epi) {
  PDM_CHECK(pdm::gemm_check(a, epi));
  PDM_CHECK(pdm::gemm_check(b, epi));
  const pdm_uvit* h = c.h;
  // not grouped: two launches, each with its own profiling entry (the roofline counts launches)
  if (!pdm::gemm_pair_groups(a, b, epi)) {
    const int r = launch_gemm(c, a, epi);
    return r != PDM_OK ? r : launch_gemm(c, b, epi);
  }
  const bool prof = h->prof_on && 2 * (h->prof_n + 1) <= (int)h->prof_ev.size();
  if (prof) PDM_HIP(hipEventRecord(h->prof_ev[2 * h->prof_n], c.s));
  PDM_HIP(pdm::gemm_launch_pair(a, b, epi, c.s));
  if (prof) {
    PDM_HIP(hipEventRecord(h->prof_ev[2 * h->prof_n + 1], c.s));
    h->prof_flops[h->prof_n] = 2.0 * a.M * a.N * a.K + 2.0 * b.M * b.N * b.K;
    ++h->prof_n;
  }
  return PDM_OK;
}

// MXFP8 block Linear (cfg.fp8): A and the weight `wkey` (+ "<wkey>_scale") on the block-scaled MFMA; the
// epilogue also writes the MXFP8 copy of what it stores into `out` when out.q is set (the next Linear's operand)
// LayerNorm consumers (ln.st_in) take their A operand group-centred (GemmArgs::ln_gcol, "<lin>.ln_gcol"); an
// MXFP8 output written beside LayerNorm partials (ln.st_out) is group-centred (GemmArgs::mx_center).
// epi == EPI_RES: the bf16 residual stream, res_in (may alias ob) added when accumulate.
int gemm8(const Ctx& c, const Q8& A, const std::string& wkey, const float* bias, int M, int N, int K, int epi,
          bf16* ob, float* of, int accumulate, LnIO ln, const Q8& out, const bf16* res_in = nullptr) {
  const pdm_uvit* h = c.h;
  pdm::GemmArgs a{};
  const int T = (h->D + 255) / 256;
  a.stats_out = ln.st_out; a.stats_ld = T;
  a.ln_stats = ln.st_in; a.ln_ld = T; a.ln_D = K; a.ln_eps = 1e-5f; a.ln_colsum = ln.colsum;
  if (ln.st_in) a.ln_gcol = h->w(wkey.substr(0, wkey.size() - 7) + ".ln_gcol");
  a.mx_center = out.q && ln.st_out ? 1 : 0;
  a.A1 = (const bf16*)A.q; a.lda1 = A.ld; a.K1 = K;
  a.W = (const bf16*)h->ptr(wkey); a.bias = bias;
  a.M = M; a.N = N; a.K = K;
  a.out_bf16 = ob; a.ldo = ob ? N : 0;
  a.out_f32 = of; a.ldr = of ? h->D : 0; a.accumulate = accumulate;
  a.fp8 = 1;
  a.a_scale = A.s; a.a_scale_ld = A.sld;
  a.w_scale = (const unsigned*)h->ptr(wkey + "_scale"); a.w_scale_ld = N;
  a.out_fp8 = out.q; a.ldo8 = out.ld; a.out_scale = out.s; a.out_scale_ld = out.sld;
  a.res_in = res_in; a.ldri = res_in ? N : 0;
  return launch_gemm(c, a, epi);
}

// One U-ViT Block (libs/uvit.py:115-120) on `rows_L` token rows of width D held in X (fp32), with norm1 /
// norm2 fused into qkv / fc1 (GemmArgs): on entry xb_in = bf16(X) and st_in = the LayerNorm partials of X;
// the producing epilogues (skip_linear, proj, fc2) leave bf16(x) and its partials for the next consumer.
//   skip_in:          bf16 [rows_L, D] long-skip activation (out-blocks)
//   xb_out / st_out:  where fc2's epilogue writes bf16 of the block output and its partials (either may be null)
int run_block(const Ctx& c, const std::string& pre, float* X, int nseq, int L, const bf16* xb_in, const float* st_in,
              const bf16* skip_in, bf16* xb_out, float* st_out, const Workspace& w) {
  const pdm_uvit* h = c.h;
  const int D = h->D, M = nseq * L;
  const bf16* xb = xb_in;
  const float* st = st_in;
  if (skip_in) {  // x = skip_linear(cat([x, skip], -1)): split-K over the two bf16 operands
    LnIO io;
    io.st_out = w.STT;
    PDM_TRY(gemm(c, xb_in, D, h->w(pre + ".skip_linear.weight"), h->f(pre + ".skip_linear.bias"), M, D, 2 * D,
                 pdm::EPI_F32, w.XT, D, X, D, 0, skip_in, D, D, 0, 0, io));
    xb = w.XT;
    st = w.STT;
  }
  {  // qkv = norm1(x) W^T
    LnIO io;
    io.st_in = st;
    io.colsum = h->f(pre + ".attn.qkv.ln_colsum");
    PDM_TRY(gemm(c, xb, D, h->w(pre + ".attn.qkv.weight"), h->f(pre + ".attn.qkv.ln_bias"), M, 3 * D, D,
                 pdm::EPI_BF16, w.QKV, 3 * D, nullptr, 0, 0, nullptr, 0, 0, 0, 0, io));
  }
  {
    pdm::AttentionArgs a{};
    a.qkv = w.QKV; a.ldq = 3 * D;
    a.out = w.ATT; a.ldo = D;
    a.B = nseq; a.L = L; a.H = h->H; a.Dh = h->Dh;
    a.scale = 1.0f / sqrtf((float)h->Dh);
    a.q_log2 = 1;   // attn.qkv's q rows are packed pre-scaled by Dh^-0.5 log2(e) (include/pdm.h)
    PDM_CHECK(pdm::attention_check(a));
    PDM_HIP(pdm::attention_launch(a, c.s));
  }
  {  // x += proj(attn)
    LnIO io;
    io.st_out = w.STT;
    PDM_TRY(gemm(c, w.ATT, D, h->w(pre + ".attn.proj.weight"), h->f(pre + ".attn.proj.bias"), M, D, D, pdm::EPI_F32,
                 w.XT, D, X, D, 1, nullptr, 0, 0, 0, 0, io));
  }
  {  // h = GELU(fc1(norm2(x)))
    LnIO io;
    io.st_in = w.STT;
    io.colsum = h->f(pre + ".mlp.fc1.ln_colsum");
    PDM_TRY(gemm(c, w.XT, D, h->w(pre + ".mlp.fc1.weight"), h->f(pre + ".mlp.fc1.ln_bias"), M, h->Hid, D,
                 pdm::EPI_GELU, w.MLP, h->Hid, nullptr, 0, 0, nullptr, 0, 0, 0, 0, io));
  }
  {  // x += fc2(h)
    LnIO io;
    io.st_out = st_out;
    PDM_TRY(gemm(c, w.MLP, h->Hid, h->w(pre + ".mlp.fc2.weight"), h->f(pre + ".mlp.fc2.bias"), M, D, h->Hid,
                 pdm::EPI_F32, xb_out, D, X, D, 1, nullptr, 0, 0, 0, 0, io));
  }
  return PDM_OK;
}

// Residual GEMM on the bf16 residual stream (EPI_RES): out = bf16(A W^T + bias (+ res_in)) and its LayerNorm
// partials (st_out).  res_in may alias out.
int gemm_res(const Ctx& c, const bf16* A, int lda, const bf16* W, const float* bias, int M, int N, int K,
             const bf16* res_in, bf16* out, float* st_out, const bf16* A2 = nullptr, int lda2 = 0, int K1 = 0) {
  pdm::GemmArgs a{};
  a.A1 = A; a.lda1 = lda;
  a.A2 = A2; a.lda2 = lda2;
  a.K1 = A2 ? K1 : K;
  a.W = W; a.bias = bias;
  a.M = M; a.N = N; a.K = K;
  a.out_bf16 = out; a.ldo = N;
  a.res_in = res_in; a.ldri = N; a.accumulate = res_in ? 1 : 0;
  a.stats_out = st_out; a.stats_ld = (N + 255) / 256;
  return launch_gemm(c, a, pdm::EPI_RES);
}

// One U-ViT Block on the bf16 residual stream (the reference under bf16 autocast keeps x in the autocast dtype:
// each Linear's output is added to x in that dtype).  xin = the block input x (bf16) with partials st_in; the
// block output goes to xout (may equal xin only when xin is not needed afterwards) with partials st_out.  The
// block-internal x lives in XT.  Per residual GEMM the epilogue moves 2 + 2 bytes per element instead of the
// fp32 stream's 4 + 4 + a 2-byte bf16 operand copy.
int run_block16(const Ctx& c, const std::string& pre, int nseq, int L, const bf16* xin, const float* st_in,
                const bf16* skip_in, bf16* xout, float* st_out, const Workspace& w) {
  const pdm_uvit* h = c.h;
  const int D = h->D, M = nseq * L;
  const bf16* x = xin;
  const float* st = st_in;
  if (skip_in) {  // x = skip_linear(cat([x, skip], -1)): split-K over the two bf16 operands
    PDM_TRY(gemm_res(c, xin, D, h->w(pre + ".skip_linear.weight"), h->f(pre + ".skip_linear.bias"), M, D, 2 * D,
                     nullptr, w.XT, w.STT, skip_in, D, D));
    x = w.XT;
    st = w.STT;
  }
  {  // qkv = norm1(x) W^T
    LnIO io;
    io.st_in = st;
    io.colsum = h->f(pre + ".attn.qkv.ln_colsum");
    PDM_TRY(gemm(c, x, D, h->w(pre + ".attn.qkv.weight"), h->f(pre + ".attn.qkv.ln_bias"), M, 3 * D, D,
                 pdm::EPI_BF16, w.QKV, 3 * D, nullptr, 0, 0, nullptr, 0, 0, 0, 0, io));
  }
  {
    pdm::AttentionArgs a{};
    a.qkv = w.QKV; a.ldq = 3 * D;
    a.out = w.ATT; a.ldo = D;
    a.B = nseq; a.L = L; a.H = h->H; a.Dh = h->Dh;
    a.scale = 1.0f / sqrtf((float)h->Dh);
    a.q_log2 = 1;   // attn.qkv's q rows are packed pre-scaled by Dh^-0.5 log2(e) (include/pdm.h)
    PDM_CHECK(pdm::attention_check(a));
    PDM_HIP(pdm::attention_launch(a, c.s));
  }
  // x += proj(attn) -> XT (in place when x already is XT; xin itself may be a long-skip operand kept for later)
  PDM_TRY(gemm_res(c, w.ATT, D, h->w(pre + ".attn.proj.weight"), h->f(pre + ".attn.proj.bias"), M, D, D, x, w.XT,
                   w.STT));
  {  // h = GELU(fc1(norm2(x)))
    LnIO io;
    io.st_in = w.STT;
    io.colsum = h->f(pre + ".mlp.fc1.ln_colsum");
    PDM_TRY(gemm(c, w.XT, D, h->w(pre + ".mlp.fc1.weight"), h->f(pre + ".mlp.fc1.ln_bias"), M, h->Hid, D,
                 pdm::EPI_GELU, w.MLP, h->Hid, nullptr, 0, 0, nullptr, 0, 0, 0, 0, io));
  }
  // x += fc2(h) -> xout
  PDM_TRY(gemm_res(c, w.MLP, h->Hid, h->w(pre + ".mlp.fc2.weight"), h->f(pre + ".mlp.fc2.bias"), M, D, h->Hid, w.XT,
                   xout, st_out));
  return PDM_OK;
}

// One block of each t2i stream in lockstep on the bf16 residual stream (run_block16's sequence): every Linear of the
// two blocks (same D / Hid, different weights, rows and buffers) is one grouped launch, attention runs per stream.
// The t2i layer's image (L = 334) and mask (L = 590) blocks are independent given x, and each alone launches under
// one wave of 256-row tiles at the bench's rows (t2i B = 32 per GPU as two lanes: 84 / 148 tiles for N = 512).
struct BlockIO {
  std::string pre;
  int L;
  const bf16* xin;
  const float* st_in;
  const bf16* skip_in;
  bf16* xout;
  float* st_out;
  bf16 *XT, *QKV, *ATT, *MLP;
  float* STT;
};
int run_block16_pair(const Ctx& c, int nseq, const BlockIO& A, const BlockIO& B) {
  const pdm_uvit* h = c.h;
  const int D = h->D;
  const int Ma = nseq * A.L, Mb = nseq * B.L;
  const bf16* xa = A.xin;
  const bf16* xb = B.xin;
  const float* sa = A.st_in;
  const float* sb = B.st_in;
  if (A.skip_in || B.skip_in) {   // x = skip_linear(cat([x, skip], -1)); both streams have long skips or neither
    if (!A.skip_in || !B.skip_in) return fail(PDM_ERR_STATE, "run_block16_pair: long skip in one stream only");
    PDM_TRY(launch_gemm_pair(c,
        res_args(A.xin, D, h->w(A.pre + ".skip_linear.weight"), h->f(A.pre + ".skip_linear.bias"), Ma, D, 2 * D, nullptr,
                 A.XT, A.STT, A.skip_in, D, D),
        res_args(B.xin, D, h->w(B.pre + ".skip_linear.weight"), h->f(B.pre + ".skip_linear.bias"), Mb, D, 2 * D, nullptr,
                 B.XT, B.STT, B.skip_in, D, D),
        pdm::EPI_RES));
    xa = A.XT; sa = A.STT;
    xb = B.XT; sb = B.STT;
  }
  PDM_TRY(launch_gemm_pair(c,   // qkv = norm1(x) W^T
      ln_args(h, xa, h->w(A.pre + ".attn.qkv.weight"), h->f(A.pre + ".attn.qkv.ln_bias"), Ma, 3 * D, D, A.QKV, sa,
              h->f(A.pre + ".attn.qkv.ln_colsum")),
      ln_args(h, xb, h->w(B.pre + ".attn.qkv.weight"), h->f(B.pre + ".attn.qkv.ln_bias"), Mb, 3 * D, D, B.QKV, sb,
              h->f(B.pre + ".attn.qkv.ln_colsum")),
      pdm::EPI_BF16));
  for (const BlockIO* io : {&A, &B}) {
    pdm::AttentionArgs a{};
    a.qkv = io->QKV; a.ldq = 3 * D;
    a.out = io->ATT; a.ldo = D;
    a.B = nseq; a.L = io->L; a.H = h->H; a.Dh = h->Dh;
    a.scale = 1.0f / sqrtf((float)h->Dh);
    a.q_log2 = 1;
    PDM_CHECK(pdm::attention_check(a));
    PDM_HIP(pdm::attention_launch(a, c.s));
  }
  PDM_TRY(launch_gemm_pair(c,   // x += proj(attn) -> XT
      res_args(A.ATT, D, h->w(A.pre + ".attn.proj.weight"), h->f(A.pre + ".attn.proj.bias"), Ma, D, D, xa, A.XT, A.STT),
      res_args(B.ATT, D, h->w(B.pre + ".attn.proj.weight"), h->f(B.pre + ".attn.proj.bias"), Mb, D, D, xb, B.XT, B.STT),
      pdm::EPI_RES));
  PDM_TRY(launch_gemm_pair(c,   // h = GELU(fc1(norm2(x)))
      ln_args(h, A.XT, h->w(A.pre + ".mlp.fc1.weight"), h->f(A.pre + ".mlp.fc1.ln_bias"), Ma, h->Hid, D, A.MLP, A.STT,
              h->f(A.pre + ".mlp.fc1.ln_colsum")),
      ln_args(h, B.XT, h->w(B.pre + ".mlp.fc1.weight"), h->f(B.pre + ".mlp.fc1.ln_bias"), Mb, h->Hid, D, B.MLP, B.STT,
              h->f(B.pre + ".mlp.fc1.ln_colsum")),
      pdm::EPI_GELU));
  PDM_TRY(launch_gemm_pair(c,   // x += fc2(h) -> xout
      res_args(A.MLP, h->Hid, h->w(A.pre + ".mlp.fc2.weight"), h->f(A.pre + ".mlp.fc2.bias"), Ma, D, h->Hid, A.XT, A.xout,
               A.st_out),
      res_args(B.MLP, h->Hid, h->w(B.pre + ".mlp.fc2.weight"), h->f(B.pre + ".mlp.fc2.bias"), Mb, D, h->Hid, B.XT, B.xout,
               B.st_out),
      pdm::EPI_RES));
  return PDM_OK;
}

// bf16 copy + LayerNorm partials of fp32 rows no GEMM epilogue produced (token assembly, mask-stream refresh)
int row_stats(const Ctx& c, const float* X, int rows, bf16* xb, float* st) {
  const int D = c.h->D;
  PDM_HIP(pdm::rowstats_launch(X, D, rows, D, xb, D, st, (D + 255) / 256, c.s));
  return PDM_OK;
}

// The single-stream block stack (libs/uvit.py:213-222, libs/uvit_t2i.py:407-410 / 516): X holds the assembled
// tokens; in-block i leaves bf16 of its output in SK[i] (the long-skip operand and the next block's A operand).
int run_stack(const Ctx& c, const Workspace& w, int rows, int L) {
  const pdm_uvit* h = c.h;
  const size_t MD = (size_t)rows * L * h->D;
  PDM_TRY(row_stats(c, w.X, rows * L, w.XB, w.ST));
  const bf16* xb = w.XB;
  for (int i = 0; i < h->nhalf; ++i) {
    PDM_TRY(run_block(c, "in_blocks." + std::to_string(i), w.X, rows, L, xb, w.ST, nullptr, w.SK + i * MD, w.ST, w));
    xb = w.SK + i * MD;
  }
  PDM_TRY(run_block(c, "mid_block", w.X, rows, L, xb, w.ST, nullptr, w.XB, w.ST, w));
  for (int i = 0; i < h->nhalf; ++i) {
    const bf16* sk = h->cfg.skip ? w.SK + (h->nhalf - 1 - i) * MD : nullptr;
    const bool last = i + 1 == h->nhalf;
    PDM_TRY(run_block(c, "out_blocks." + std::to_string(i), w.X, rows, L, w.XB, w.ST, sk, last ? nullptr : w.XB,
                      last ? nullptr : w.ST, w));
  }
  return PDM_OK;
}

// The block stack on the bf16 residual stream: the assembled fp32 tokens X become bf16 XB (+ partials); in-block
// i leaves its output in SK[i] (the long skip and the next block's input); mid / out-blocks update XB.
int run_stack16(const Ctx& c, const Workspace& w, int rows, int L) {
  const pdm_uvit* h = c.h;
  const size_t MD = (size_t)rows * L * h->D;
  PDM_TRY(row_stats(c, w.X, rows * L, w.XB, w.ST));
  const bf16* x = w.XB;
  for (int i = 0; i < h->nhalf; ++i) {
    PDM_TRY(run_block16(c, "in_blocks." + std::to_string(i), rows, L, x, w.ST, nullptr, w.SK + i * MD, w.ST, w));
    x = w.SK + i * MD;
  }
  PDM_TRY(run_block16(c, "mid_block", rows, L, x, w.ST, nullptr, w.XB, w.ST, w));
  for (int i = 0; i < h->nhalf; ++i) {
    const bf16* sk = h->cfg.skip ? w.SK + (h->nhalf - 1 - i) * MD : nullptr;
    PDM_TRY(run_block16(c, "out_blocks." + std::to_string(i), rows, L, w.XB, w.ST, sk, w.XB, w.ST, w));
  }
  return PDM_OK;
}

// One U-ViT Block with MXFP8 qkv / proj / fc1 / fc2 (cfg.fp8, BASELINE configs[4]).  `in` is the MXFP8 block
// input x with LayerNorm partials st_in.  Out-blocks with a long skip start from skip_linear(cat([x, skip]))
// (libs/uvit.py:116-117) instead, kept in bf16 on the split-K GEMM over xb_in / skip_in: its output REPLACES the
// residual stream, and in MXFP8 it alone costs 6.3e-2 rel-L2 of the H/4 forward (vs 1.6-4.4e-2 for each of the
// other Linears; fp32 fake-quant of the oracle) for 7 % of the FLOPs.  Attention stays bf16 (a
// 72-deep QK^T cannot fill the 128-deep scaled MFMA, and the unscaled fp8 MFMA runs at the bf16 rate); its output
// is MX-quantised for proj.  fc2 leaves the block output as MXFP8 in out8 and / or bf16 in outb (either may be
// null) and its partials in st_out.
//
// X == nullptr: the bf16 residual stream (cfg.residual_fp32 == 0): xb_in is the block input x itself (bf16), the
// residual epilogues are EPI_RES, the block-internal x lives in XT and the block output goes to outb (required).
int run_block8(const Ctx& c, const std::string& pre, float* X, int M, int L, const Q8& in, const float* st_in,
               const bf16* xb_in, const bf16* skip_in, const Q8& out8, bf16* outb, float* st_out, const Workspace& w) {
  const pdm_uvit* h = c.h;
  const int D = h->D;
  const bool r16 = X == nullptr;
  Q8 a = in;
  const float* st = st_in;
  const bf16* res = xb_in;   // (r16) the residual x the block adds to
  if (skip_in) {  // x = skip_linear(cat([x, skip], -1)) -> X (fp32) / XT (bf16) + its MXFP8 copy (qkv operand) + partials
    pdm::GemmArgs g{};
    g.A1 = xb_in; g.lda1 = D; g.A2 = skip_in; g.lda2 = D; g.K1 = D;
    g.W = h->w(pre + ".skip_linear.weight"); g.bias = h->f(pre + ".skip_linear.bias");
    g.M = M; g.N = D; g.K = 2 * D;
    if (r16) { g.out_bf16 = w.XT; g.ldo = D; }
    else { g.out_f32 = X; g.ldr = D; }
    g.stats_out = w.STT; g.stats_ld = (D + 255) / 256;
    g.out_fp8 = w.xtq.q; g.ldo8 = w.xtq.ld; g.out_scale = w.xtq.s; g.out_scale_ld = w.xtq.sld;
    g.mx_center = 1;
    PDM_TRY(launch_gemm(c, g, r16 ? pdm::EPI_RES : pdm::EPI_F32));
    a = w.xtq;
    st = w.STT;
    res = w.XT;
  }
  {  // qkv = norm1(x) W^T (bf16 for the attention kernel)
    LnIO io;
    io.st_in = st;
    io.colsum = h->f(pre + ".attn.qkv.ln_colsum");
    PDM_TRY(gemm8(c, a, pre + ".attn.qkv.weight", h->f(pre + ".attn.qkv.ln_bias"), M, 3 * D, D, pdm::EPI_BF16, w.QKV,
                  nullptr, 0, io, Q8()));
  }
  {
    pdm::AttentionArgs at{};
    at.qkv = w.QKV; at.ldq = 3 * D;
    at.out = w.ATT; at.ldo = D;
    at.B = M / L; at.L = L; at.H = h->H; at.Dh = h->Dh;
    at.scale = 1.0f / sqrtf((float)h->Dh);
    at.q_log2 = 1;
    PDM_CHECK(pdm::attention_check(at));
    PDM_HIP(pdm::attention_launch(at, c.s));
    PDM_HIP(pdm::mxq_launch(w.ATT, 1, D, M, D, w.atq.q, w.atq.ld, w.atq.s, w.atq.sld, c.s));
  }
  const bool fc1_8 = h->f8(2);
  {  // x += proj(attn) -> X / XT, its partials and the fc1 operand (centred MXFP8, or bf16 for a bf16 fc1)
    LnIO io;
    io.st_out = w.STT;
    if (r16)
      PDM_TRY(gemm8(c, w.atq, pre + ".attn.proj.weight", h->f(pre + ".attn.proj.bias"), M, D, D, pdm::EPI_RES, w.XT,
                    nullptr, 1, io, fc1_8 ? w.xtq : Q8(), res));
    else
      PDM_TRY(gemm8(c, w.atq, pre + ".attn.proj.weight", h->f(pre + ".attn.proj.bias"), M, D, D, pdm::EPI_F32,
                    fc1_8 ? nullptr : w.XT, X, 1, io, fc1_8 ? w.xtq : Q8()));
  }
  {  // h = GELU(fc1(norm2(x))), stored only as the MXFP8 fc2 operand
    LnIO io;
    io.st_in = w.STT;
    io.colsum = h->f(pre + ".mlp.fc1.ln_colsum");
    if (fc1_8) {
      PDM_TRY(gemm8(c, w.xtq, pre + ".mlp.fc1.weight", h->f(pre + ".mlp.fc1.ln_bias"), M, h->Hid, D, pdm::EPI_GELU,
                    nullptr, nullptr, 0, io, w.mlq));
    } else {   // bf16 MFMA, fused LayerNorm on the bf16 copy, GELU epilogue emitting the MXFP8 fc2 operand only
      pdm::GemmArgs g{};
      const int T = (D + 255) / 256;
      g.A1 = w.XT; g.lda1 = D; g.K1 = D;
      g.W = h->w(pre + ".mlp.fc1.weight"); g.bias = h->f(pre + ".mlp.fc1.ln_bias");
      g.M = M; g.N = h->Hid; g.K = D;
      g.ln_stats = w.STT; g.ln_ld = T; g.ln_D = D; g.ln_eps = 1e-5f; g.ln_colsum = io.colsum;
      g.out_fp8 = w.mlq.q; g.ldo8 = w.mlq.ld; g.out_scale = w.mlq.s; g.out_scale_ld = w.mlq.sld;
      PDM_TRY(launch_gemm(c, g, pdm::EPI_GELU));
    }
  }
  {  // x += fc2(h)
    LnIO io;
    io.st_out = st_out;
    if (r16)
      PDM_TRY(gemm8(c, w.mlq, pre + ".mlp.fc2.weight", h->f(pre + ".mlp.fc2.bias"), M, D, h->Hid, pdm::EPI_RES, outb,
                    nullptr, 1, io, out8, w.XT));
    else
      PDM_TRY(gemm8(c, w.mlq, pre + ".mlp.fc2.weight", h->f(pre + ".mlp.fc2.bias"), M, D, h->Hid, pdm::EPI_F32, outb,
                    X, 1, io, out8));
  }
  return PDM_OK;
}

// run_stack8 on the bf16 residual stream: in-block i leaves x in SK[i] (bf16: the long skip and the next block's
// residual) and MXFP8 xq (the next qkv operand); the mid / out-blocks update XB.
int run_stack8_16(const Ctx& c, const Workspace& w, int rows, int L) {
  const pdm_uvit* h = c.h;
  const int D = h->D, M = rows * L, n = h->nhalf;
  const bool skip = h->cfg.skip != 0;
  const size_t MD = (size_t)M * D;
  PDM_HIP(pdm::rowstats_launch(w.X, D, M, D, w.XB, D, w.ST, (D + 255) / 256, c.s, w.xq.q, w.xq.ld, w.xq.s,
                               w.xq.sld, 1));
  // a block reads its input x (skip_linear or proj) before fc2 writes the output, so XB can be updated in place;
  // in-block outputs with long skips are kept in SK[i]
  const bf16* x = w.XB;
  for (int i = 0; i < n; ++i) {
    bf16* o = skip ? w.SK + i * MD : w.XB;
    PDM_TRY(run_block8(c, "in_blocks." + std::to_string(i), nullptr, M, L, w.xq, w.ST, x, nullptr, w.xq, o, w.ST, w));
    x = o;
  }
  PDM_TRY(run_block8(c, "mid_block", nullptr, M, L, w.xq, w.ST, x, nullptr, skip ? Q8() : w.xq, w.XB, w.ST, w));
  for (int i = 0; i < n; ++i)
    PDM_TRY(run_block8(c, "out_blocks." + std::to_string(i), nullptr, M, L, w.xq, w.ST, w.XB,
                       skip ? w.SK + (n - 1 - i) * MD : nullptr, skip ? Q8() : w.xq, w.XB, w.ST, w));
  return PDM_OK;
}

// The block stack with MXFP8 block Linears: in-blocks leave their output as MXFP8 (the next block's operand) and
// as bf16 in SK[i] (the long skip); the mid block and out-blocks leave bf16 x in XB for the next skip_linear (or,
// without long skips, MXFP8 x for the next qkv).  Every activation is produced once, by the epilogue that computes
// it, in the precision and layout of its consumer.
int run_stack8(const Ctx& c, const Workspace& w, int rows, int L) {
  const pdm_uvit* h = c.h;
  const int D = h->D, M = rows * L, n = h->nhalf;
  const bool skip = h->cfg.skip != 0;
  const size_t MD = (size_t)M * D;
  PDM_HIP(pdm::rowstats_launch(w.X, D, M, D, nullptr, 0, w.ST, (D + 255) / 256, c.s, w.xq.q, w.xq.ld, w.xq.s,
                               w.xq.sld, 1));
  for (int i = 0; i < n; ++i)
    PDM_TRY(run_block8(c, "in_blocks." + std::to_string(i), w.X, M, L, w.xq, w.ST, nullptr, nullptr, w.xq,
                       skip ? w.SK + i * MD : nullptr, w.ST, w));
  PDM_TRY(run_block8(c, "mid_block", w.X, M, L, w.xq, w.ST, nullptr, nullptr, skip ? Q8() : w.xq,
                     skip ? w.XB : nullptr, w.ST, w));
  for (int i = 0; i < n; ++i) {
    const bool last = i + 1 == n;
    PDM_TRY(run_block8(c, "out_blocks." + std::to_string(i), w.X, M, L, w.xq, w.ST, w.XB,
                       skip ? w.SK + (n - 1 - i) * MD : nullptr, last || skip ? Q8() : w.xq,
                       last || !skip ? nullptr : w.XB, last ? nullptr : w.ST, w));
  }
  return PDM_OK;
}

int check_ready(pdm_uvit* h) {
  for (auto& n : h->order)
    if (!h->params[n].ptr) return fail(PDM_ERR_STATE, "pdm_uvit: weight not registered: " + n);
  return PDM_OK;
}

// decoder_pred-style head on bf16 token rows: token (b, i) is row b * group_stride + row_offset + i of `hin`.
int run_head(const Ctx& c, const bf16* hin, int group_stride, int row_offset, int rows, const std::string& head,
             int Cout, int P, int P_pad, float* out) {
  const pdm_uvit* h = c.h;
  pdm::HeadArgs a{};
  a.x = hin; a.ldx = h->D;
  a.in_group_stride = group_stride; a.in_row_offset = row_offset;
  a.W = h->w(head + ".weight"); a.bias = h->f(head + ".bias");
  a.out = out;
  a.B = rows; a.D = h->D; a.C = Cout; a.p = h->p; a.Himg = h->cfg.img_size; a.Wimg = h->cfg.img_size;
  a.P = P; a.P_pad = P_pad; a.act_tanh = 0;
  PDM_CHECK(pdm::head_check(a));
  PDM_HIP(pdm::head_launch(a, c.s));
  return PDM_OK;
}

// final LayerNorm over the patch tokens of X (rows extras .. L-1 of each sequence) -> HEADIN, optionally
// adding fp32 rows `add` (use_ground_truth: libs/uvit_t2i.py:486-494) after the affine
int final_norm(const Ctx& c, const Workspace& w, int rows, const float* X, int L, const float* add = nullptr,
               int add_gs = 0, int add_off = 0, const bf16* Xb = nullptr, const bf16* addb = nullptr) {
  const pdm_uvit* h = c.h;
  pdm::LayerNormArgs a{};
  a.x = Xb ? nullptr : X; a.xb = Xb; a.ldx = h->D;
  a.addb = addb;
  a.gamma = h->f("norm.weight"); a.beta = h->f("norm.bias");
  a.y = w.HEADIN; a.ldy = h->D;
  a.rows = rows * h->n_patch; a.D = h->D;
  a.rows_per_group = h->n_patch; a.group_stride = L; a.row_offset = h->extras;
  a.eps = 1e-5f;
  a.add = add; a.add_ld = h->D; a.add_group_stride = add_gs; a.add_row_offset = add_off;
  PDM_CHECK(pdm::layernorm_check(a));
  PDM_HIP(pdm::layernorm_launch(a, c.s));
  return PDM_OK;
}

// The panoptic two-stream U-ViT (libs/uvit_t2i.py:411-525) on the bf16 residual stream, after the image tokens
// (X) and the mask tokens (MX[:, Lx:]) were assembled in fp32.  Per layer: the mask stream input mb = cat(x, m)
// is rebuilt in MB (image rows copied from the image block's INPUT x, 426 / 443 / 459; mask rows from the
// previous mask block's output), both blocks run, then x += zeroconv(mask block output[:, :Lx]) (435-436,
// 452-453, 470-472) as a residual GEMM into the image output buffer.
int t2i_two_stream16(const Ctx& c, const Workspace& w, int rows, int use_ground_truth, float* eps_pre,
                     float* mask_pre) {
  const pdm_uvit* h = c.h;
  const int D = h->D, Lx = h->Lx, Lm = h->Lm, n = h->nhalf, T = (D + 255) / 256;
  const size_t MDx = (size_t)rows * Lx * D, MDm = (size_t)rows * Lm * D;
  // bf16 row copies of D columns (as fp32 words: D / 2 per row), optionally with the rows' LayerNorm partials
  auto copy_rows = [&](bf16* dst, const bf16* src, int rpg, int dgs, int sgs, float* st_dst = nullptr,
                       const float* st_src = nullptr) -> int {
    PDM_HIP(pdm::rowcopy_launch((float*)dst, D / 2, (const float*)src, D / 2, rows * rpg, D / 2, rpg, dgs, sgs, c.s,
                                st_dst, 2 * T, st_src, 2 * T, 2 * T));
    return PDM_OK;
  };
  // mb = cat(x_img, m_src[:, Lx:]) + its partials (m_src == MB: the mask rows are already in place).  The mask
  // rows' LayerNorm partials are already in STM (written there by the mask block that produced m_src, in its fc2
  // epilogue, or by the token assembly).  The image rows and their partials come from the injection GEMM's second
  // output (img_in_place), and only before the first layer from x itself (XB / ST of the assembly).
  auto refresh = [&](const bf16* x_img, const bf16* m_src, bool img_in_place) -> int {
    if (!img_in_place) PDM_TRY(copy_rows(w.MB, x_img, Lx, Lm, Lx, w.STM, w.ST));
    if (m_src != w.MB) PDM_TRY(copy_rows(w.MB + (size_t)Lx * D, m_src + (size_t)Lx * D, Lm - Lx, Lm, Lm));
    return PDM_OK;
  };
  // x_out = x_res + zeroconv(mout[:, :Lx]), also stored (with its partials) as the image rows of MB -- the next
  // layer's mask-stream input; mout (SKM[i] / MXB) is never MB, so no tile reads rows another one writes
  auto inject = [&](int layer, const bf16* mout, const bf16* x_res, bf16* x_out) -> int {
    const std::string zc = "zero_convs." + std::to_string(2 * layer + 1) + ".conv";
    pdm::GemmArgs a{};
    a.A1 = mout; a.lda1 = D; a.K1 = D;
    a.a_rows_per_group = Lx; a.a_group_stride = Lm;
    a.W = h->w(zc + ".weight"); a.bias = h->f(zc + ".bias");
    a.M = rows * Lx; a.N = D; a.K = D;
    a.out_bf16 = x_out; a.ldo = D;
    a.res_in = x_res; a.ldri = D; a.accumulate = 1;
    a.stats_out = w.ST; a.stats_ld = T;
    a.out2 = w.MB; a.out2_rpg = Lx; a.out2_gs = Lm;
    a.stats_out2 = w.STM;
    return launch_gemm(c, a, pdm::EPI_RES);
  };
  // image tokens -> XB + ST; mask tokens -> MB[:, Lx:] (the image rows of this pass are overwritten by refresh)
  PDM_TRY(row_stats(c, w.X, rows * Lx, w.XB, w.ST));
  PDM_TRY(row_stats(c, w.MX, rows * Lm, w.MB, w.STM));
  const bf16* x = w.XB;
  const bf16* m = w.MB;
  int layer = 0;
  // Per layer the mask block runs first (its input only needs the image block's INPUT x), then the image block,
  // whose output stays in XT (its proj / fc2 update XT in place), then the injection writes the layer's x.  The
  // mask block's fc2 writes its output's partials into STM (the next refresh keeps the mask rows' ones); the
  // image block's are not needed (the injection produces x's).
  // the mask block and the image block of a layer: paired (one grouped launch per Linear) when the image stream has
  // its own scratch (the image block's output then lives in XT2 instead of XT), else one after the other
  const bool pair = w.XT2 != nullptr;
  bf16* ximg = pair ? w.XT2 : w.XT;   // the image block's output (the injection's residual)
  auto blocks = [&](const std::string& mpre, const std::string& ipre, const bf16* skm, const bf16* sk, const bf16* xin,
                    bf16* mout) -> int {
    if (pair) {
      const BlockIO mio{mpre, Lm, w.MB, w.STM, skm, mout, w.STM, w.XT, w.QKV, w.ATT, w.MLP, w.STT};
      // the image block's fc2 partials are not needed (the injection produces x's); they land in its scratch STT2
      // so both fc2s take the same epilogue and group
      const BlockIO iio{ipre, Lx, xin, w.ST, sk, w.XT2, w.STT2, w.XT2, w.QKV2, w.ATT2, w.MLP2, w.STT2};
      return run_block16_pair(c, rows, mio, iio);
    }
    PDM_TRY(run_block16(c, mpre, rows, Lm, w.MB, w.STM, skm, mout, w.STM, w));
    return run_block16(c, ipre, rows, Lx, xin, w.ST, sk, w.XT, nullptr, w);
  };
  for (int i = 0; i < n; ++i, ++layer) {
    PDM_TRY(refresh(x, m, i > 0));
    PDM_TRY(blocks("in_blocks_mask." + std::to_string(i), "in_blocks." + std::to_string(i), nullptr, nullptr, x,
                   w.SKM + i * MDm));
    PDM_TRY(inject(layer, w.SKM + i * MDm, ximg, w.SK + i * MDx));
    x = w.SK + i * MDx;
    m = w.SKM + i * MDm;
  }
  PDM_TRY(refresh(x, m, n > 0));
  PDM_TRY(blocks("mid_block_mask", "mid_block", nullptr, nullptr, x, w.MXB));
  PDM_TRY(inject(layer, w.MXB, ximg, w.XB));
  ++layer;
  for (int i = 0; i < n; ++i, ++layer) {
    PDM_TRY(refresh(w.XB, w.MXB, true));
    const bf16* skm = h->cfg.skip ? w.SKM + (n - 1 - i) * MDm : nullptr;
    const bf16* sk = h->cfg.skip ? w.SK + (n - 1 - i) * MDx : nullptr;
    PDM_TRY(blocks("out_blocks_mask." + std::to_string(i), "out_blocks." + std::to_string(i), skm, sk, w.XB, w.MXB));
    PDM_TRY(inject(layer, w.MXB, ximg, w.XB));
  }
  // heads (477-519): noise from norm(x) patch tokens; mask head on the un-normalised m (the last mask output)
  if (use_ground_truth) {
    PDM_TRY(final_norm(c, w, rows, nullptr, Lx, nullptr, Lm, Lx, w.XB, w.MXB));
  } else {
    PDM_TRY(final_norm(c, w, rows, nullptr, Lx, nullptr, 0, 0, w.XB));
    PDM_TRY(run_head(c, w.MXB, Lm, Lx, rows, "decoder_pred_mask", h->K, h->PK, h->PK_pad, mask_pre));
  }
  PDM_TRY(run_head(c, w.HEADIN, h->n_patch, 0, rows, "decoder_pred", h->C, h->P, h->P_pad, eps_pre));
  return PDM_OK;
}

}  // namespace

// ==================================================================================================
extern "C" {

const char* pdm_last_error(void) { return g_err.c_str(); }

int pdm_version(void) { return 1; }

int pdm_set_gemm_algo(int algo) {
  if (algo < 0 || algo > 11 || algo == 10)
    return fail(PDM_ERR_ARG, "pdm_set_gemm_algo: algo must be 0 (auto), 1..9 or 11");
  pdm::gemm_set_algo(algo);
  return PDM_OK;
}

int pdm_set_gemm_sk(int mode) {
  if ((mode & 3) > 2 || mode < 0 || mode > 7) return fail(PDM_ERR_ARG, "pdm_set_gemm_sk: mode must be 0..2 (+4)");
  pdm::gemm_set_sk(mode & 3);
  g_sk_standalone = (mode & 4) != 0;
  return PDM_OK;
}

long long pdm_gemm_sk_launches(void) { return pdm::gemm_sk_launches(); }

int pdm_gemm_seg_stats(unsigned long long* out25) {
  if (!out25) return fail(PDM_ERR_ARG, "pdm_gemm_seg_stats: null output");
  if (pdm::gemm_seg_stats(out25)) return fail(PDM_ERR_HIP, "pdm_gemm_seg_stats: device copy failed");
  return PDM_OK;
}
int pdm_gemm_sk_stats(unsigned long long* out3) {
  if (!out3) return fail(PDM_ERR_ARG, "pdm_gemm_sk_stats: null output");
  if (pdm::gemm_sk_stats(out3)) return fail(PDM_ERR_HIP, "pdm_gemm_sk_stats: device copy failed");
  return PDM_OK;
}

int pdm_set_gemm_tuning(int raster, int dbg_tile0) {
  if (raster < 0 || raster > 64) return fail(PDM_ERR_ARG, "pdm_set_gemm_tuning: raster must be in [0, 64]");
  pdm::gemm_set_tuning(raster, dbg_tile0);
  return PDM_OK;
}

int pdm_set_attention_algo(int algo) {
  if (algo < 0 || algo > 16)
    return fail(PDM_ERR_ARG, "pdm_set_attention_algo: algo must be 0 (auto) or 1..16 (5, 6, 8, 9, 12, 13, 15, 16: timing "
                             "experiments)");
  pdm::attention_set_algo(algo);
  return PDM_OK;
}

int pdm_device_arch(char* buf, int len) {
  int dev = 0;
  PDM_HIP(hipGetDevice(&dev));
  hipDeviceProp_t prop;
  PDM_HIP(hipGetDeviceProperties(&prop, dev));
  snprintf(buf, len, "%s", prop.gcnArchName);
  return PDM_OK;
}

int pdm_uvit_create(const pdm_uvit_cfg* cfg, pdm_uvit** out) {
  if (!cfg || !out) return fail(PDM_ERR_ARG, "pdm_uvit_create: null argument");
  const pdm_uvit_cfg& c = *cfg;
  if (c.embed_dim <= 0 || c.num_heads <= 0 || c.embed_dim % c.num_heads) return fail(PDM_ERR_ARG, "embed_dim must be divisible by num_heads");
  if (c.patch_size <= 0 || c.img_size % c.patch_size) return fail(PDM_ERR_ARG, "img_size must be divisible by patch_size");
  if (c.mlp_time_embed) return fail(PDM_ERR_ARG, "mlp_time_embed=True is not supported by the HIP path");
  if (c.embed_dim % 64) return fail(PDM_ERR_ARG, "embed_dim must be a multiple of 64");
  if (c.mlp_hidden % 64) return fail(PDM_ERR_ARG, "mlp hidden size must be a multiple of 64");
  if (c.t2i && c.enable_panoptic && !c.separate)
    return fail(PDM_ERR_ARG, "uvit_t2i with enable_panoptic and separate=False is not supported by the HIP path");
  if (c.fp8 && c.t2i) return fail(PDM_ERR_ARG, "fp8: only the class-conditional / unconditional U-ViT has an MXFP8 path");
  if (c.fp8 && (c.embed_dim % 128 || c.mlp_hidden % 128))
    return fail(PDM_ERR_ARG, "fp8: embed_dim and the mlp hidden size must be multiples of 128 (MXFP8 K-tiles)");
  if (c.fp8 && c.fp8_linears != 0 && c.fp8_linears != 0xF && c.fp8_linears != 0xB)
    return fail(PDM_ERR_ARG, "fp8_linears: supported sets are all four block Linears (0 / 0xF) and 0xB (mlp.fc1 bf16)");
  if (c.embed_dim > 2048 && c.fp8) return fail(PDM_ERR_ARG, "fp8: embed_dim must be <= 2048 (centred LayerNorm groups)");
  pdm_uvit* h = new pdm_uvit();
  h->cfg = c;
  h->D = c.embed_dim;
  h->H = c.num_heads;
  h->Dh = c.embed_dim / c.num_heads;
  h->Hid = c.mlp_hidden;
  h->C = c.in_chans;
  h->p = c.patch_size;
  h->n_patch = (c.img_size / c.patch_size) * (c.img_size / c.patch_size);
  h->depth = c.depth;
  h->nhalf = c.depth / 2;
  h->P = c.patch_size * c.patch_size * c.in_chans;
  h->P_pad = (h->P + 15) / 16 * 16;
  h->K = c.num_panoptic_class;
  h->PK = c.patch_size * c.patch_size * c.num_panoptic_class;
  h->PK_pad = (h->PK + 15) / 16 * 16;
  if (h->P_pad > 64 || (c.t2i && c.enable_panoptic && h->PK_pad > 64)) {
    delete h;
    return fail(PDM_ERR_ARG, "patch_size^2 * channels must be <= 64");
  }
  if (!c.t2i) {
    h->extras = c.num_classes > 0 ? 2 : 1;
  } else {
    h->extras = 1 + c.num_clip_token;
    if (c.clip_dim % 64) {
      delete h;
      return fail(PDM_ERR_ARG, "clip_dim must be a multiple of 64");
    }
  }
  h->Lx = h->extras + h->n_patch;
  h->Lm = h->Lx + h->n_patch;
  const int D = h->D;
  const int pk = c.in_chans * c.patch_size * c.patch_size;
  h->add("pos_embed", PDM_F32, (long long)h->Lx * D);
  h->add("patch_embed.proj.weight", PDM_F32, (long long)D * pk);
  h->add("patch_embed.proj.bias", PDM_F32, D);
  if (!c.t2i && c.num_classes > 0) h->add("label_emb.weight", PDM_F32, (long long)c.num_classes * D);
  if (c.t2i) {
    h->add("context_embed.weight", PDM_BF16, (long long)D * c.clip_dim);
    h->add("context_embed.bias", PDM_F32, D);
  }
  for (int i = 0; i < h->nhalf; ++i) h->add_block("in_blocks." + std::to_string(i), false);
  h->add_block("mid_block", false);
  for (int i = 0; i < h->nhalf; ++i) h->add_block("out_blocks." + std::to_string(i), c.skip != 0);
  h->add("norm.weight", PDM_F32, D);
  h->add("norm.bias", PDM_F32, D);
  h->add("decoder_pred.weight", PDM_BF16, (long long)h->P_pad * D);
  h->add("decoder_pred.bias", PDM_F32, h->P);
  if (c.t2i && c.enable_panoptic && c.separate) {
    h->add("pos_embed_mask", PDM_F32, (long long)h->n_patch * D);
    h->add("mask_embed.proj.weight", PDM_F32, (long long)D * h->PK);
    h->add("mask_embed.proj.bias", PDM_F32, D);
    h->add("decoder_pred_mask.weight", PDM_BF16, (long long)h->PK_pad * D);
    h->add("decoder_pred_mask.bias", PDM_F32, h->PK);
    for (int i = 0; i < h->nhalf; ++i) h->add_block("in_blocks_mask." + std::to_string(i), false);
    h->add_block("mid_block_mask", false);
    for (int i = 0; i < h->nhalf; ++i) h->add_block("out_blocks_mask." + std::to_string(i), c.skip != 0);
    for (int i = 0; i <= c.depth; ++i) {
      const std::string zc = "zero_convs." + std::to_string(2 * i + 1) + ".conv";
      h->add(zc + ".weight", PDM_BF16, (long long)D * D);
      h->add(zc + ".bias", PDM_F32, D);
    }
  }
  *out = h;
  return PDM_OK;
}

int pdm_uvit_destroy(pdm_uvit* h) {
  if (h)
    for (auto e : h->prof_ev) (void)hipEventDestroy(e);
  delete h;
  return PDM_OK;
}

int pdm_uvit_profile(pdm_uvit* h, int max_launches) {
  if (!h || max_launches < 0) return fail(PDM_ERR_ARG, "pdm_uvit_profile: bad argument");
  if (max_launches == 0) {
    h->prof_on = false;
    return PDM_OK;
  }
  while ((int)h->prof_ev.size() < 2 * max_launches) {
    hipEvent_t e;
    PDM_HIP(hipEventCreate(&e));
    h->prof_ev.push_back(e);
  }
  h->prof_flops.assign(max_launches, 0.0);
  h->prof_n = 0;
  h->prof_on = true;
  return PDM_OK;
}

int pdm_uvit_profile_read(pdm_uvit* h, float* ms, double* flops, int cap, int* n) {
  if (!h || !n) return fail(PDM_ERR_ARG, "pdm_uvit_profile_read: bad argument");
  *n = h->prof_n;
  for (int i = 0; i < h->prof_n && i < cap; ++i) {
    PDM_HIP(hipEventSynchronize(h->prof_ev[2 * i + 1]));
    PDM_HIP(hipEventElapsedTime(&ms[i], h->prof_ev[2 * i], h->prof_ev[2 * i + 1]));
    flops[i] = h->prof_flops[i];
  }
  return PDM_OK;
}

int pdm_uvit_param_count(const pdm_uvit* h) { return h ? (int)h->order.size() : 0; }

int pdm_uvit_param_info(const pdm_uvit* h, int i, char* name, int len, int* dtype, long long* numel) {
  if (!h || i < 0 || i >= (int)h->order.size()) return fail(PDM_ERR_ARG, "pdm_uvit_param_info: index out of range");
  const std::string& n = h->order[i];
  snprintf(name, len, "%s", n.c_str());
  const ParamSpec& s = h->params.at(n);
  *dtype = s.dtype;
  *numel = s.numel;
  return PDM_OK;
}

int pdm_uvit_set_param(pdm_uvit* h, const char* name, const void* dev_ptr, int dtype, long long numel) {
  if (!h || !name) return fail(PDM_ERR_ARG, "pdm_uvit_set_param: null argument");
  auto it = h->params.find(name);
  if (it == h->params.end()) return fail(PDM_ERR_ARG, std::string("pdm_uvit_set_param: unexpected key ") + name);
  if (it->second.dtype != dtype || it->second.numel != numel)
    return fail(PDM_ERR_ARG, std::string("pdm_uvit_set_param: dtype/size mismatch for ") + name);
  if (((uintptr_t)dev_ptr) & 15) return fail(PDM_ERR_ARG, std::string("pdm_uvit_set_param: 16-byte alignment required for ") + name);
  it->second.ptr = dev_ptr;
  return PDM_OK;
}

int pdm_uvit_validate(pdm_uvit* h) {
  if (!h) return fail(PDM_ERR_ARG, "null handle");
  return check_ready(h);
}

int pdm_uvit_workspace_size(const pdm_uvit* h, int rows, size_t* bytes) {
  if (!h || rows <= 0 || !bytes) return fail(PDM_ERR_ARG, "pdm_uvit_workspace_size: bad argument");
  *bytes = layout(h, rows, nullptr).bytes;
  return PDM_OK;
}

int pdm_uvit_forward(pdm_uvit* h, const float* x, const float* t, const int64_t* y, float* eps_pre, int rows,
                     void* workspace, size_t workspace_bytes, void* stream) {
  if (!h || !x || !t || !eps_pre || rows <= 0) return fail(PDM_ERR_ARG, "pdm_uvit_forward: bad argument");
  if (h->cfg.t2i) return fail(PDM_ERR_ARG, "pdm_uvit_forward: t2i network, use pdm_uvit_t2i_forward");
  if (h->cfg.num_classes > 0 && !y) return fail(PDM_ERR_ARG, "pdm_uvit_forward: labels required (num_classes > 0)");
  if (h->cfg.num_classes <= 0 && y) return fail(PDM_ERR_ARG, "pdm_uvit_forward: labels given to an unconditional net");
  PDM_TRY(check_ready(h));
  Workspace w = layout(h, rows, (char*)workspace);
  if (w.bytes > workspace_bytes) return fail(PDM_ERR_ARG, "pdm_uvit_forward: workspace too small");
  h->prof_n = 0;
  Ctx c{h, (hipStream_t)stream};
  int skn = 0;
  PDM_TRY(sk_begin(c, &skn));
  const int D = h->D, L = h->Lx;
  {
    pdm::AssembleArgs a{};
    a.img = x; a.C = h->C; a.Himg = h->cfg.img_size; a.Wimg = h->cfg.img_size; a.p = h->p;
    a.patch_w = h->f("patch_embed.proj.weight"); a.patch_b = h->f("patch_embed.proj.bias");
    a.t = t; a.y = y;
    a.label_emb = h->cfg.num_classes > 0 ? h->f("label_emb.weight") : nullptr;
    a.pos = h->f("pos_embed");
    a.out = w.X; a.ld_out = D;
    a.B = rows; a.D = D; a.L_total = L;
    a.row0_patch = h->extras;
    a.time_row = h->extras - 1;
    a.label_row = h->cfg.num_classes > 0 ? 0 : -1;   // token order [label, time, patches] (libs/uvit.py:205-211)
    a.ctx_row = -1;
    PDM_CHECK(pdm::assemble_check(a));
    PDM_HIP(pdm::assemble_launch(a, c.s));
  }
  if (h->res16()) {
    PDM_TRY(h->cfg.fp8 ? run_stack8_16(c, w, rows, L) : run_stack16(c, w, rows, L));
    PDM_TRY(final_norm(c, w, rows, nullptr, L, nullptr, 0, 0, w.XB));
  } else {
    PDM_TRY(h->cfg.fp8 ? run_stack8(c, w, rows, L) : run_stack(c, w, rows, L));
    PDM_TRY(final_norm(c, w, rows, w.X, L));
  }
  PDM_TRY(run_head(c, w.HEADIN, h->n_patch, 0, rows, "decoder_pred", h->C, h->P, h->P_pad, eps_pre));
  return PDM_OK;
}

int pdm_uvit_t2i_forward(pdm_uvit* h, const float* x, const float* t, const float* context, const float* mask_token,
                         int use_ground_truth, float* eps_pre, float* mask_pre, int rows, void* workspace,
                         size_t workspace_bytes, void* stream) {
  if (!h || !x || !t || !context || !eps_pre || rows <= 0) return fail(PDM_ERR_ARG, "pdm_uvit_t2i_forward: bad argument");
  if (!h->cfg.t2i) return fail(PDM_ERR_ARG, "pdm_uvit_t2i_forward: not a t2i network");
  const bool two = mask_token && h->cfg.separate && h->cfg.enable_panoptic;
  if (mask_token && !two) return fail(PDM_ERR_ARG, "pdm_uvit_t2i_forward: mask tokens need enable_panoptic and separate");
  if (two && !use_ground_truth && !mask_pre) return fail(PDM_ERR_ARG, "pdm_uvit_t2i_forward: mask_pre output missing");
  PDM_TRY(check_ready(h));
  Workspace w = layout(h, rows, (char*)workspace);
  if (w.bytes > workspace_bytes) return fail(PDM_ERR_ARG, "pdm_uvit_t2i_forward: workspace too small");
  h->prof_n = 0;
  Ctx c{h, (hipStream_t)stream};
  int skn = 0;
  PDM_TRY(sk_begin(c, &skn));
  const int D = h->D, Lx = h->Lx, Lm = h->Lm, nctx = h->cfg.num_clip_token;
  // context_embed (libs/uvit_t2i.py:387): bf16 cast + GEMM (+bias) -> fp32 context tokens
  PDM_HIP(pdm::cast_bf16_launch(context, w.CTXB, (long long)rows * nctx * h->cfg.clip_dim, c.s));
  PDM_TRY(gemm(c, w.CTXB, h->cfg.clip_dim, h->w("context_embed.weight"), h->f("context_embed.bias"), rows * nctx, D,
               h->cfg.clip_dim, pdm::EPI_F32, nullptr, 0, w.CTXF, D, 0));
  {  // image stream tokens [time, context x nctx, patches] + pos_embed (401-405 / 408-409)
    pdm::AssembleArgs a{};
    a.img = x; a.C = h->C; a.Himg = h->cfg.img_size; a.Wimg = h->cfg.img_size; a.p = h->p;
    a.patch_w = h->f("patch_embed.proj.weight"); a.patch_b = h->f("patch_embed.proj.bias");
    a.t = t; a.ctx_tokens = w.CTXF; a.n_ctx = nctx;
    a.pos = h->f("pos_embed");
    a.out = w.X; a.ld_out = D; a.B = rows; a.D = D; a.L_total = Lx;
    a.row0_patch = h->extras; a.time_row = 0; a.label_row = -1; a.ctx_row = 1;
    PDM_CHECK(pdm::assemble_check(a));
    PDM_HIP(pdm::assemble_launch(a, c.s));
  }
  const size_t MDx = (size_t)rows * Lx * D;
  if (!two) {  // plain text-conditioned U-ViT (mask_token None: 407-410, 516-517)
    if (h->res16()) {
      PDM_TRY(run_stack16(c, w, rows, Lx));
      PDM_TRY(final_norm(c, w, rows, nullptr, Lx, nullptr, 0, 0, w.XB));
    } else {
      PDM_TRY(run_stack(c, w, rows, Lx));
      PDM_TRY(final_norm(c, w, rows, w.X, Lx));
    }
    PDM_TRY(run_head(c, w.HEADIN, h->n_patch, 0, rows, "decoder_pred", h->C, h->P, h->P_pad, eps_pre));
    return PDM_OK;
  }
  {  // mask tokens m = mask_embed(mask_token) + pos_embed_mask (390, 406), stored at MX[:, Lx:Lm]
    pdm::AssembleArgs a{};
    a.img = mask_token; a.C = h->K; a.Himg = h->cfg.img_size; a.Wimg = h->cfg.img_size; a.p = h->p;
    a.patch_w = h->f("mask_embed.proj.weight"); a.patch_b = h->f("mask_embed.proj.bias");
    a.pos = h->f("pos_embed_mask");
    a.out = w.MX + (size_t)Lx * D; a.ld_out = D; a.B = rows; a.D = D; a.L_total = Lm;
    a.row0_patch = 0; a.time_row = -1; a.label_row = -1; a.ctx_row = -1;
    PDM_CHECK(pdm::assemble_check(a));
    PDM_HIP(pdm::assemble_launch(a, c.s));
  }
  const size_t MDm = (size_t)rows * Lm * D;
  if (h->res16()) return t2i_two_stream16(c, w, rows, use_ground_truth, eps_pre, mask_pre);
  // mx = cat(x, m): refresh the image half of the mask stream before every mask block (426, 443, 459), then
  // the bf16 copy + LayerNorm partials of the whole mask stream (its blocks' qkv / skip_linear operand)
  auto refresh = [&]() -> int {
    PDM_HIP(pdm::rowcopy_launch(w.MX, D, w.X, D, rows * Lx, D, Lx, Lm, Lx, c.s));
    return row_stats(c, w.MX, rows * Lm, w.MXIN, w.STM);
  };
  // x += zeroconv_{2l+1}(mx[:, :Lx]) (435-436, 452-453, 470-472) from the bf16 copy of the mask block output;
  // the epilogue also leaves bf16 of the new x (the skip / next block's operand) in xb and its partials in ST
  auto inject = [&](int layer, const bf16* mxb, bf16* xb) -> int {
    const std::string zc = "zero_convs." + std::to_string(2 * layer + 1) + ".conv";
    LnIO io;
    io.st_out = w.ST;
    return gemm(c, mxb, D, h->w(zc + ".weight"), h->f(zc + ".bias"), rows * Lx, D, D, pdm::EPI_F32, xb, D, w.X, D, 1,
                nullptr, 0, 0, Lx, Lm, io);
  };
  PDM_TRY(row_stats(c, w.X, rows * Lx, w.XB, w.ST));
  const bf16* xb = w.XB;
  int layer = 0;
  for (int i = 0; i < h->nhalf; ++i, ++layer) {
    PDM_TRY(refresh());
    PDM_TRY(run_block(c, "in_blocks." + std::to_string(i), w.X, rows, Lx, xb, w.ST, nullptr, nullptr, nullptr, w));
    PDM_TRY(run_block(c, "in_blocks_mask." + std::to_string(i), w.MX, rows, Lm, w.MXIN, w.STM, nullptr,
                      w.SKM + i * MDm, nullptr, w));
    PDM_TRY(inject(layer, w.SKM + i * MDm, w.SK + i * MDx));
    xb = w.SK + i * MDx;
  }
  PDM_TRY(refresh());
  PDM_TRY(run_block(c, "mid_block", w.X, rows, Lx, xb, w.ST, nullptr, nullptr, nullptr, w));
  PDM_TRY(run_block(c, "mid_block_mask", w.MX, rows, Lm, w.MXIN, w.STM, nullptr, w.MXB, nullptr, w));
  PDM_TRY(inject(layer, w.MXB, w.XB));
  ++layer;
  for (int i = 0; i < h->nhalf; ++i, ++layer) {
    PDM_TRY(refresh());
    const bf16* sk = h->cfg.skip ? w.SK + (h->nhalf - 1 - i) * MDx : nullptr;
    PDM_TRY(run_block(c, "out_blocks." + std::to_string(i), w.X, rows, Lx, w.XB, w.ST, sk, nullptr, nullptr, w));
    const bf16* skm = h->cfg.skip ? w.SKM + (h->nhalf - 1 - i) * MDm : nullptr;
    PDM_TRY(run_block(c, "out_blocks_mask." + std::to_string(i), w.MX, rows, Lm, w.MXIN, w.STM, skm, w.MXB, nullptr, w));
    PDM_TRY(inject(layer, w.MXB, w.XB));
  }
  // heads (477-519): noise from norm(x) patch tokens; mask head on the un-normalised m (= MX[:, Lx:])
  if (use_ground_truth) {
    PDM_TRY(final_norm(c, w, rows, w.X, Lx, w.MX, Lm, Lx));
  } else {
    PDM_TRY(final_norm(c, w, rows, w.X, Lx));
    const bf16* mb = h->nhalf > 0 ? w.MXB : w.MXB;  // bf16 copy of the last mask block output
    PDM_TRY(run_head(c, mb, Lm, Lx, rows, "decoder_pred_mask", h->K, h->PK, h->PK_pad, mask_pre));
  }
  PDM_TRY(run_head(c, w.HEADIN, h->n_patch, 0, rows, "decoder_pred", h->C, h->P, h->P_pad, eps_pre));
  return PDM_OK;
}

int pdm_stage_epilogue(const pdm_stage_epilogue_args* a, void* stream) {
  if (!a) return fail(PDM_ERR_ARG, "pdm_stage_epilogue: null args");
  pdm::EpilogueArgs e{};
  e.pre = a->pre; e.w = a->conv_w; e.bias = a->conv_b;
  e.B = a->B; e.C = a->C; e.Himg = a->H; e.Wimg = a->W;
  e.has_uncond = a->has_uncond; e.cfg_scale = a->cfg_scale;
  e.act_tanh = a->act_tanh;
  e.xin = a->xin; e.ax = a->ax; e.ae = a->ae;
  e.m_out = a->m_out;
  e.n_terms = a->n_terms;
  for (int i = 0; i < 6; ++i) { e.T[i] = a->T[i]; e.c[i] = a->c[i]; }
  e.cm = a->cm;
  e.x_out = a->x_out;
  e.x_out2 = a->x_out2;
  e.x_out3 = a->x_out3;
  PDM_CHECK(pdm::epilogue_check(e));
  PDM_HIP(pdm::epilogue_launch(e, (hipStream_t)stream));
  return PDM_OK;
}

int pdm_lincomb(float* out, int n_terms, const float* const* T, const float* c, long long n, void* stream) {
  if (!out || n_terms < 0 || n_terms > 8 || (n_terms && (!T || !c))) return fail(PDM_ERR_ARG, "pdm_lincomb: bad argument");
  PDM_HIP(pdm::lincomb_launch(out, n_terms, T, c, n, (hipStream_t)stream));
  return PDM_OK;
}

int pdm_gemm_bf16(const void* A1, int lda1, const void* A2, int lda2, int K1, const void* W, const float* bias, int M,
                  int N, int K, int epi, void* out_bf16, int ldo, float* out_f32, int ldr, int accumulate,
                  void* stream) {
  pdm::GemmArgs a{};
  a.A1 = (const bf16*)A1; a.lda1 = lda1;
  a.A2 = (const bf16*)A2; a.lda2 = lda2;
  a.K1 = A2 ? K1 : K;
  a.W = (const bf16*)W; a.bias = bias;
  a.M = M; a.N = N; a.K = K;
  a.out_bf16 = (bf16*)out_bf16; a.ldo = ldo;
  a.out_f32 = out_f32; a.ldr = ldr;
  a.accumulate = accumulate;
  PDM_CHECK(pdm::gemm_check(a, epi));
  PDM_HIP(pdm::gemm_launch(a, epi, (hipStream_t)stream));
  return PDM_OK;
}

int pdm_gemm_bf16_ln(const void* A, int lda, const void* W, const float* bias, int M, int N, int K, int epi,
                     void* out_bf16, int ldo, float* out_f32, int ldr, int accumulate, float* stats_out,
                     const float* ln_stats, const float* ln_colsum, float ln_eps, void* stream) {
  pdm::GemmArgs a{};
  a.A1 = (const bf16*)A; a.lda1 = lda; a.K1 = K;
  a.W = (const bf16*)W; a.bias = bias;
  a.M = M; a.N = N; a.K = K;
  a.out_bf16 = (bf16*)out_bf16; a.ldo = ldo;
  a.out_f32 = out_f32; a.ldr = ldr;
  a.accumulate = accumulate;
  a.stats_out = stats_out; a.stats_ld = (N + 255) / 256;
  a.ln_stats = ln_stats; a.ln_ld = (K + 255) / 256; a.ln_D = K; a.ln_eps = ln_eps; a.ln_colsum = ln_colsum;
  PDM_CHECK(pdm::gemm_check(a, epi));
  PDM_HIP(pdm::gemm_launch(a, epi, (hipStream_t)stream));
  return PDM_OK;
}

int pdm_rowstats(const float* x, int ldx, int rows, int D, void* xb, float* stats, void* stream) {
  if (!x || !stats || rows <= 0 || D <= 0 || D % 4 || D > 2048) return fail(PDM_ERR_ARG, "pdm_rowstats: bad argument");
  PDM_HIP(pdm::rowstats_launch(x, ldx, rows, D, (bf16*)xb, D, stats, (D + 255) / 256, (hipStream_t)stream));
  return PDM_OK;
}

// stream-K state for standalone pdm_gemm calls (pdm_set_gemm_sk mode bit 2; tests and tools): the calling stream's
// ring (sk_state), its next flag block per call, the ring zeroed on the stream whenever it wraps
static int sk_standalone(pdm::GemmArgs& a, hipStream_t s) {
  SkState* st = nullptr;
  PDM_TRY(sk_state(s, &st));
  if (!st) return PDM_OK;   // capturing without a state: whole tiles
  if (st->next == SK_RING) {
    PDM_HIP(hipMemsetAsync(st->flags, 0, (size_t)SK_RING * pdm::SK_FLAG_WORDS * 4, s));
    st->next = 0;
  }
  a.sk_flags = st->flags + (size_t)st->next++ * pdm::SK_FLAG_WORDS;
  a.sk_slab = st->slab;
  return PDM_OK;
}

static pdm::GemmArgs to_gemm_args(const pdm_gemm_args* g) {
  pdm::GemmArgs a{};
  a.A1 = (const bf16*)g->A1; a.lda1 = g->lda1;
  a.A2 = (const bf16*)g->A2; a.lda2 = g->lda2;
  a.K1 = g->A2 ? g->K1 : g->K;
  a.W = (const bf16*)g->W; a.ldw = g->ldw; a.bias = g->bias;
  a.M = g->M; a.N = g->N; a.K = g->K;
  a.out_bf16 = (bf16*)g->out_bf16; a.ldo = g->ldo;
  a.out_f32 = g->out_f32; a.ldr = g->ldr; a.accumulate = g->accumulate;
  a.stats_out = g->stats_out; a.stats_ld = (g->N + 255) / 256;
  a.ln_stats = g->ln_stats; a.ln_ld = (g->K + 255) / 256; a.ln_D = g->K; a.ln_eps = g->ln_eps; a.ln_colsum = g->ln_colsum;
  a.fp8 = g->fp8;
  a.a_scale = g->a_scale; a.a_scale_ld = g->a_scale_ld;
  a.w_scale = g->w_scale; a.w_scale_ld = g->w_scale_ld;
  a.out_fp8 = (unsigned char*)g->out_fp8; a.ldo8 = g->ldo8;
  a.out_scale = g->out_scale; a.out_scale_ld = g->out_scale_ld;
  a.mx_center = g->mx_center; a.ln_gcol = (const bf16*)g->ln_gcol;
  a.res_in = (const bf16*)g->res_in; a.ldri = g->ldri;
  a.res_f32 = g->res_f32; a.ldrf = g->ldrf;
  a.a_rows_per_group = g->a_rows_per_group; a.a_group_stride = g->a_group_stride;
  a.out2 = (bf16*)g->out2; a.out2_rpg = g->out2_rows_per_group; a.out2_gs = g->out2_group_stride;
  a.stats_out2 = g->stats_out2;
  return a;
}

int pdm_gemm(const pdm_gemm_args* g, int epi, void* stream) {
  if (!g) return fail(PDM_ERR_ARG, "pdm_gemm: null args");
  pdm::GemmArgs a = to_gemm_args(g);
  PDM_CHECK(pdm::gemm_check(a, epi));
  if (g_sk_standalone) PDM_TRY(sk_standalone(a, (hipStream_t)stream));
  PDM_HIP(pdm::gemm_launch(a, epi, (hipStream_t)stream));
  return PDM_OK;
}

int pdm_gemm_pair(const pdm_gemm_args* ga, const pdm_gemm_args* gb, int epi, void* stream) {
  if (!ga || !gb) return fail(PDM_ERR_ARG, "pdm_gemm_pair: null args");
  const pdm::GemmArgs a = to_gemm_args(ga), b = to_gemm_args(gb);
  PDM_CHECK(pdm::gemm_check(a, epi));
  PDM_CHECK(pdm::gemm_check(b, epi));
  PDM_HIP(pdm::gemm_launch_pair(a, b, epi, (hipStream_t)stream));
  return PDM_OK;
}

int pdm_gemm_args_size(void) { return (int)sizeof(pdm_gemm_args); }

int pdm_gemm_conv3x3_bf16(const void* in, int B, int H, int W, int Cin, int up, const void* Wt, const float* bias,
                          int N, int epi, void* out_bf16, float* out_f32, int accumulate, void* stream) {
  static bf16* zero = nullptr;   // zero page for the tile policies that address padded taps explicitly
  if (!zero) {
    PDM_HIP(hipMalloc(&zero, 4096));
    PDM_HIP(hipMemset(zero, 0, 4096));
  }
  pdm::GemmArgs a{};
  a.A1 = (const bf16*)in; a.lda1 = Cin; a.K1 = 9 * Cin;
  a.W = (const bf16*)Wt; a.bias = bias;
  a.M = B * H * W; a.N = N; a.K = 9 * Cin;
  a.out_bf16 = (bf16*)out_bf16; a.ldo = N;
  a.out_f32 = out_f32; a.ldr = N;
  a.accumulate = accumulate;
  a.conv = 1; a.convH = H; a.convW = W; a.convC = Cin; a.conv_up = up; a.zero = zero;
  PDM_CHECK(pdm::gemm_check(a, epi));
  PDM_HIP(pdm::gemm_launch(a, epi, (hipStream_t)stream));
  return PDM_OK;
}

int pdm_gemm_batched_bf16(const void* A, int lda, long long sA, const void* W, int ldw, long long sW,
                          const float* bias, int M, int N, int K, int batch, int epi, void* out_bf16, int ldo,
                          long long sO, float* out_f32, int ldr, long long sR, int accumulate, void* stream) {
  pdm::GemmArgs a{};
  a.A1 = (const bf16*)A; a.lda1 = lda; a.K1 = K;
  a.W = (const bf16*)W; a.ldw = ldw; a.bias = bias;
  a.M = M; a.N = N; a.K = K;
  a.out_bf16 = (bf16*)out_bf16; a.ldo = ldo;
  a.out_f32 = out_f32; a.ldr = ldr;
  a.accumulate = accumulate;
  a.batch = batch; a.sA = sA; a.sW = sW; a.sO = sO; a.sR = sR;
  if (batch < 1) return fail(PDM_ERR_ARG, "pdm_gemm_batched_bf16: batch must be >= 1");
  PDM_CHECK(pdm::gemm_check(a, epi));
  PDM_HIP(pdm::gemm_launch(a, epi, (hipStream_t)stream));
  return PDM_OK;
}

int pdm_layernorm(const float* x, int ldx, const float* gamma, const float* beta, void* y, int ldy, int rows, int D,
                  float eps, void* stream) {
  pdm::LayerNormArgs a{};
  a.x = x; a.ldx = ldx; a.gamma = gamma; a.beta = beta; a.y = (bf16*)y; a.ldy = ldy;
  a.rows = rows; a.D = D; a.rows_per_group = 1; a.group_stride = 1; a.row_offset = 0; a.eps = eps;
  PDM_CHECK(pdm::layernorm_check(a));
  PDM_HIP(pdm::layernorm_launch(a, (hipStream_t)stream));
  return PDM_OK;
}

int pdm_attention(const void* qkv, int ldq, void* out, int ldo, int B, int L, int H, int Dh, float scale,
                  void* stream) {
  pdm::AttentionArgs a{};
  a.qkv = (const bf16*)qkv; a.ldq = ldq; a.out = (bf16*)out; a.ldo = ldo;
  a.B = B; a.L = L; a.H = H; a.Dh = Dh; a.scale = scale;
  PDM_CHECK(pdm::attention_check(a));
  PDM_HIP(pdm::attention_launch(a, (hipStream_t)stream));
  return PDM_OK;
}

int pdm_attention_log2(const void* qkv, int ldq, void* out, int ldo, int B, int L, int H, int Dh, void* stream) {
  pdm::AttentionArgs a{};
  a.qkv = (const bf16*)qkv; a.ldq = ldq; a.out = (bf16*)out; a.ldo = ldo;
  a.B = B; a.L = L; a.H = H; a.Dh = Dh; a.scale = 1.0f / sqrtf((float)Dh); a.q_log2 = 1;
  PDM_CHECK(pdm::attention_check(a));
  PDM_HIP(pdm::attention_launch(a, (hipStream_t)stream));
  return PDM_OK;
}

int pdm_mx_quantize(const void* x, int dtype, int ldx, int rows, int K, void* q, int ldq, unsigned* s, int s_ld,
                    void* stream) {
  if (dtype != PDM_F32 && dtype != PDM_BF16) return fail(PDM_ERR_ARG, "pdm_mx_quantize: dtype must be PDM_F32 or PDM_BF16");
  const hipError_t e = pdm::mxq_launch(x, dtype == PDM_F32 ? 0 : 1, ldx, rows, K, (unsigned char*)q, ldq, s, s_ld,
                                       (hipStream_t)stream);
  if (e == hipErrorInvalidValue)
    return fail(PDM_ERR_ARG, "pdm_mx_quantize: K % 32, ldx / ldq >= K, s_ld >= rows and 16-byte aligned rows required");
  PDM_HIP(e);
  return PDM_OK;
}

int pdm_f32_to_bf16(const float* x, void* y, long long n, void* stream) {
  if (n == 0) return PDM_OK;   // empty tensors may carry null data pointers
  if (!x || !y || n < 0) return fail(PDM_ERR_ARG, "pdm_f32_to_bf16: bad argument");
  PDM_HIP(pdm::cast_bf16_launch(x, (bf16*)y, n, (hipStream_t)stream));
  return PDM_OK;
}

}  // extern "C"

// CLIP text encoder (the t2i conditioning producer) on gfx950.
//
// Reference: libs/clip.py:13-38 FrozenCLIPEmbedder = transformers CLIPTextModel (openai/clip-vit-large-patch14:
// vocab 49408, width 768, 12 layers, 12 heads, MLP 3072, quick GELU, 77 positions) -> last_hidden_state,
// the [B, 77, 768] context of libs/uvit_t2i.py:378 (sample_t2i_discrete.py:49-53).  Per layer (transformers
// CLIPEncoderLayer): x += out_proj(causal_attn(q/k/v_proj(LN1 x))); x += fc2(quick_gelu(fc1(LN2 x))); then
// final_layer_norm.  Tokenisation is host string work and stays outside (token ids are the input).
//
// HBM layout per forward of B sequences of L tokens (M = B*L rows, width D):
//   X fp32 [M, D] residual stream; XB / XT bf16 [M, D] GEMM operands; ST / STT the fused-LayerNorm row
//   partials; QKV bf16 [M, 3D] (q | k | v, heads contiguous inside each); ATT bf16 [M, D]; MLP bf16 [M, F].
// The GEMMs are the U-ViT block GEMMs (gemm.hip): LN1 / LN2 folded into qkv / fc1 (gamma-scaled weights,
// column sums, folded bias; row statistics emitted by the previous residual epilogue), quick GELU in fc1's
// epilogue, residual adds in out_proj / fc2's fp32 epilogues.  The causal attention over L <= 128 keys
// and the embedding / final LayerNorm are small kernels of their own (below): together < 2 % of the FLOPs.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <string>
#include <vector>

#include "../../include/pdm.h"
#include "pdm_common.h"
#include "pdm_kernels.h"

namespace pdm {
namespace {

// token + position embedding (transformers CLIPTextEmbeddings): X[b*L + l] = tok[ids[b, l]] + pos[l].
// One wave per row, float4 lanes.  Ids outside [0, V) are rejected on the host; clamped here for safety.
__global__ __launch_bounds__(256) void clip_embed_kernel(const long long* ids, const float* tok, const float* pos,
                                                         float* X, int M, int L, int D, int V) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  long long id = ids[row];
  id = id < 0 ? 0 : (id >= V ? V - 1 : id);
  const f32x4* t = reinterpret_cast<const f32x4*>(tok + id * D);
  const f32x4* p = reinterpret_cast<const f32x4*>(pos + (long long)(row % L) * D);
  f32x4* x = reinterpret_cast<f32x4*>(X + (long long)row * D);
  for (int c = lane; c < D / 4; c += 64) x[c] = t[c] + p[c];
}

// Causal self-attention of one (sequence, head) per workgroup, L <= 128 keys, Dh <= 64 (transformers
// CLIPAttention with the causal mask: softmax(q k^T * Dh^-1/2 + mask) v).  K and V of the head are staged in
// LDS as fp32; thread q owns query row q: pass 1 takes the row max over keys 0..q, pass 2 accumulates
// exp(s - max) and the weighted V rows; every LDS read is a broadcast (all threads read the same key).
template <int DH>
__global__ __launch_bounds__(128) void clip_attention_kernel(const bf16* qkv, int ldq, bf16* out, int ldo, int L,
                                                             int D, float scale) {
  __shared__ float Ks[128][DH];
  __shared__ float Vs[128][DH];
  const int h = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const long long row0 = (long long)b * L;
  for (int i = t; i < L * DH; i += 128) {
    const int r = i / DH, d = i - r * DH;
    const bf16* src = qkv + (row0 + r) * ldq + h * DH + d;
    Ks[r][d] = (float)src[D];
    Vs[r][d] = (float)src[2 * D];
  }
  __syncthreads();
  if (t >= L) return;
  float q[DH];
  const bf16* qs = qkv + (row0 + t) * ldq + h * DH;
#pragma unroll
  for (int d = 0; d < DH; ++d) q[d] = (float)qs[d] * scale;
  float mx = -INFINITY;
  for (int j = 0; j <= t; ++j) {
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < DH; ++d) s = fmaf(q[d], Ks[j][d], s);
    mx = fmaxf(mx, s);
  }
  float acc[DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) acc[d] = 0.f;
  float l = 0.f;
  for (int j = 0; j <= t; ++j) {
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < DH; ++d) s = fmaf(q[d], Ks[j][d], s);
    const float pj = __expf(s - mx);
    l += pj;
#pragma unroll
    for (int d = 0; d < DH; ++d) acc[d] = fmaf(pj, Vs[j][d], acc[d]);
  }
  const float inv = 1.0f / l;
  bf16* o = out + (row0 + t) * ldo + h * DH;
#pragma unroll
  for (int d = 0; d < DH; d += 4)
    *reinterpret_cast<bf16x4*>(o + d) = to_bf16x4(acc[d] * inv, acc[d + 1] * inv, acc[d + 2] * inv, acc[d + 3] * inv);
}

// final_layer_norm: fp32 rows -> fp32 rows (two-pass mean / variance in registers), one wave per row
template <int PER>
__global__ __launch_bounds__(256) void clip_final_ln_kernel(const float* X, const float* g, const float* bta, float* Y,
                                                            int M, int D, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* x = X + (long long)row * D;
  float v[PER];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < D ? x[c] : 0.f;
    s += v[i];
  }
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    const float d = c < D ? v[i] - mean : 0.f;
    q += d * d;
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
  float* y = Y + (long long)row * D;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    if (c < D) y[c] = (v[i] - mean) * rstd * g[c] + bta[c];
  }
}

}  // namespace
}  // namespace pdm

using pdm::bf16;

namespace {

int cfail(int code, const std::string& m) { return pdm::set_error(code, m); }
#define C_HIP(call)                                                                                   \
  do {                                                                                                \
    hipError_t e_ = (call);                                                                           \
    if (e_ != hipSuccess) return cfail(PDM_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define C_CHECK(m)                              \
  do {                                          \
    const char* m_ = (m);                       \
    if (m_) return cfail(PDM_ERR_ARG, m_);      \
  } while (0)
#define C_TRY(x)        \
  do {                  \
    int r_ = (x);       \
    if (r_) return r_;  \
  } while (0)

struct CParam {
  int dtype;
  long long numel;
  const void* ptr = nullptr;
};

size_t calign(size_t x) { return (x + 255) / 256 * 256; }

}  // namespace

struct pdm_clip {
  pdm_clip_cfg cfg;
  int Dh, T;
  std::vector<std::string> order;
  std::map<std::string, CParam> params;
  void add(const std::string& n, int dt, long long ne) {
    order.push_back(n);
    params[n] = CParam{dt, ne, nullptr};
  }
  const float* f(const std::string& n) const { return static_cast<const float*>(params.at(n).ptr); }
  const bf16* w(const std::string& n) const { return static_cast<const bf16*>(params.at(n).ptr); }
};

namespace {

struct CWork {
  float *X, *ST, *STT;
  bf16 *XB, *XT, *QKV, *ATT, *MLP;
  size_t bytes;
};

CWork clayout(const pdm_clip* c, int B, char* base) {
  CWork w{};
  size_t off = 0;
  auto take = [&](size_t n) {
    char* p = base ? base + off : nullptr;
    off = calign(off + n);
    return p;
  };
  const size_t M = (size_t)B * c->cfg.max_position, D = c->cfg.width;
  w.X = (float*)take(M * D * 4);
  w.ST = (float*)take(M * c->T * 8);
  w.STT = (float*)take(M * c->T * 8);
  w.XB = (bf16*)take(M * D * 2);
  w.XT = (bf16*)take(M * D * 2);
  w.QKV = (bf16*)take(M * 3 * D * 2);
  w.ATT = (bf16*)take(M * D * 2);
  w.MLP = (bf16*)take(M * c->cfg.mlp_hidden * 2);
  w.bytes = off;
  return w;
}

// one block Linear on the shared GEMM (gemm.hip): LN-consumer (st_in + colsum) or residual producer (st_out)
int clip_gemm(hipStream_t s, const pdm_clip* c, const bf16* A, int lda, const bf16* W, const float* bias, int M, int N,
              int K, int epi, bf16* ob, float* of, int accumulate, const float* st_in, const float* colsum,
              float* st_out) {
  pdm::GemmArgs a{};
  a.A1 = A; a.lda1 = lda; a.K1 = K;
  a.W = W; a.bias = bias;
  a.M = M; a.N = N; a.K = K;
  a.out_bf16 = ob; a.ldo = ob ? N : 0;
  a.out_f32 = of; a.ldr = of ? N : 0; a.accumulate = accumulate;
  a.stats_out = st_out; a.stats_ld = c->T;
  a.ln_stats = st_in; a.ln_ld = c->T; a.ln_D = K; a.ln_eps = c->cfg.eps; a.ln_colsum = colsum;
  a.act = epi == pdm::EPI_GELU ? 1 : 0;   // CLIP hidden_act = quick_gelu
  C_CHECK(pdm::gemm_check(a, epi));
  C_HIP(pdm::gemm_launch(a, epi, s));
  return PDM_OK;
}

}  // namespace

extern "C" {

int pdm_clip_create(const pdm_clip_cfg* cfg, pdm_clip** out) {
  if (!cfg || !out) return cfail(PDM_ERR_ARG, "pdm_clip_create: null argument");
  const pdm_clip_cfg& k = *cfg;
  if (k.width <= 0 || k.heads <= 0 || k.width % k.heads) return cfail(PDM_ERR_ARG, "clip: width must be a multiple of heads");
  const int Dh = k.width / k.heads;
  if (Dh != 64 && Dh != 32) return cfail(PDM_ERR_ARG, "clip: head dim must be 32 or 64");
  if (k.width % 64 || k.mlp_hidden % 64 || k.width > 2048) return cfail(PDM_ERR_ARG, "clip: width / mlp_hidden must be multiples of 64, width <= 2048");
  if (k.max_position < 1 || k.max_position > 128) return cfail(PDM_ERR_ARG, "clip: 1..128 positions supported");
  if (k.layers < 1 || k.vocab < 1) return cfail(PDM_ERR_ARG, "clip: layers and vocab must be positive");
  pdm_clip* c = new pdm_clip();
  c->cfg = k;
  c->Dh = Dh;
  c->T = (k.width + 255) / 256;
  const long long D = k.width, F = k.mlp_hidden;
  c->add("embeddings.token_embedding.weight", PDM_F32, (long long)k.vocab * D);
  c->add("embeddings.position_embedding.weight", PDM_F32, (long long)k.max_position * D);
  for (int i = 0; i < k.layers; ++i) {
    const std::string p = "encoder.layers." + std::to_string(i);
    c->add(p + ".self_attn.qkv.weight", PDM_BF16, 3 * D * D);
    c->add(p + ".self_attn.qkv.ln_colsum", PDM_F32, 3 * D);
    c->add(p + ".self_attn.qkv.ln_bias", PDM_F32, 3 * D);
    c->add(p + ".self_attn.out_proj.weight", PDM_BF16, D * D);
    c->add(p + ".self_attn.out_proj.bias", PDM_F32, D);
    c->add(p + ".mlp.fc1.weight", PDM_BF16, F * D);
    c->add(p + ".mlp.fc1.ln_colsum", PDM_F32, F);
    c->add(p + ".mlp.fc1.ln_bias", PDM_F32, F);
    c->add(p + ".mlp.fc2.weight", PDM_BF16, D * F);
    c->add(p + ".mlp.fc2.bias", PDM_F32, D);
  }
  c->add("final_layer_norm.weight", PDM_F32, D);
  c->add("final_layer_norm.bias", PDM_F32, D);
  *out = c;
  return PDM_OK;
}

int pdm_clip_destroy(pdm_clip* c) {
  delete c;
  return PDM_OK;
}

int pdm_clip_param_count(const pdm_clip* c) { return c ? (int)c->order.size() : 0; }

int pdm_clip_param_info(const pdm_clip* c, int i, char* name, int len, int* dtype, long long* numel) {
  if (!c || i < 0 || i >= (int)c->order.size()) return cfail(PDM_ERR_ARG, "pdm_clip_param_info: index out of range");
  snprintf(name, len, "%s", c->order[i].c_str());
  *dtype = c->params.at(c->order[i]).dtype;
  *numel = c->params.at(c->order[i]).numel;
  return PDM_OK;
}

int pdm_clip_set_param(pdm_clip* c, const char* name, const void* ptr, int dtype, long long numel) {
  if (!c || !name) return cfail(PDM_ERR_ARG, "pdm_clip_set_param: null argument");
  auto it = c->params.find(name);
  if (it == c->params.end()) return cfail(PDM_ERR_ARG, std::string("pdm_clip_set_param: unexpected key ") + name);
  if (it->second.dtype != dtype || it->second.numel != numel)
    return cfail(PDM_ERR_ARG, std::string("pdm_clip_set_param: dtype/size mismatch for ") + name);
  if ((uintptr_t)ptr & 15) return cfail(PDM_ERR_ARG, std::string("pdm_clip_set_param: unaligned ") + name);
  it->second.ptr = ptr;
  return PDM_OK;
}

int pdm_clip_workspace_size(const pdm_clip* c, int B, size_t* bytes) {
  if (!c || B <= 0 || !bytes) return cfail(PDM_ERR_ARG, "pdm_clip_workspace_size: bad argument");
  *bytes = clayout(c, B, nullptr).bytes;
  return PDM_OK;
}

int pdm_clip_encode(pdm_clip* c, const int64_t* ids, int B, int L, float* out, void* workspace, size_t workspace_bytes,
                    void* stream) {
  if (!c || !ids || !out || B <= 0) return cfail(PDM_ERR_ARG, "pdm_clip_encode: bad argument");
  if (L < 1 || L > c->cfg.max_position) return cfail(PDM_ERR_ARG, "pdm_clip_encode: sequence length must be in [1, max_position]");
  for (auto& n : c->order)
    if (!c->params[n].ptr) return cfail(PDM_ERR_STATE, "pdm_clip: weight not registered: " + n);
  CWork w = clayout(c, B, (char*)workspace);
  if (w.bytes > workspace_bytes) return cfail(PDM_ERR_ARG, "pdm_clip_encode: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int D = c->cfg.width, F = c->cfg.mlp_hidden, M = B * L;
  hipLaunchKernelGGL(pdm::clip_embed_kernel, dim3((M + 3) / 4), dim3(256), 0, s, (const long long*)ids,
                     c->f("embeddings.token_embedding.weight"), c->f("embeddings.position_embedding.weight"), w.X, M, L,
                     D, c->cfg.vocab);
  C_HIP(hipGetLastError());
  C_HIP(pdm::rowstats_launch(w.X, D, M, D, w.XB, D, w.ST, c->T, s));
  for (int i = 0; i < c->cfg.layers; ++i) {
    const std::string p = "encoder.layers." + std::to_string(i);
    // qkv = q/k/v_proj(LN1 x)
    C_TRY(clip_gemm(s, c, w.XB, D, c->w(p + ".self_attn.qkv.weight"), c->f(p + ".self_attn.qkv.ln_bias"), M, 3 * D, D,
                    pdm::EPI_BF16, w.QKV, nullptr, 0, w.ST, c->f(p + ".self_attn.qkv.ln_colsum"), nullptr));
    const float scale = 1.0f / sqrtf((float)c->Dh);
    if (c->Dh == 64)
      hipLaunchKernelGGL(pdm::clip_attention_kernel<64>, dim3(c->cfg.heads, B), dim3(128), 0, s, w.QKV, 3 * D, w.ATT, D,
                         L, D, scale);
    else
      hipLaunchKernelGGL(pdm::clip_attention_kernel<32>, dim3(c->cfg.heads, B), dim3(128), 0, s, w.QKV, 3 * D, w.ATT, D,
                         L, D, scale);
    C_HIP(hipGetLastError());
    // x += out_proj(attn)   (epilogue: bf16 copy + LN2 partials of the new x)
    C_TRY(clip_gemm(s, c, w.ATT, D, c->w(p + ".self_attn.out_proj.weight"), c->f(p + ".self_attn.out_proj.bias"), M, D,
                    D, pdm::EPI_F32, w.XT, w.X, 1, nullptr, nullptr, w.STT));
    // h = quick_gelu(fc1(LN2 x))
    C_TRY(clip_gemm(s, c, w.XT, D, c->w(p + ".mlp.fc1.weight"), c->f(p + ".mlp.fc1.ln_bias"), M, F, D, pdm::EPI_GELU,
                    w.MLP, nullptr, 0, w.STT, c->f(p + ".mlp.fc1.ln_colsum"), nullptr));
    // x += fc2(h)           (epilogue: bf16 copy + LN1 partials for the next layer)
    C_TRY(clip_gemm(s, c, w.MLP, F, c->w(p + ".mlp.fc2.weight"), c->f(p + ".mlp.fc2.bias"), M, D, F, pdm::EPI_F32,
                    w.XB, w.X, 1, nullptr, nullptr, w.ST));
  }
  const int per = (D + 63) / 64;
  const dim3 g((M + 3) / 4), b(256);
  const float* lg = c->f("final_layer_norm.weight");
  const float* lb = c->f("final_layer_norm.bias");
  if (per <= 4) hipLaunchKernelGGL(pdm::clip_final_ln_kernel<4>, g, b, 0, s, w.X, lg, lb, out, M, D, c->cfg.eps);
  else if (per <= 8) hipLaunchKernelGGL(pdm::clip_final_ln_kernel<8>, g, b, 0, s, w.X, lg, lb, out, M, D, c->cfg.eps);
  else if (per <= 16) hipLaunchKernelGGL(pdm::clip_final_ln_kernel<16>, g, b, 0, s, w.X, lg, lb, out, M, D, c->cfg.eps);
  else hipLaunchKernelGGL(pdm::clip_final_ln_kernel<32>, g, b, 0, s, w.X, lg, lb, out, M, D, c->cfg.eps);
  C_HIP(hipGetLastError());
  return PDM_OK;
}

}  // extern "C"

// KL-f8 decoder (libs/autoencoder.py:303-409 + FrozenAutoencoderKL.decode 446-450) on gfx950.
//
// Activations are NHWC; the residual stream is fp32, every conv input is a bf16 NHWC tensor produced by a
// fused GroupNorm(32)+swish apply (or a plain cast).  Every 3x3 conv is an implicit GEMM on the U-ViT GEMM
// kernels (conv mode: per-row tap addressing, padded taps read a zero page, the nearest-x2 upsample folded
// into the source address), with bias and the residual add fused into the epilogue (EPI_F32 accumulate
// into the residual stream).  The mid attention block (single head over h*w tokens, C = 512) runs as a
// packed qkv GEMM, batched Q K^T / P V GEMMs and a row softmax.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <string>
#include <vector>

#include "../../include/pdm.h"
#include "pdm_common.h"
#include "pdm_kernels.h"

using pdm::bf16;

namespace pdm {
namespace {

// ---------------------------------------------------------------------------------------------------
// GroupNorm statistics: grid (nchunk, B); each block reduces `pix` pixels x C channels in fp64 (sum, sumsq)
// per group, partials -> [B, nchunk, 32, 2]; gn_final combines them into (mean, rstd) per (b, g).  pix is chosen
// per level so that a block streams ~256 KiB (gn_pix below): 64-pixel chunks left every block latency-bound.
constexpr int GN_PIX = 64;   // smallest chunk (sizes the partials buffer)
inline int gn_pix(int C) { return C >= 1024 ? GN_PIX : 65536 / C; }

template <typename T>
__global__ __launch_bounds__(256) void gn_partial_kernel(const T* x, int P, int C, int nchunk, int pix, double* part) {
  // thread -> one channel quad q of pixel lane `plane` (C <= 1024): per-channel fp32 sums over its <= pix/planes
  // pixels in registers (compile-time indexed: a runtime group index sent the accumulators to scratch), then
  // one fp64 pass per group over the [plane][channel] partials in LDS
  __shared__ float2 red[1024];
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int nq = C >> 2, q = threadIdx.x % nq, plane = threadIdx.x / nq, planes = 256 / nq;
  const int p0 = chunk * pix, p1 = min(P, p0 + pix);
  if (plane < planes) {
    const T* xb = x + (size_t)b * P * C + q * 4;
    float su[4] = {0.f, 0.f, 0.f, 0.f}, sq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int pi = p0 + plane; pi < p1; pi += planes) {
      float v[4];
      if constexpr (sizeof(T) == 4) {
        const f32x4 t = *reinterpret_cast<const f32x4*>(xb + (size_t)pi * C);
        v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
      } else {
        const bf16x4 t = *reinterpret_cast<const bf16x4*>(xb + (size_t)pi * C);
        v[0] = (float)t[0]; v[1] = (float)t[1]; v[2] = (float)t[2]; v[3] = (float)t[3];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        su[j] += v[j];
        sq[j] = fmaf(v[j], v[j], sq[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) red[plane * C + q * 4 + j] = make_float2(su[j], sq[j]);
  }
  __syncthreads();
  if (threadIdx.x < 32) {
    const int g = threadIdx.x, cpg = C / 32;
    double s = 0.0, qq = 0.0;
    for (int pl = 0; pl < planes; ++pl)
      for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
        const float2 r = red[pl * C + c];
        s += r.x;
        qq += r.y;
      }
    double* o = part + (((size_t)b * nchunk + chunk) * 32 + g) * 2;
    o[0] = s;
    o[1] = qq;
  }
}

// one wave per (b, g): lanes stride over the chunks, then a wave reduction (a serial per-thread loop over the
// chunks was a chain of dependent global loads, ~135 us per call)
__global__ __launch_bounds__(256) void gn_final_kernel(const double* part, int nchunk, double count, float eps,
                                                       float* stats, int B) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;   // (b, g)
  if (i >= B * 32) return;
  const int b = i / 32, g = i % 32;
  double s = 0.0, q = 0.0;
  for (int c = lane; c < nchunk; c += 64) {
    const double* o = part + (((size_t)b * nchunk + c) * 32 + g) * 2;
    s += o[0];
    q += o[1];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    q += __shfl_xor(q, o, 64);
  }
  if (lane) return;
  const double mean = s / count;
  double var = q / count - mean * mean;
  var = var < 0.0 ? 0.0 : var;
  stats[i * 2] = (float)mean;
  stats[i * 2 + 1] = (float)(1.0 / sqrt(var + (double)eps));
}

// y = [swish]((x - mean) * rstd * gamma + beta), NHWC, bf16 out.  Grid (gx, B): a block stays in one image and
// every thread keeps one channel octet q (C <= 2048, C % 8 == 0) for all its pixels, so the per-channel affine
// a = rstd * gamma, b = beta - mean * a is folded once into registers and the pixel loop is two 16-byte loads
// (fp32; one for bf16), one FMA + swish per element and one 16-byte store, 32-bit indexing only.  (The first
// version decoded (image, pixel, channel) from a flat 64-bit index per element and reloaded stats, gamma and
// beta per element: ~40 % of HBM bandwidth.)  swish = u / (1 + 2^(-u log2 e)) with the hardware exp2 and
// reciprocal (u -> -inf gives -0, no NaN).
template <typename T>
__global__ __launch_bounds__(256) void gn_apply_kernel(const T* x, const float* stats, const float* gamma,
                                                       const float* beta, bf16* y, int P, int C, int swish) {
  const int no = C >> 3, planes = 256 / no, q = threadIdx.x % no, plane = threadIdx.x / no;
  if (plane >= planes) return;
  const int b = blockIdx.y, c = q * 8, cpg = C / 32;
  float a[8], o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int g = (c + j) / cpg;   // cpg may be 2 or 6: an octet can straddle groups
    const float mean = stats[(b * 32 + g) * 2], rstd = stats[(b * 32 + g) * 2 + 1];
    a[j] = rstd * gamma[c + j];
    o[j] = fmaf(-mean, a[j], beta[c + j]);
  }
  const T* xb = x + (size_t)b * P * C + c;
  bf16* yb = y + (size_t)b * P * C + c;
  const int step = gridDim.x * planes;
#pragma unroll 4
  for (int pi = blockIdx.x * planes + plane; pi < P; pi += step) {
    float v[8];
    if constexpr (sizeof(T) == 4) {
      const f32x4 t0 = *reinterpret_cast<const f32x4*>(xb + (size_t)pi * C);
      const f32x4 t1 = *reinterpret_cast<const f32x4*>(xb + (size_t)pi * C + 4);
      v[0] = t0[0]; v[1] = t0[1]; v[2] = t0[2]; v[3] = t0[3];
      v[4] = t1[0]; v[5] = t1[1]; v[6] = t1[2]; v[7] = t1[3];
    } else {
      const bf16x8 t = *reinterpret_cast<const bf16x8*>(xb + (size_t)pi * C);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (float)t[j];
    }
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float u = fmaf(v[j], a[j], o[j]);
      if (swish) u *= __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(u * -1.4426950408889634f));
      r[j] = (bf16)u;
    }
    *reinterpret_cast<bf16x8*>(yb + (size_t)pi * C) = r;
  }
}

// z [B, 4, h, w] fp32 -> z / scale -> post_quant_conv (1x1, 4->4) -> conv_in (3x3, 4->Cout) -> NHWC fp32
__global__ __launch_bounds__(256) void conv_in_kernel(const float* z, float inv_scale, const float* pq_w,
                                                      const float* pq_b, const float* w, const float* bias,
                                                      float* out, int h, int wd, int Cout) {
  const int b = blockIdx.y, y = blockIdx.x;
  __shared__ float rows[3][4][66];   // 3 input rows x 4 channels x (w + 2 halo), post_quant applied
  for (int e = threadIdx.x; e < 3 * 4 * (wd + 2); e += 256) {
    const int r = e / (4 * (wd + 2)), rem = e % (4 * (wd + 2)), c = rem / (wd + 2), xx = rem % (wd + 2) - 1;
    const int yy = y + r - 1;
    float v = 0.f;
    if (yy >= 0 && yy < h && xx >= 0 && xx < wd) {
      v = pq_b[c];
      for (int ci = 0; ci < 4; ++ci) v += pq_w[c * 4 + ci] * z[(((size_t)b * 4 + ci) * h + yy) * wd + xx] * inv_scale;
    }
    rows[r][c][xx + 1] = v;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < wd * Cout; e += 256) {
    const int x = e / Cout, co = e % Cout;
    float acc = bias[co];
    const float* wp = w + (size_t)co * 36;
    for (int ci = 0; ci < 4; ++ci)
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) acc = fmaf(wp[ci * 9 + ky * 3 + kx], rows[ky][ci][x + kx], acc);
    out[(((size_t)b * h + y) * wd + x) * Cout + co] = acc;
  }
}

// row softmax of fp32 scores * scale -> bf16 probabilities (rows of n <= 4096), one block per row; the row is
// read once into registers (16 values per thread; the three-pass form re-read it for the max, the sum and
// the output: 1.38 ms for 32 x 4096 rows of 4096)
__global__ __launch_bounds__(256) void softmax_rows_kernel(const float* s, bf16* p, int n, float scale) {
  const float* row = s + (size_t)blockIdx.x * n;
  bf16* out = p + (size_t)blockIdx.x * n;
  __shared__ float red[8];
  float v[16];
  float m = -3.0e38f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int i = threadIdx.x + j * 256;
    v[j] = i < n ? row[i] * scale : -3.0e38f;
    m = fmaxf(m, v[j]);
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    v[j] = __expf(v[j] - m);   // 0 past n
    sum += v[j];
  }
  sum = wave_sum(sum);
  if ((threadIdx.x & 63) == 0) red[4 + (threadIdx.x >> 6)] = sum;
  __syncthreads();
  const float inv = 1.0f / ((red[4] + red[5]) + (red[6] + red[7]));
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int i = threadIdx.x + j * 256;
    if (i < n) out[i] = (bf16)(v[j] * inv);
  }
}

// [B][n][ld] column block -> [B][C][n] transpose (bf16), 32x32 tiles through LDS
__global__ __launch_bounds__(256) void transpose_kernel(const bf16* src, int ld, int col0, bf16* dst, int n, int C) {
  __shared__ bf16 t[32][33];
  const int b = blockIdx.z;
  const int r0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
  const bf16* s = src + (size_t)b * n * ld + col0;
  bf16* d = dst + (size_t)b * C * n;
  for (int i = threadIdx.x; i < 1024; i += 256) {
    const int r = i / 32, c = i % 32;
    t[r][c] = s[(size_t)(r0 + r) * ld + c0 + c];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 1024; i += 256) {
    const int c = i / 32, r = i % 32;
    d[(size_t)(c0 + c) * n + r0 + r] = t[r][c];
  }
}

// conv_out (libs/autoencoder.py:408-409): 3x3 conv, Cin -> out_ch <= 4, on the GN+swish bf16 NHWC input, written
// straight to the NCHW fp32 image.  N = 3 is far too narrow for an MFMA tile (a 128-wide tile wastes 97 % of
// its work), so one thread computes one pixel's outputs on the VALU: 9 taps x Cin/8 16-byte loads (neighbour
// rows come from L1 / L2); the weights are staged once per block into LDS as fp32 [tap][ci][4 outputs], so each
// input channel costs one broadcast ds_read_b128 + 4 FMAs (per-lane weight loads from global cost 4x the input
// bandwidth).
__global__ __launch_bounds__(256) void conv_out_kernel(const bf16* g, int B, int H, int W, int C, const bf16* w,
                                                       const float* bias, float* img, int out_ch) {
  extern __shared__ __attribute__((aligned(16))) f32x4 wl[];   // [9 * C]
  for (int i = threadIdx.x; i < 9 * C; i += 256)
    wl[i] = f32x4{(float)w[i], (float)w[9 * C + i], (float)w[18 * C + i], (float)w[27 * C + i]};
  __syncthreads();
  const long long pix = (long long)blockIdx.x * 256 + threadIdx.x;
  if (pix >= (long long)B * H * W) return;
  const int b = (int)(pix / ((long long)H * W));
  const int r = (int)(pix - (long long)b * H * W), y = r / W, x = r - (r / W) * W;
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int tap = 0; tap < 9; ++tap) {
    const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
    if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
    const bf16* src = g + (((size_t)b * H + yy) * W + xx) * C;
    const f32x4* wt = wl + tap * C;
    for (int c0 = 0; c0 < C; c0 += 8) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(src + c0);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += (float)v[j] * wt[c0 + j];
    }
  }
  for (int o = 0; o < out_ch; ++o) img[((size_t)b * out_ch + o) * H * W + r] = acc[o] + bias[o];
}

// The same conv for C in {64, 128} (every shipped decoder) on the matrix cores: out[pixel][o] is a GEMM of the
// 9 * C im2col row with a 9C x 16 weight block (o >= out_ch zero), one v_mfma_f32_16x16x32_bf16 per 32-channel
// slice of a tap.  A block owns two output rows of one image and walks them in 64-pixel segments (4 waves x 16
// pixels x 2 rows); per segment the 4 x 66 halo of input pixels is staged in LDS once by LDS-DMA (every input
// pixel was re-read by 9 taps from L2 in the VALU version: 4.7 ms for 32 images at 512^2; register-staged loads
// with one load in flight per thread: 1.9 ms), each pixel's 16-byte channel chunks XOR-swizzled by the pixel
// index so the 16 lanes of an A-fragment read (16 consecutive pixels, one chunk) hit distinct banks.  The DMA
// writes lane-linearly, so the swizzle is applied to the SOURCE chunk; halo pixels outside the image read as
// zeros through the buffer descriptor's range check.  Two blocks per CU (68 KiB of LDS each) overlap one's
// staging with the other's MFMAs.  A lane keeps its B fragments (w[o = lane % 16][k-slice]) for the whole K in
// registers.
template <int C>
__global__ __launch_bounds__(256) void conv_out_mfma_kernel(const bf16* g, int H, int W, const bf16* w,
                                                            const float* bias, float* img, int out_ch) {
  constexpr int NQ = C / 8;                  // 16-byte chunks per pixel
  constexpr int SW = (NQ < 16 ? NQ : 16) - 1;
  constexpr int SEG = 64, PX = SEG + 2;      // output pixels per segment, staged pixels per row
  constexpr int SLOTS = 4 * PX * NQ;         // 16-byte LDS slots per segment (4 input rows)
  constexpr int KS = 9 * C / 32;             // MFMA k-steps (a k-step never straddles a tap: C % 32 == 0)
  static_assert(SLOTS % 64 == 0, "every LDS-DMA wave-instruction lands 64 slots inside the tile");
  __shared__ __attribute__((aligned(16))) bf16 tile[SLOTS * 8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int y0 = blockIdx.x * 2, b = blockIdx.y;
  const int o = lane & 15, kq = (lane >> 4) * 8;
  bf16x8 wf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    wf[ks] = bf16x8{};
    if (o < out_ch) wf[ks] = *reinterpret_cast<const bf16x8*>(w + (size_t)o * 9 * C + ks * 32 + kq);
  }
  const float bo = o < out_ch ? bias[o] : 0.f;
  const long long img_bytes = (long long)H * W * C * 2;
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16*>(g + (size_t)b * H * W * C), 0, (int)(img_bytes < 0x7fffffffLL ? img_bytes : 0x7fffffffLL), 0x00020000);
  for (int x0 = 0; x0 < W; x0 += SEG) {
    // slot e = (r * PX + px) * NQ + s holds logical chunk s ^ (px & SW) of input pixel (y0 - 1 + r, x0 - 1 + px)
    for (int e0 = wave * 64; e0 < SLOTS; e0 += 256) {
      const int e = e0 + lane;
      const int r = e / (PX * NQ), rem = e - r * (PX * NQ), px = rem / NQ, sl = rem - px * NQ;
      const int yy = y0 + r - 1, xx = x0 + px - 1;
      const unsigned off = (e < SLOTS && yy >= 0 && yy < H && xx >= 0 && xx < W)
                               ? (unsigned)((yy * W + xx) * C + ((sl ^ (px & SW)) << 3)) * 2u : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rg, (PDM_LDS void*)(tile + e0 * 8), 16, (int)off, 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int dy = tap / 3, dx = tap - (tap / 3) * 3;
      const int px = wave * 16 + (lane & 15) + dx;
#pragma unroll
      for (int c0 = 0; c0 < C; c0 += 32) {
        const int q = (c0 + kq) >> 3;
        const int sw = (q ^ (px & SW)) * 8;
        const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(tile + (dy * PX + px) * NQ * 8 + sw);
        const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(tile + ((dy + 1) * PX + px) * NQ * 8 + sw);
        acc0 = mfma16x16x32(a0, wf[tap * (C / 32) + c0 / 32], acc0);
        acc1 = mfma16x16x32(a1, wf[tap * (C / 32) + c0 / 32], acc1);
      }
    }
    // D[pixel 4 * (lane / 16) + i][o = lane % 16]: 4 consecutive pixels of output channel o
    if (o < out_ch) {
      float* op = img + (((size_t)b * out_ch + o) * H + y0) * W + x0 + wave * 16 + 4 * (lane >> 4);
      *reinterpret_cast<f32x4*>(op) = acc0 + bo;
      *reinterpret_cast<f32x4*>(op + W) = acc1 + bo;
    }
    __syncthreads();   // every wave is done reading the tile before the next segment restages it
  }
}

}  // namespace
}  // namespace pdm

// =====================================================================================================
namespace {

int dfail(int code, const std::string& m) { return pdm::set_error(code, m); }
#define D_HIP(call)                                                                                   \
  do {                                                                                                \
    hipError_t e_ = (call);                                                                           \
    if (e_ != hipSuccess) return dfail(PDM_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define D_CHECK(m)                              \
  do {                                          \
    const char* m_ = (m);                       \
    if (m_) return dfail(PDM_ERR_ARG, m_);      \
  } while (0)
#define D_TRY(x)        \
  do {                  \
    int r_ = (x);       \
    if (r_) return r_;  \
  } while (0)

struct DParam {
  int dtype;
  long long numel;
  const void* ptr = nullptr;
};

}  // namespace

struct pdm_decoder {
  pdm_decoder_cfg cfg;
  int nlev, top_ch, h0;
  std::vector<std::string> order;
  std::map<std::string, DParam> params;
  void add(const std::string& n, int dt, long long ne) {
    order.push_back(n);
    params[n] = DParam{dt, ne, nullptr};
  }
  const float* f(const std::string& n) const { return (const float*)params.at(n).ptr; }
  const bf16* w(const std::string& n) const { return (const bf16*)params.at(n).ptr; }
  void add_res(const std::string& p, int cin, int cout) {
    add(p + ".norm1.weight", PDM_F32, cin);
    add(p + ".norm1.bias", PDM_F32, cin);
    add(p + ".conv1.weight", PDM_BF16, 9LL * cin * cout);
    add(p + ".conv1.bias", PDM_F32, cout);
    add(p + ".norm2.weight", PDM_F32, cout);
    add(p + ".norm2.bias", PDM_F32, cout);
    add(p + ".conv2.weight", PDM_BF16, 9LL * cout * cout);
    add(p + ".conv2.bias", PDM_F32, cout);
    if (cin != cout) {
      add(p + ".nin_shortcut.weight", PDM_BF16, 1LL * cin * cout);
      add(p + ".nin_shortcut.bias", PDM_F32, cout);
    }
  }
};

namespace {

struct DWork {
  float* X;       // residual stream fp32 NHWC (max pixels x channels)
  float* X2;      // second residual buffer (nin shortcut / upsample output)
  bf16* G;        // bf16 conv input
  bf16* H;        // bf16 conv1 output
  bf16* XB;       // bf16 copy of X for the next block's nin_shortcut, written by the producing conv's epilogue
  bf16* QKV;      // attention: [B*hw, 3C]
  float* S;       // attention scores [B, hw, hw]
  bf16* P;        // probabilities [B, hw, hw]
  bf16* VT;       // V^T [B, C, hw]
  bf16* O;        // attention output [B*hw, C]
  double* part;   // GN partials
  float* stats;   // GN (mean, rstd) [B, 32, 2]
  bf16* zero;     // 256 zero bytes
  size_t bytes;
};

size_t aup(size_t x) { return (x + 255) / 256 * 256; }
using pdm::GN_PIX;

DWork dlayout(const pdm_decoder* d, int B, char* base) {
  DWork w{};
  size_t off = 0;
  auto take = [&](size_t n) {
    char* p = base ? base + off : nullptr;
    off = aup(off + n);
    return p;
  };
  // largest activation: after the last upsample, 2^(nlev-1) * h0 squared pixels x the preceding level's C
  size_t maxe = 0;
  int res = d->h0, cin = d->top_ch;
  for (int lvl = d->nlev - 1; lvl >= 0; --lvl) {
    const int cout = d->cfg.ch * d->cfg.ch_mult[lvl];
    size_t e = (size_t)res * res * (cin > cout ? cin : cout);
    if (e > maxe) maxe = e;
    cin = cout;
    if (lvl != 0) {
      res *= 2;
      e = (size_t)res * res * cin;
      if (e > maxe) maxe = e;
    }
  }
  const size_t hw = (size_t)d->h0 * d->h0;
  w.X = (float*)take((size_t)B * maxe * 4);
  w.X2 = (float*)take((size_t)B * maxe * 4);
  w.G = (bf16*)take((size_t)B * maxe * 2);
  w.H = (bf16*)take((size_t)B * maxe * 2);
  w.XB = (bf16*)take((size_t)B * maxe * 2);
  w.QKV = (bf16*)take((size_t)B * hw * 3 * d->top_ch * 2);
  w.S = (float*)take((size_t)B * hw * hw * 4);
  w.P = (bf16*)take((size_t)B * hw * hw * 2);
  w.VT = (bf16*)take((size_t)B * hw * d->top_ch * 2);
  w.O = (bf16*)take((size_t)B * hw * d->top_ch * 2);
  w.part = (double*)take((size_t)B * ((size_t)res * res / GN_PIX + 1) * 32 * 2 * sizeof(double));
  w.stats = (float*)take((size_t)B * 32 * 2 * 4);
  w.zero = (bf16*)take(256);
  w.bytes = off;
  return w;
}

struct DCtx {
  const pdm_decoder* d;
  hipStream_t s;
  const DWork* w;
  // set by the GEMM / conv that just wrote the next GroupNorm's input with GemmArgs::gn_part (its partials in w->part,
  // 256-pixel chunks), cleared by the GroupNorm that consumes them
  bool* gn_ready;
};

template <typename T>
int groupnorm(const DCtx& c, const T* x, int B, int P, int C, const std::string& norm, bf16* y, bool swish) {
  // statistics pass: skipped when the producing epilogue already left the partials (one read of x fewer)
  const bool pre = *c.gn_ready;
  *c.gn_ready = false;
  const int pix = pre ? 256 : pdm::gn_pix(C);
  const int nchunk = (P + pix - 1) / pix;
  if (!pre)
    hipLaunchKernelGGL(pdm::gn_partial_kernel<T>, dim3(nchunk, B), dim3(256), 0, c.s, x, P, C, nchunk, pix, c.w->part);
  hipLaunchKernelGGL(pdm::gn_final_kernel, dim3((B * 32 + 3) / 4), dim3(256), 0, c.s, c.w->part, nchunk,
                     (double)P * (C / 32), 1e-6f, c.w->stats, B);
  if (C % 8 || C > 2048) return dfail(PDM_ERR_ARG, "decoder: GroupNorm needs C % 8 == 0 and C <= 2048");
  const int planes = 256 / (C / 8);
  // >= ~8192 blocks (up to 32 waves per CU): the pixel loop keeps 4 pixels' loads in flight per thread, and at
  // ~2048 blocks the fp32 apply streamed at ~2.5 TB/s (512^2 decode, profiles/r03r_dec512_kernel_stats.csv)
  const int gx = std::max(1, std::min((P + planes - 1) / planes, 8192 / B + 1));
  hipLaunchKernelGGL(pdm::gn_apply_kernel<T>, dim3(gx, B), dim3(256), 0, c.s, x, c.w->stats,
                     c.d->f(norm + ".weight"), c.d->f(norm + ".bias"), y, P, C, swish ? 1 : 0);
  D_HIP(hipGetLastError());
  return PDM_OK;
}

// implicit-GEMM conv3x3 (in: bf16 NHWC [B, res>>up, res>>up, cin]) -> epilogue
bool g_gn_fusion = true;   // pdm_decoder_set_gn_fusion

// gn_P > 0: the output is the next GroupNorm's input (gn_P pixels per image): its epilogue also writes the GroupNorm
// partials where it can (pdm::gemm_gn_fusable; c.gn_ready tells the GroupNorm)
int launch_gn(const DCtx& c, pdm::GemmArgs& a, int epi, int gn_P) {
  if (gn_P > 0 && g_gn_fusion) {
    a.gn_part = c.w->part; a.gn_P = gn_P; a.gn_cpg = a.N / 32;
    if (!pdm::gemm_gn_fusable(a, epi)) a.gn_part = nullptr;
  }
  D_CHECK(pdm::gemm_check(a, epi));
  D_HIP(pdm::gemm_launch(a, epi, c.s));
  *c.gn_ready = a.gn_part != nullptr;
  return PDM_OK;
}

int conv3(const DCtx& c, const bf16* in, int B, int res, int cin, int cout, const std::string& name, int epi,
          bf16* ob, float* of, int accumulate, int up = 0, bool gn = false) {
  pdm::GemmArgs a{};
  a.A1 = in; a.lda1 = cin; a.K1 = 9 * cin;
  a.W = c.d->w(name + ".weight"); a.bias = c.d->f(name + ".bias");
  a.M = B * res * res; a.N = cout; a.K = 9 * cin;
  a.out_bf16 = ob; a.ldo = cout; a.out_f32 = of; a.ldr = cout; a.accumulate = accumulate;
  a.conv = 1; a.convH = res; a.convW = res; a.convC = cin; a.conv_up = up; a.zero = c.w->zero;
  return launch_gn(c, a, epi, gn ? res * res : 0);
}

int linear(const DCtx& c, const bf16* A, int M, int K, const bf16* W, const float* bias, int N, int epi, bf16* ob,
           float* of, int accumulate, int gn_P = 0) {
  pdm::GemmArgs a{};
  a.A1 = A; a.lda1 = K; a.K1 = K; a.W = W; a.bias = bias; a.M = M; a.N = N; a.K = K;
  a.out_bf16 = ob; a.ldo = N; a.out_f32 = of; a.ldr = N; a.accumulate = accumulate;
  return launch_gn(c, a, epi, gn_P);
}

// ResnetBlock (libs/autoencoder.py:75-134): X (fp32 NHWC, cin) -> X (cout) in place (or via X2 for nin).
// xb: bf16(X) already made by the epilogue that produced X (else the nin_shortcut casts X itself); copy_out:
// where conv2's epilogue also stores bf16 of the block output (the next upsample conv's source), or null.
int resblock(const DCtx& c, float*& X, float*& X2, int B, int res, int cin, int cout, const std::string& p,
             const bf16* xb = nullptr, bf16* copy_out = nullptr) {
  const DWork& w = *c.w;
  const int P = res * res;
  D_TRY(groupnorm<float>(c, X, B, P, cin, p + ".norm1", w.G, true));
  D_TRY(conv3(c, w.G, B, res, cin, cout, p + ".conv1", pdm::EPI_BF16, w.H, nullptr, 0, 0, true));
  D_TRY(groupnorm<bf16>(c, w.H, B, P, cout, p + ".norm2", w.G, true));
  if (cin != cout) {
    // x = nin_shortcut(x): 1x1 conv = GEMM on a bf16 copy of x, into X2; then X2 += conv2(h)
    if (!xb) {
      D_HIP(pdm::cast_bf16_launch(X, w.H, (long long)B * P * cin, c.s));
      xb = w.H;
    }
    D_TRY(linear(c, xb, B * P, cin, c.d->w(p + ".nin_shortcut.weight"), c.d->f(p + ".nin_shortcut.bias"), cout,
                 pdm::EPI_F32, nullptr, X2, 0));
    D_TRY(conv3(c, w.G, B, res, cout, cout, p + ".conv2", pdm::EPI_F32, copy_out, X2, 1, 0, true));
    float* t = X;
    X = X2;
    X2 = t;
  } else {
    D_TRY(conv3(c, w.G, B, res, cout, cout, p + ".conv2", pdm::EPI_F32, copy_out, X, 1, 0, true));
  }
  return PDM_OK;
}

// AttnBlock (libs/autoencoder.py:143-195), single head over hw tokens, channels C
int attnblock(const DCtx& c, float* X, int B, int res, int C, const std::string& p) {
  const DWork& w = *c.w;
  const int hw = res * res;
  D_TRY(groupnorm<float>(c, X, B, hw, C, p + ".norm", w.G, false));
  D_TRY(linear(c, w.G, B * hw, C, c.d->w(p + ".qkv.weight"), c.d->f(p + ".qkv.bias"), 3 * C, pdm::EPI_BF16, w.QKV,
               nullptr, 0));
  {  // S[b] = Q[b] K[b]^T  (batched over b)
    pdm::GemmArgs a{};
    a.A1 = w.QKV; a.lda1 = 3 * C; a.K1 = C;
    a.W = w.QKV + C; a.ldw = 3 * C;
    a.M = hw; a.N = hw; a.K = C;
    a.out_f32 = w.S; a.ldr = hw;
    a.batch = B; a.sA = (long long)hw * 3 * C; a.sW = (long long)hw * 3 * C; a.sR = (long long)hw * hw;
    D_CHECK(pdm::gemm_check(a, pdm::EPI_F32));
    D_HIP(pdm::gemm_launch(a, pdm::EPI_F32, c.s));
  }
  hipLaunchKernelGGL(pdm::softmax_rows_kernel, dim3(B * hw), dim3(256), 0, c.s, w.S, w.P, hw, 1.0f / sqrtf((float)C));
  hipLaunchKernelGGL(pdm::transpose_kernel, dim3(hw / 32, C / 32, B), dim3(256), 0, c.s, w.QKV, 3 * C, 2 * C, w.VT, hw, C);
  D_HIP(hipGetLastError());
  {  // O[b] = P[b] V[b]  with V^T as the [N][K] operand
    pdm::GemmArgs a{};
    a.A1 = w.P; a.lda1 = hw; a.K1 = hw;
    a.W = w.VT;
    a.M = hw; a.N = C; a.K = hw;
    a.out_bf16 = w.O; a.ldo = C;
    a.batch = B; a.sA = (long long)hw * hw; a.sW = (long long)C * hw; a.sO = (long long)hw * C;
    D_CHECK(pdm::gemm_check(a, pdm::EPI_BF16));
    D_HIP(pdm::gemm_launch(a, pdm::EPI_BF16, c.s));
  }
  // x + proj_out(o)
  D_TRY(linear(c, w.O, B * hw, C, c.d->w(p + ".proj_out.weight"), c.d->f(p + ".proj_out.bias"), C, pdm::EPI_F32,
               nullptr, X, 1, hw));
  return PDM_OK;
}

}  // namespace

extern "C" {

int pdm_decoder_create(const pdm_decoder_cfg* cfg, pdm_decoder** out) {
  if (!cfg || !out) return dfail(PDM_ERR_ARG, "pdm_decoder_create: null argument");
  const pdm_decoder_cfg& c = *cfg;
  if (c.num_levels < 1 || c.num_levels > 4) return dfail(PDM_ERR_ARG, "decoder: 1..4 levels supported");
  if (c.z_channels != 4) return dfail(PDM_ERR_ARG, "decoder: z_channels must be 4");
  if (c.out_ch > 4) return dfail(PDM_ERR_ARG, "decoder: out_ch must be <= 4");
  for (int i = 0; i < c.num_levels; ++i)
    if ((c.ch * c.ch_mult[i]) % 64) return dfail(PDM_ERR_ARG, "decoder: channel counts must be multiples of 64");
  if (c.latent_size % 8 || c.latent_size > 64) return dfail(PDM_ERR_ARG, "decoder: latent size must be a multiple of 8, <= 64");
  for (int i = 0; i < c.num_levels; ++i)
    if (c.ch * c.ch_mult[i] > 1024) return dfail(PDM_ERR_ARG, "decoder: channel counts must be <= 1024");
  pdm_decoder* d = new pdm_decoder();
  d->cfg = c;
  d->nlev = c.num_levels;
  d->top_ch = c.ch * c.ch_mult[c.num_levels - 1];
  d->h0 = c.latent_size;
  const int T = d->top_ch;
  d->add("post_quant_conv.weight", PDM_F32, 16);
  d->add("post_quant_conv.bias", PDM_F32, 4);
  d->add("decoder.conv_in.weight", PDM_F32, (long long)T * 36);
  d->add("decoder.conv_in.bias", PDM_F32, T);
  d->add_res("decoder.mid.block_1", T, T);
  d->add("decoder.mid.attn_1.norm.weight", PDM_F32, T);
  d->add("decoder.mid.attn_1.norm.bias", PDM_F32, T);
  d->add("decoder.mid.attn_1.qkv.weight", PDM_BF16, 3LL * T * T);
  d->add("decoder.mid.attn_1.qkv.bias", PDM_F32, 3LL * T);
  d->add("decoder.mid.attn_1.proj_out.weight", PDM_BF16, 1LL * T * T);
  d->add("decoder.mid.attn_1.proj_out.bias", PDM_F32, T);
  d->add_res("decoder.mid.block_2", T, T);
  int cin = T;
  for (int lvl = d->nlev - 1; lvl >= 0; --lvl) {
    const int cout = c.ch * c.ch_mult[lvl];
    for (int b = 0; b <= c.num_res_blocks; ++b) {
      d->add_res("decoder.up." + std::to_string(lvl) + ".block." + std::to_string(b), cin, cout);
      cin = cout;
    }
    if (lvl != 0) {
      d->add("decoder.up." + std::to_string(lvl) + ".upsample.conv.weight", PDM_BF16, 9LL * cin * cin);
      d->add("decoder.up." + std::to_string(lvl) + ".upsample.conv.bias", PDM_F32, cin);
    }
  }
  d->add("decoder.norm_out.weight", PDM_F32, cin);
  d->add("decoder.norm_out.bias", PDM_F32, cin);
  d->add("decoder.conv_out.weight", PDM_BF16, 4LL * 9 * cin);   // padded to 4 output rows
  d->add("decoder.conv_out.bias", PDM_F32, 4);
  *out = d;
  return PDM_OK;
}

int pdm_decoder_set_gn_fusion(int on) {
  g_gn_fusion = on != 0;
  return PDM_OK;
}

int pdm_decoder_destroy(pdm_decoder* d) {
  delete d;
  return PDM_OK;
}

int pdm_decoder_param_count(const pdm_decoder* d) { return d ? (int)d->order.size() : 0; }

int pdm_decoder_param_info(const pdm_decoder* d, int i, char* name, int len, int* dtype, long long* numel) {
  if (!d || i < 0 || i >= (int)d->order.size()) return dfail(PDM_ERR_ARG, "pdm_decoder_param_info: index out of range");
  snprintf(name, len, "%s", d->order[i].c_str());
  *dtype = d->params.at(d->order[i]).dtype;
  *numel = d->params.at(d->order[i]).numel;
  return PDM_OK;
}

int pdm_decoder_set_param(pdm_decoder* d, const char* name, const void* ptr, int dtype, long long numel) {
  if (!d || !name) return dfail(PDM_ERR_ARG, "pdm_decoder_set_param: null argument");
  auto it = d->params.find(name);
  if (it == d->params.end()) return dfail(PDM_ERR_ARG, std::string("pdm_decoder_set_param: unexpected key ") + name);
  if (it->second.dtype != dtype || it->second.numel != numel)
    return dfail(PDM_ERR_ARG, std::string("pdm_decoder_set_param: dtype/size mismatch for ") + name);
  if ((uintptr_t)ptr & 15) return dfail(PDM_ERR_ARG, std::string("pdm_decoder_set_param: unaligned ") + name);
  it->second.ptr = ptr;
  return PDM_OK;
}

int pdm_decoder_workspace_size(const pdm_decoder* d, int B, size_t* bytes) {
  if (!d || B <= 0 || !bytes) return dfail(PDM_ERR_ARG, "pdm_decoder_workspace_size: bad argument");
  *bytes = dlayout(d, B, nullptr).bytes;
  return PDM_OK;
}

int pdm_decoder_decode(pdm_decoder* d, const float* z, float* img, int B, void* workspace, size_t workspace_bytes,
                       void* stream) {
  if (!d || !z || !img || B <= 0) return dfail(PDM_ERR_ARG, "pdm_decoder_decode: bad argument");
  for (auto& n : d->order)
    if (!d->params[n].ptr) return dfail(PDM_ERR_STATE, "pdm_decoder: weight not registered: " + n);
  DWork w = dlayout(d, B, (char*)workspace);
  if (w.bytes > workspace_bytes) return dfail(PDM_ERR_ARG, "pdm_decoder_decode: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  bool gn_ready = false;
  DCtx c{d, s, &w, &gn_ready};
  D_HIP(hipMemsetAsync(w.zero, 0, 256, s));
  const int T = d->top_ch;
  int res = d->h0;
  float* X = w.X;
  float* X2 = w.X2;
  hipLaunchKernelGGL(pdm::conv_in_kernel, dim3(res, B), dim3(256), 0, s, z, 1.0f / d->cfg.scale_factor,
                     d->f("post_quant_conv.weight"), d->f("post_quant_conv.bias"), d->f("decoder.conv_in.weight"),
                     d->f("decoder.conv_in.bias"), X, res, res, T);
  D_HIP(hipGetLastError());
  D_TRY(resblock(c, X, X2, B, res, T, T, "decoder.mid.block_1"));
  D_TRY(attnblock(c, X, B, res, T, "decoder.mid.attn_1"));
  D_TRY(resblock(c, X, X2, B, res, T, T, "decoder.mid.block_2"));
  int cin = T;
  const bf16* xb = nullptr;   // bf16(X) from the epilogue that produced X, when the next block's nin needs it
  for (int lvl = d->nlev - 1; lvl >= 0; --lvl) {
    const int cout = d->cfg.ch * d->cfg.ch_mult[lvl];
    for (int b = 0; b <= d->cfg.num_res_blocks; ++b) {
      // the level's last block also stores bf16 of its output into H: the upsample conv's source (H is free
      // once norm2 has consumed conv1's output)
      bf16* cp = (b == d->cfg.num_res_blocks && lvl != 0) ? w.H : nullptr;
      D_TRY(resblock(c, X, X2, B, res, cin, cout, "decoder.up." + std::to_string(lvl) + ".block." + std::to_string(b),
                     cin != cout ? xb : nullptr, cp));
      xb = nullptr;
      cin = cout;
    }
    if (lvl != 0) {  // nearest x2 upsample folded into the conv's source addressing (35-50)
      res *= 2;
      const int next = d->cfg.ch * d->cfg.ch_mult[lvl - 1];
      bf16* cp = next != cin ? w.XB : nullptr;   // the next level's first block changes width: its nin input
      D_TRY(conv3(c, w.H, B, res, cin, cin, "decoder.up." + std::to_string(lvl) + ".upsample.conv", pdm::EPI_F32,
                  cp, X2, 0, 1, true));
      xb = cp;
      float* t = X;
      X = X2;
      X2 = t;
    }
  }
  D_TRY(groupnorm<float>(c, X, B, res * res, cin, "decoder.norm_out", w.G, true));
  {
    const long long npix = (long long)B * res * res;
    const bf16* cw = d->w("decoder.conv_out.weight");
    const float* cb = d->f("decoder.conv_out.bias");
    if (cin == 128 && res % 64 == 0)
      hipLaunchKernelGGL(pdm::conv_out_mfma_kernel<128>, dim3(res / 2, B), dim3(256), 0, s, w.G, res, res, cw, cb, img,
                         d->cfg.out_ch);
    else if (cin == 64 && res % 64 == 0)
      hipLaunchKernelGGL(pdm::conv_out_mfma_kernel<64>, dim3(res / 2, B), dim3(256), 0, s, w.G, res, res, cw, cb, img,
                         d->cfg.out_ch);
    else
      hipLaunchKernelGGL(pdm::conv_out_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 9 * cin * 16, s, w.G,
                         B, res, res, cin, cw, cb, img, d->cfg.out_ch);
  }
  D_HIP(hipGetLastError());
  return PDM_OK;
}

}  // extern "C"

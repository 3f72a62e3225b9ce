// Memory-bound kernels around the U-ViT GEMMs (gfx950): LayerNorm, token assembly, the decoder_pred head
// with unpatchify, and the final-conv + CFG + solver-stage epilogue.
#include "pdm_common.h"
#include "pdm_kernels.h"

namespace pdm {

namespace {

// ------------------------------------------------------------------------------------------------
// LayerNorm (nn.LayerNorm, eps 1e-5: libs/uvit.py:100,103,180): one wave per row, float4 loads kept in
// registers (two-pass mean / variance like torch), bf16 output for the next GEMM.
constexpr int LN_MAXV = 8;  // float4 per lane -> D <= 2048

template <int NV>
__global__ __launch_bounds__(256) void layernorm_kernel(LayerNormArgs p) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + wave;
  if (r >= p.rows) return;
  const int src = (r / p.rows_per_group) * p.group_stride + p.row_offset + (r % p.rows_per_group);
  const int nv = p.D >> 2;
  f32x4 v[NV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int idx = lane + i * 64;
    if (idx < nv) {
      if (p.xb) {   // bf16 residual stream
        const bf16x4 b = reinterpret_cast<const bf16x4*>(p.xb + (size_t)src * p.ldx)[idx];
        v[i] = f32x4{(float)b[0], (float)b[1], (float)b[2], (float)b[3]};
      } else {
        v[i] = reinterpret_cast<const f32x4*>(p.x + (size_t)src * p.ldx)[idx];
      }
      s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
    }
  }
  const float mean = wave_sum(s) / (float)p.D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int idx = lane + i * 64;
    if (idx < nv) {
      const f32x4 d = v[i] - mean;
      q += (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
    }
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)p.D + p.eps);
  const f32x4* gm = reinterpret_cast<const f32x4*>(p.gamma);
  const f32x4* bt = reinterpret_cast<const f32x4*>(p.beta);
  bf16x4* y = reinterpret_cast<bf16x4*>(p.y + (size_t)r * p.ldy);
  const f32x4* ad = nullptr;
  const bf16x4* adb = nullptr;
  if (p.add || p.addb) {
    const int arow = (r / p.rows_per_group) * p.add_group_stride + p.add_row_offset + (r % p.rows_per_group);
    if (p.addb) adb = reinterpret_cast<const bf16x4*>(p.addb + (size_t)arow * p.add_ld);
    else ad = reinterpret_cast<const f32x4*>(p.add + (size_t)arow * p.add_ld);
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int idx = lane + i * 64;
    if (idx < nv) {
      f32x4 o = (v[i] - mean) * rstd * gm[idx] + bt[idx];
      if (ad) o += ad[idx];
      if (adb) {
        const bf16x4 b = adb[idx];
        o += f32x4{(float)b[0], (float)b[1], (float)b[2], (float)b[3]};
      }
      y[idx] = to_bf16x4(o[0], o[1], o[2], o[3]);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// LayerNorm row partials for the fused LayerNorm (see GemmArgs): one wave per row; float4 chunk i of the row
// covers columns 256 i .. 256 i + 255, i.e. exactly one partial group, so each group is two wave sums.
template <int NV>
__global__ __launch_bounds__(256) void rowstats_kernel(const float* x, int ldx, int rows, int D, bf16* xb, int ldb,
                                                       float* stats, int stats_ld, unsigned char* xq, int ldq,
                                                       unsigned* xs, int xs_ld, int center) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + wave;
  if (r >= rows) return;
  const f32x4* xr = reinterpret_cast<const f32x4*>(x + (size_t)r * ldx);
  const int nv = D >> 2;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int idx = lane + i * 64;
    if (i * 64 >= nv) break;
    const bool ok = idx < nv;
    const f32x4 v = ok ? xr[idx] : f32x4{0.f, 0.f, 0.f, 0.f};
    if (ok && xb) *reinterpret_cast<bf16x4*>(xb + (size_t)r * ldb + 4 * idx) = to_bf16x4(v[0], v[1], v[2], v[3]);
    const float s = wave_sum((v[0] + v[1]) + (v[2] + v[3]));
    const float mu = s / (float)min(256, D - 256 * i);
    const f32x4 d = v - mu;
    if (xq) {   // MXFP8 copy (group-centred: GemmArgs::mx_center): 8 consecutive lanes hold one 32-column block
      unsigned e8;
      const unsigned q = mx_quant4(center ? d : v, &e8);
      if (ok) {
        *reinterpret_cast<unsigned*>(xq + (size_t)r * ldq + 4 * idx) = q;
        if ((lane & 7) == 0)
          reinterpret_cast<unsigned char*>(xs)[((size_t)(idx >> 5) * xs_ld + r) * 4 + ((idx >> 3) & 3)] = (unsigned char)e8;
      }
    }
    const float q = wave_sum(ok ? (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]) : 0.f);
    if (lane == 0) *reinterpret_cast<float2*>(stats + ((size_t)r * stats_ld + i) * 2) = make_float2(s, q);
  }
}

// LayerNorm row partials of bf16 rows (EPI_RES outputs behind the 128-tile GEMM): one wave per row, lane l holds
// columns 4 (l + 64 i) .. +3, so chunk i is again exactly one 256-column group
__global__ __launch_bounds__(256) void rowstats_bf16_kernel(const bf16* x, int ldx, int rows, int D, float* stats,
                                                            int stats_ld) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + wave;
  if (r >= rows) return;
  const int nv = D >> 2;
  for (int i = 0; i * 64 < nv; ++i) {
    const int idx = lane + i * 64;
    const bool ok = idx < nv;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (ok) {
      const bf16x4 b = *reinterpret_cast<const bf16x4*>(x + (size_t)r * ldx + 4 * idx);
      v = f32x4{(float)b[0], (float)b[1], (float)b[2], (float)b[3]};
    }
    const float s = wave_sum((v[0] + v[1]) + (v[2] + v[3]));
    const float mu = s / (float)min(256, D - 256 * i);
    const f32x4 d = v - mu;
    const float q = wave_sum(ok ? (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]) : 0.f);
    if (lane == 0) *reinterpret_cast<float2*>(stats + ((size_t)r * stats_ld + i) * 2) = make_float2(s, q);
  }
}

// ------------------------------------------------------------------------------------------------
// Token assembly (libs/uvit.py:201-212; libs/uvit_t2i.py:382-409): block (x = 0) writes the extra
// tokens of one sample, blocks x >= 1 write 16 patch tokens each: PatchEmbed conv (k = s = p, K order
// (C, p1, p2): libs/uvit.py:129) + bias + pos_embed, fp32.
constexpr int ASM_TOK = 16;
constexpr int ASM_MAXK = 64;

template <int K>
__device__ __forceinline__ void assemble_patches(const AssembleArgs& p, float* out, const float (*patch)[ASM_MAXK],
                                                 int i0, int ntok) {
  const int D = p.D;
  for (int d = threadIdx.x; d < D; d += 256) {
    float w[K];
    const float* wr = p.patch_w + (size_t)d * K;
#pragma unroll
    for (int k = 0; k < K; ++k) w[k] = wr[k];
    const float bias = p.patch_b[d];
    for (int tk = 0; tk < ntok; ++tk) {
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) acc = fmaf(w[k], patch[tk][k], acc);
      const int row = p.row0_patch + i0 + tk;
      out[(size_t)row * p.ld_out + d] = acc + bias + p.pos[(size_t)row * D + d];
    }
  }
}

__global__ __launch_bounds__(256) void assemble_kernel(AssembleArgs p) {
  const int b = blockIdx.y;
  const int D = p.D;
  float* out = p.out + (size_t)b * p.L_total * p.ld_out;
  if (blockIdx.x == 0) {
    for (int d = threadIdx.x; d < D; d += 256) {
      if (p.time_row >= 0) {
        float v;
        if (p.time_emb) {
          v = p.time_emb[(size_t)b * D + d];
        } else {
          // timestep_embedding, libs/uvit.py:20-38 (fp32, cos half first, zero pad for odd D)
          const int half = D >> 1;
          if (d < 2 * half) {
            const int i = d < half ? d : d - half;
            const float f = expf((-9.210340371976184f * (float)i) / (float)half);
            const float a = p.t[b] * f;
            v = d < half ? cosf(a) : sinf(a);
          } else {
            v = 0.f;
          }
        }
        out[(size_t)p.time_row * p.ld_out + d] = v + p.pos[(size_t)p.time_row * D + d];
      }
      if (p.label_row >= 0) {
        const int64_t y = p.y[b];
        out[(size_t)p.label_row * p.ld_out + d] = p.label_emb[(size_t)y * D + d] + p.pos[(size_t)p.label_row * D + d];
      }
      if (p.ctx_row >= 0) {
        for (int i = 0; i < p.n_ctx; ++i) {
          const int row = p.ctx_row + i;
          out[(size_t)row * p.ld_out + d] = p.ctx_tokens[((size_t)b * p.n_ctx + i) * D + d] + p.pos[(size_t)row * D + d];
        }
      }
    }
    return;
  }
  __shared__ float patch[ASM_TOK][ASM_MAXK];
  const int wp_n = p.Wimg / p.p;
  const int n_patch = (p.Himg / p.p) * wp_n;
  const int K = p.C * p.p * p.p;
  const int i0 = (blockIdx.x - 1) * ASM_TOK;
  const float* img = p.img + (size_t)b * p.C * p.Himg * p.Wimg;
  for (int e = threadIdx.x; e < ASM_TOK * K; e += 256) {
    const int tk = e / K, k = e % K;
    const int i = i0 + tk;
    float v = 0.f;
    if (i < n_patch) {
      const int c = k / (p.p * p.p), p1 = (k / p.p) % p.p, p2 = k % p.p;
      const int hp = i / wp_n, wq = i % wp_n;
      v = img[((size_t)c * p.Himg + hp * p.p + p1) * p.Wimg + wq * p.p + p2];
    }
    patch[tk][k] = v;
  }
  __syncthreads();
  const int ntok = min(ASM_TOK, n_patch - i0);
  switch (K) {  // C * p * p of the configs: 12 (CIFAR), 16 (L/2, H/2, t2i image), 32 (t2i mask), 64 (H/4)
    case 12: assemble_patches<12>(p, out, patch, i0, ntok); break;
    case 16: assemble_patches<16>(p, out, patch, i0, ntok); break;
    case 32: assemble_patches<32>(p, out, patch, i0, ntok); break;
    case 64: assemble_patches<64>(p, out, patch, i0, ntok); break;
    default:
      for (int d = threadIdx.x; d < D; d += 256) {
        const float* wr = p.patch_w + (size_t)d * K;
        for (int tk = 0; tk < ntok; ++tk) {
          float acc = 0.f;
          for (int k = 0; k < K; ++k) acc = fmaf(wr[k], patch[tk][k], acc);
          const int row = p.row0_patch + i0 + tk;
          out[(size_t)row * p.ld_out + d] = acc + p.patch_b[d] + p.pos[(size_t)row * D + d];
        }
      }
  }
}

// ------------------------------------------------------------------------------------------------
// decoder_pred head (N = p*p*C <= 64 outputs) + unpatchify scatter.  One wave = 16 tokens, MFMA
// 16x16x32 with the weight as the A operand (lane owns 4 consecutive output columns of one token).
__global__ __launch_bounds__(256) void head_kernel(HeadArgs p) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int hp_n = p.Himg / p.p, wp_n = p.Wimg / p.p;
  const int N = hp_n * wp_n;
  const int rows = p.B * N;
  const int tok0 = (blockIdx.x * 4 + wave) * 16;
  if (tok0 >= rows) return;
  const int g = lane >> 4, col = lane & 15;
  int m = tok0 + col;
  const int mc0 = m < rows ? m : rows - 1;
  const int mc = (mc0 / N) * p.in_group_stride + p.in_row_offset + mc0 % N;
  const int NT = p.P_pad >> 4;
  f32x4 acc[4] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f},
                  f32x4{0.f, 0.f, 0.f, 0.f}};
  for (int k0 = 0; k0 < p.D; k0 += 32) {
    const int kk = k0 + g * 8;
    bf16x8 af = bf16x8{};
    if (kk < p.D) af = *reinterpret_cast<const bf16x8*>(p.x + (size_t)mc * p.ldx + kk);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      if (nt < NT) {
        bf16x8 wf = bf16x8{};
        if (kk < p.D) wf = *reinterpret_cast<const bf16x8*>(p.W + (size_t)(nt * 16 + col) * p.D + kk);
        acc[nt] = mfma16x16x32(wf, af, acc[nt]);
      }
    }
  }
  if (m >= rows) return;
  const int b = m / N, i = m % N;
  const int hp = i / wp_n, wq = i % wp_n;
  float* out = p.out + (size_t)b * p.C * p.Himg * p.Wimg;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    if (nt < NT) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = nt * 16 + g * 4 + r;
        if (n < p.P) {
          const int c = n % p.C, p2 = (n / p.C) % p.p, p1 = n / (p.C * p.p);
          float v = acc[nt][r] + p.bias[n];
          if (p.act_tanh) v = tanhf(v);
          out[((size_t)c * p.Himg + hp * p.p + p1) * p.Wimg + wq * p.p + p2] = v;
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// final_layer conv3x3 (libs/uvit.py:183,229) + CFG (eval_ldm_discrete.py:77) + solver stage.
__device__ __forceinline__ float conv3x3_at(const float* img, const float* w, const float* bias, int C, int H, int W,
                                            int c, int y, int x) {
  float acc = bias[c];
  for (int ci = 0; ci < C; ++ci) {
    const float* ip = img + (size_t)ci * H * W;
    const float* wp = w + ((size_t)c * C + ci) * 9;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int yy = y + ky - 1;
      if (yy < 0 || yy >= H) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int xx = x + kx - 1;
        if (xx < 0 || xx >= W) continue;
        acc = fmaf(wp[ky * 3 + kx], ip[(size_t)yy * W + xx], acc);
      }
    }
  }
  return acc;
}

__global__ __launch_bounds__(256) void epilogue_kernel(EpilogueArgs p) {
  const long long per = (long long)p.C * p.Himg * p.Wimg;
  const long long n = per * p.B;
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    const int b = (int)(e / per);
    const int r = (int)(e % per);
    const int c = r / (p.Himg * p.Wimg), yx = r % (p.Himg * p.Wimg);
    const int y = yx / p.Wimg, x = yx % p.Wimg;
    float v;
    if (p.w) v = conv3x3_at(p.pre + (size_t)b * per, p.w, p.bias, p.C, p.Himg, p.Wimg, c, y, x);
    else v = p.pre[(size_t)b * per + r];
    if (p.act_tanh) v = tanhf(v);  // libs/uvit_t2i.py:513 applies tanh per call, before the CFG combine
    if (p.has_uncond) {
      float u;
      if (p.w) u = conv3x3_at(p.pre + (size_t)(b + p.B) * per, p.w, p.bias, p.C, p.Himg, p.Wimg, c, y, x);
      else u = p.pre[(size_t)(b + p.B) * per + r];
      if (p.act_tanh) u = tanhf(u);
      v = v + p.cfg_scale * (v - u);
    }
    float m = v;
    if (p.xin) m = p.ax * p.xin[e] + p.ae * v;
    else m = p.ae * v;
    if (p.m_out) p.m_out[e] = m;
    if (p.x_out) {
      float acc = p.cm * m;
      for (int i = 0; i < p.n_terms; ++i) acc += p.c[i] * p.T[i][e];
      p.x_out[e] = acc;
      if (p.x_out2) p.x_out2[e] = acc;
      if (p.x_out3) p.x_out3[e] = acc;
    }
  }
}

struct LinArgs {
  const float* T[8];
  float c[8];
};

__global__ __launch_bounds__(256) void lincomb_kernel(float* out, int n_terms, LinArgs a, long long n) {
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    float acc = 0.f;
    for (int i = 0; i < n_terms; ++i) acc += a.c[i] * a.T[i][e];
    out[e] = acc;
  }
}

// one wave per row (4 rows per block): the row's D floats as 16-byte chunks when rows and pointers allow, else
// scalar; optionally a second, narrow row with the same row mapping (the row's LayerNorm partials)
__global__ __launch_bounds__(256) void rowcopy_kernel(float* dst, int ldd, const float* src, int lds, int rows, int D,
                                                     int rpg, int dgs, int sgs, float* dst2, int ldd2,
                                                     const float* src2, int lds2, int D2) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= rows) return;
  const int grp = r / rpg, k = r % rpg;
  const size_t ds = (size_t)grp * dgs + k, ss = (size_t)grp * sgs + k;
  const float* sr = src + ss * lds;
  float* dr = dst + ds * ldd;
  if (((D | ldd | lds) & 3) == 0 && (((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    const f32x4* s4 = reinterpret_cast<const f32x4*>(sr);
    f32x4* d4 = reinterpret_cast<f32x4*>(dr);
    for (int j = lane; j < (D >> 2); j += 64) d4[j] = s4[j];
  } else {
    for (int j = lane; j < D; j += 64) dr[j] = sr[j];
  }
  if (dst2)
    for (int j = lane; j < D2; j += 64) dst2[ds * ldd2 + j] = src2[ss * lds2 + j];
}

// fp32 -> bf16 (round to nearest even).  Eight elements per thread when x and y are 16-B aligned: two
// 16-byte loads and one 16-byte store (the scalar 4-B load / 2-B store form ran at ~45 % of HBM bandwidth);
// the scalar loop covers the n % 8 tail and unaligned views.
__global__ __launch_bounds__(256) void cast_bf16_kernel(const float* x, bf16* y, long long n) {
  const long long stride = (long long)gridDim.x * 256;
  long long done = 0;
  if ((((uintptr_t)x | (uintptr_t)y) & 15) == 0) {
    const long long n8 = n >> 3;
    for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n8; e += stride) {
      const f32x4 a = reinterpret_cast<const f32x4*>(x)[2 * e], b = reinterpret_cast<const f32x4*>(x)[2 * e + 1];
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) { o[j] = (bf16)a[j]; o[4 + j] = (bf16)b[j]; }
      reinterpret_cast<bf16x8*>(y)[e] = o;
    }
    done = n8 << 3;
  }
  for (long long e = done + blockIdx.x * 256ll + threadIdx.x; e < n; e += stride) y[e] = (bf16)x[e];
}

// ------------------------------------------------------------------------------------------------
// MXFP8 quantisation of rows (pdm_mx_quantize; in the fp8 forward: attention output -> attn.proj operand), tiled as
// 16 rows x 128 columns per block, 16 lanes per row with 8 consecutive columns each: the 4 lanes of a 32-column block
// reduce its amax with two xor-shuffles (mx_quant8: the quantiser of the MXFP8-emitting GEMM epilogues, bit for bit),
// then a row's four E8M0 bytes of its 128-column group are gathered into its first lane and stored as ONE dword -- the
// 16 rows' dwords of a group are consecutive in the [K/128][s_ld] scale layout.  (Round 4's one-thread-per-8-columns
// form stored one scattered byte per 32-column block: 15.0 us per H/4 call at 50 rows.)  Blocks past K get scale byte
// 0, the zero padding of a partial last group.
template <typename T>
__global__ __launch_bounds__(256) void mxq_tiled_kernel(const T* x, int ldx, int rows, int K, unsigned char* q,
                                                        int ldq, unsigned* s, int s_ld) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 16 + (threadIdx.x >> 4);
  const int c = blockIdx.y * 128 + (threadIdx.x & 15) * 8;
  const bool ok = r < rows && c < K;
  float f[8];
  if (ok) {
    const T* p = x + (size_t)r * ldx + c;
    if constexpr (sizeof(T) == 4) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { f[j] = a[j]; f[4 + j] = b[j]; }
    } else {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = (float)v[j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = 0.f;
  }
  unsigned e8;
  const uint2 w = mx_quant8(f, &e8);
  if (ok) *reinterpret_cast<uint2*>(q + (size_t)r * ldq + c) = w;
  const int base = lane & ~15;
  const int g0 = blockIdx.y * 128;
  unsigned dw = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const unsigned eb = (unsigned)__shfl((int)e8, base + 4 * b, 64);
    dw |= (g0 + 32 * b < K ? eb : 0u) << (8 * b);
  }
  if ((threadIdx.x & 15) == 0 && r < rows) s[(size_t)blockIdx.y * s_ld + r] = dw;
}

inline int grid_for(long long n) {
  long long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

const char* layernorm_check(const LayerNormArgs& p) {
  if (p.rows <= 0 || p.D <= 0) return "layernorm: rows and D must be positive";
  if (p.D % 4 || p.D > 4 * 64 * LN_MAXV) return "layernorm: D must be a multiple of 4 and <= 2048";
  if (p.ldx % 4 || p.ldy % 4) return "layernorm: row strides must be multiples of 4";
  if (p.rows_per_group <= 0) return "layernorm: rows_per_group must be positive";
  if ((!p.x && !p.xb) || !p.gamma || !p.beta || !p.y) return "layernorm: null pointer";
  return nullptr;
}

hipError_t layernorm_launch(const LayerNormArgs& p, hipStream_t stream) {
  const dim3 grid((p.rows + 3) / 4), block(256);
  switch ((p.D / 4 + 63) / 64) {
    case 1: hipLaunchKernelGGL(layernorm_kernel<1>, grid, block, 0, stream, p); break;
    case 2: hipLaunchKernelGGL(layernorm_kernel<2>, grid, block, 0, stream, p); break;
    case 3: hipLaunchKernelGGL(layernorm_kernel<3>, grid, block, 0, stream, p); break;
    case 4: hipLaunchKernelGGL(layernorm_kernel<4>, grid, block, 0, stream, p); break;
    case 5: hipLaunchKernelGGL(layernorm_kernel<5>, grid, block, 0, stream, p); break;
    case 6: hipLaunchKernelGGL(layernorm_kernel<6>, grid, block, 0, stream, p); break;
    default: hipLaunchKernelGGL(layernorm_kernel<8>, grid, block, 0, stream, p); break;
  }
  return hipGetLastError();
}

hipError_t rowstats_launch(const float* x, int ldx, int rows, int D, bf16* xb, int ldb, float* stats, int stats_ld,
                           hipStream_t stream, unsigned char* xq, int ldq, unsigned* xs, int xs_ld, int center) {
  if (!x || !stats || rows <= 0 || D <= 0 || D % 4 || D > 2048 || stats_ld < (D + 255) / 256 || ldx % 4 ||
      (xb && ldb % 4) || (xq && (D % 32 || ldq % 4 || !xs || xs_ld < rows)))
    return hipErrorInvalidValue;
  dim3 grid((rows + 3) / 4), block(256);
  hipLaunchKernelGGL(rowstats_kernel<8>, grid, block, 0, stream, x, ldx, rows, D, xb, ldb, stats, stats_ld, xq, ldq,
                     xs, xs_ld, center);
  return hipGetLastError();
}

hipError_t rowstats_bf16_launch(const bf16* x, int ldx, int rows, int D, float* stats, int stats_ld,
                                hipStream_t stream) {
  if (!x || !stats || rows <= 0 || D <= 0 || D % 4 || stats_ld < (D + 255) / 256 || ldx % 4)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(rowstats_bf16_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, x, ldx, rows, D, stats, stats_ld);
  return hipGetLastError();
}

const char* assemble_check(const AssembleArgs& p) {
  if (p.B <= 0 || p.D <= 0) return "assemble: B and D must be positive";
  if (p.C * p.p * p.p > ASM_MAXK) return "assemble: C*p*p must be <= 64";
  if (p.Himg % p.p || p.Wimg % p.p) return "assemble: image size must be divisible by the patch size";
  if (p.label_row >= 0 && (!p.y || !p.label_emb)) return "assemble: labels / label_emb missing";
  if (p.time_row >= 0 && !p.t && !p.time_emb) return "assemble: timesteps missing";
  if (p.ctx_row >= 0 && !p.ctx_tokens) return "assemble: context tokens missing";
  if (!p.img || !p.patch_w || !p.patch_b || !p.pos || !p.out) return "assemble: null pointer";
  return nullptr;
}

hipError_t assemble_launch(const AssembleArgs& p, hipStream_t stream) {
  const int n_patch = (p.Himg / p.p) * (p.Wimg / p.p);
  dim3 grid(1 + (n_patch + ASM_TOK - 1) / ASM_TOK, p.B);
  hipLaunchKernelGGL(assemble_kernel, grid, dim3(256), 0, stream, p);
  return hipGetLastError();
}

const char* head_check(const HeadArgs& p) {
  if (p.P > p.P_pad || p.P_pad % 16 || p.P_pad > 64) return "head: P_pad must be a multiple of 16, >= P and <= 64";
  if (p.D % 8 || p.ldx % 8) return "head: D and ldx must be multiples of 8";
  if (p.P != p.p * p.p * p.C) return "head: P must equal p*p*C";
  if (!p.x || !p.W || !p.bias || !p.out) return "head: null pointer";
  return nullptr;
}

hipError_t head_launch(const HeadArgs& p, hipStream_t stream) {
  const int rows = p.B * (p.Himg / p.p) * (p.Wimg / p.p);
  const int waves = (rows + 15) / 16;
  hipLaunchKernelGGL(head_kernel, dim3((waves + 3) / 4), dim3(256), 0, stream, p);
  return hipGetLastError();
}

const char* epilogue_check(const EpilogueArgs& p) {
  if (!p.pre) return "epilogue: null input";
  if (p.n_terms < 0 || p.n_terms > 6) return "epilogue: n_terms must be in [0, 6]";
  for (int i = 0; i < p.n_terms; ++i)
    if (!p.T[i]) return "epilogue: null term";
  if (p.w && !p.bias) return "epilogue: conv bias missing";
  return nullptr;
}

hipError_t epilogue_launch(const EpilogueArgs& p, hipStream_t stream) {
  const long long n = (long long)p.B * p.C * p.Himg * p.Wimg;
  hipLaunchKernelGGL(epilogue_kernel, dim3(grid_for(n)), dim3(256), 0, stream, p);
  return hipGetLastError();
}

hipError_t lincomb_launch(float* out, int n_terms, const float* const* T, const float* c, long long n,
                          hipStream_t stream) {
  LinArgs a;
  for (int i = 0; i < 8; ++i) {
    a.T[i] = i < n_terms ? T[i] : nullptr;
    a.c[i] = i < n_terms ? c[i] : 0.f;
  }
  hipLaunchKernelGGL(lincomb_kernel, dim3(grid_for(n)), dim3(256), 0, stream, out, n_terms, a, n);
  return hipGetLastError();
}

hipError_t cast_bf16_launch(const float* x, bf16* y, long long n, hipStream_t stream) {
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(grid_for((n + 7) / 8)), dim3(256), 0, stream, x, y, n);
  return hipGetLastError();
}

hipError_t mxq_launch(const void* x, int dtype, int ldx, int rows, int K, unsigned char* q, int ldq, unsigned* s,
                      int s_ld, hipStream_t stream) {
  const bool f32 = dtype == 0;
  if (!x || !q || !s || rows <= 0 || K <= 0 || K % 32 || ldx < K || ldq < K || ldq % 8 || s_ld < rows ||
      (dtype != 0 && dtype != 1) || (f32 ? ldx % 4 : ldx % 8) || ((uintptr_t)x & 15) || ((uintptr_t)q & 7) ||
      ((uintptr_t)s & 3))
    return hipErrorInvalidValue;
  const dim3 grid((unsigned)((rows + 15) / 16), (unsigned)((K + 127) / 128)), block(256);
  if (f32) hipLaunchKernelGGL(mxq_tiled_kernel<float>, grid, block, 0, stream, (const float*)x, ldx, rows, K, q, ldq, s, s_ld);
  else hipLaunchKernelGGL(mxq_tiled_kernel<bf16>, grid, block, 0, stream, (const bf16*)x, ldx, rows, K, q, ldq, s, s_ld);
  return hipGetLastError();
}

hipError_t rowcopy_launch(float* dst, int ldd, const float* src, int lds, int rows, int D, int rows_per_group,
                          int dst_group_stride, int src_group_stride, hipStream_t stream, float* dst2, int ldd2,
                          const float* src2, int lds2, int D2) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(rowcopy_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, dst, ldd, src, lds, rows, D,
                     rows_per_group, dst_group_stride, src_group_stride, dst2, ldd2, src2, lds2, D2);
  return hipGetLastError();
}

}  // namespace pdm

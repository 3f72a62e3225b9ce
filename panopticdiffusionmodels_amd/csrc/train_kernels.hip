// Backward-pass and optimizer kernels of the LSimple training step (sde.py:270-279,
// train_ldm_discrete.py:87-90,159-175) on gfx950.  The forward GEMMs and the dX GEMMs of the backward run on the
// forward's GEMM kernels (gemm.hip: dX = dY W is A = dY against the transposed weight copy W^T, K-contiguous
// like every forward weight); what the forward has no kernel for lives here:
//   * wgrad_kernel     dW = dY^T X: both operands are stored reduction-row-major ([M][N], [M][K]); 32-row stages
//                      land in LDS by LDS-DMA as [m][128 columns] images and are read as MFMA fragments with the
//                      hardware transposing read ds_read_b64_tr_b16, so neither activation is ever transposed
//                      in HBM.  The long reduction (M = tokens) is split over workgroups into fp32 partials.
//   * attn_bwd_kernel  softmax attention backward for one (sequence, head) per workgroup, Q K V dO resident in LDS
//                      (L <= 288) or two of them at a time (L <= 608: the t2i image / mask streams)
//   * LayerNorm / GELU / bias / embedding / final conv / decoder_pred backward, the LSimple loss, AdamW + EMA.
#include <algorithm>

#include "pdm_common.h"
#include "pdm_kernels.h"
#include "pdm_train.h"

namespace pdm {

namespace {

constexpr unsigned OOB = 0x80000000u;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, unsigned voff, PDM_LDS void* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, lds, 16, (int)voff, 0, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
  const unsigned n = bytes >= 0x7fffffffLL ? 0x7fffffffu : (unsigned)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)n, 0x00020000);
}

__device__ __forceinline__ s16x4 tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((PDM_LDS s16x4*)(p));
}

// two transposed 4-row reads -> one 16x16x32 operand fragment (k-slots 0..3 from r1's rows, 4..7 from r2's)
__device__ __forceinline__ bf16x8 tr_frag(const char* r1, const char* r2) {
  const bf16x4 lo = __builtin_bit_cast(bf16x4, tr16(r1));
  const bf16x4 hi = __builtin_bit_cast(bf16x4, tr16(r2));
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 4; ++j) { f[j] = lo[j]; f[4 + j] = hi[j]; }
  return f;
}

__device__ __forceinline__ int gather_row(int m, int rpg, int gs, int off) {
  return rpg > 0 ? (m / rpg) * gs + off + m % rpg : m;
}

int grid_for(long long n, int per_block = 256) {
  long long g = (n + per_block - 1) / per_block;
  return (int)(g < 1 ? 1 : (g > 65535 * 4 ? 65535 * 4 : g));
}

// ------------------------------------------------------------------------------------------------
// dW[n][k] (+)= sum_m A[m][n] B[m][k]
// Tile TN (n) x 128 (k), 4 waves, reduction stages of 32 rows, 3-slot LDS ring filled by LDS-DMA.
//   TN = 128: waves 2 x 2, 64 x 64 each (4 x 4 mfma_f32_16x16x32_bf16 accumulators)
//   TN = 256: waves 4 x 1, 64 x 128 each (8 x 4 accumulators: 12 fragments per 32 MFMAs instead of 8 per 16)
// A stage of an operand is 32 rows of TN (A) / 128 (B) columns; 1-KiB LDS-DMA pieces hold 1024 / (2 cols) rows.  The
// 16-byte chunk c of row r is stored at chunk c ^ swz(r) so that a transposed fragment read (per 32-lane half: rows
// g*8 + q, q < 4, of both 16-lane groups, two chunks each) touches all 64 banks once, for 256- and 512-byte rows alike.
__device__ __forceinline__ int wg_swz(int r) { return ((((r >> 3) & 1) << 2) | (r & 3)) << 1; }

template <int TN>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(WgradArgs p, int tiles_k) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TA = 32 * TN * 2, TB = 32 * 128 * 2, SB = TA + TB;
  constexpr int APW = TA / 1024 / 4, BPW = TB / 1024 / 4;     // LDS-DMA pieces per wave and stage
  constexpr int ARB = TN * 2, BRB = 256;                        // row bytes
  constexpr int NI = 4, KI = TN == 256 ? 8 : 4;                 // fragments per wave along n / k
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wn = TN == 256 ? wave : wave >> 1, wk = TN == 256 ? 0 : wave & 1;
  const int tn = blockIdx.x / tiles_k, tk = blockIdx.x - tn * tiles_k;
  const int n0 = tn * TN, k0 = tk * 128;
  const int ms = blockIdx.y * p.mchunk;
  const int me = min(p.M, ms + p.mchunk);
  const int nk = (me - ms + 31) >> 5;
  float* C = p.C + (long long)blockIdx.y * p.sC;

  const long long arows = p.a_rpg > 0 ? (long long)((p.M - 1) / p.a_rpg) * p.a_gs + p.a_off + p.a_rpg : p.M;
  const long long brows = p.b_rpg > 0 ? (long long)((p.M - 1) / p.b_rpg) * p.b_gs + p.b_off + p.b_rpg : p.M;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, arows * p.lda * 2);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, brows * p.ldb * 2);

  // per-lane row (within the stage) and column byte offset of this wave's pieces
  int ar[APW], br[BPW];
  unsigned ac[APW], bc[BPW];
#pragma unroll
  for (int i = 0; i < APW; ++i) {
    constexpr int rows_pp = 1024 / ARB, cpr = ARB / 16;
    ar[i] = (wave * APW + i) * rows_pp + lane / cpr;
    ac[i] = (unsigned)(n0 + (((lane % cpr) ^ wg_swz(ar[i])) * 8)) * 2u;
  }
#pragma unroll
  for (int i = 0; i < BPW; ++i) {
    br[i] = (wave * BPW + i) * 4 + (lane >> 4);
    bc[i] = (unsigned)(k0 + (((lane & 15) ^ wg_swz(br[i])) * 8)) * 2u;
  }
  auto issue = [&](int kt, int buf) {
    char* sa = smem + buf * SB;
    char* sb = sa + TA;
    const int mb = ms + kt * 32;
#pragma unroll
    for (int i = 0; i < APW; ++i) {
      const int m = mb + ar[i];
      const unsigned o = m < me ? (unsigned)gather_row(m, p.a_rpg, p.a_gs, p.a_off) * (unsigned)(p.lda * 2) + ac[i] : OOB;
      dma16(ra, o, (PDM_LDS void*)(sa + (wave * APW + i) * 1024));
    }
#pragma unroll
    for (int i = 0; i < BPW; ++i) {
      const int m = mb + br[i];
      const unsigned o = m < me ? (unsigned)gather_row(m, p.b_rpg, p.b_gs, p.b_off) * (unsigned)(p.ldb * 2) + bc[i] : OOB;
      dma16(rb, o, (PDM_LDS void*)(sb + (wave * BPW + i) * 1024));
    }
  };

  f32x4 acc[KI][NI];
#pragma unroll
  for (int i = 0; i < KI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // bias gradient: the k0 == 0 column of tiles also sums its A columns (wk == 0 waves: one copy per n)
  const bool do_bias = p.bias_out != nullptr && tk == 0 && wk == 0;
  f32x4 bacc[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) bacc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones8;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones8[j] = (bf16)1.0f;

  const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
  const int r1 = g * 8 + qq, r2 = r1 + 4;
  const int s1 = wg_swz(r1), s2 = wg_swz(r2);
  if (nk > 0) issue(0, 0);
  if (nk > 1) issue(1, 1);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(APW + BPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 2 < nk) issue(kt + 2, (kt + 2) % 3);
    const char* sa = smem + (kt % 3) * SB;
    const char* sb = sa + TA;
    bf16x8 af[NI], bfr[KI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int ca = ((wn * 64 + i * 16) >> 3) + (pp >> 1);
      af[i] = tr_frag(sa + r1 * ARB + ((ca ^ s1) << 4) + (pp & 1) * 8, sa + r2 * ARB + ((ca ^ s2) << 4) + (pp & 1) * 8);
    }
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      const int cb = ((wk * 64 + i * 16) >> 3) + (pp >> 1);
      bfr[i] = tr_frag(sb + r1 * BRB + ((cb ^ s1) << 4) + (pp & 1) * 8, sb + r2 * BRB + ((cb ^ s2) << 4) + (pp & 1) * 8);
    }
#pragma unroll
    for (int ki = 0; ki < KI; ++ki)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) acc[ki][ni] = mfma16x16x32(bfr[ki], af[ni], acc[ki][ni]);
    if (do_bias) {
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) bacc[ni] = mfma16x16x32(ones8, af[ni], bacc[ni]);
    }
  }
  // lane: column n = .. + (lane & 15), 4 consecutive k = .. + (lane >> 4) * 4
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const int n = n0 + wn * 64 + ni * 16 + i16;
    if (n >= p.N) continue;
    if (do_bias && g == 0) {   // every output row of the ones product holds the column sum
      float* bd = p.bias_out + (long long)blockIdx.y * p.sB + n;
      *bd = p.bias_acc ? *bd + bacc[ni][0] : bacc[ni][0];
    }
#pragma unroll
    for (int ki = 0; ki < KI; ++ki) {
      const int k = k0 + wk * 64 + ki * 16 + g * 4;
      if (k >= p.K) continue;
      f32x4* dst = reinterpret_cast<f32x4*>(C + (size_t)n * p.ldc + k);
      f32x4 v = acc[ki][ni];
      if (p.accumulate) v += *dst;
      *dst = v;
    }
  }
}

// dst[n * ldc + k] (+)= sum_s part[s][n][k]  (part compact [nparts][N][K]), K % 4 == 0.  Two such reductions in one
// launch (the dW partials and the fused bias-gradient partials of one split dW GEMM): blocks [0, nblk_a) take the
// first, the rest the second.
struct PartsJob {
  const float* part; int N, K; float* dst; int ldc, accumulate;
};
__global__ __launch_bounds__(256) void reduce_parts_kernel(PartsJob ja, PartsJob jb, int nparts, int nblk_a) {
  const bool second = (int)blockIdx.x >= nblk_a;
  const PartsJob& j = second ? jb : ja;
  const int bid = second ? blockIdx.x - nblk_a : blockIdx.x, nb = second ? gridDim.x - nblk_a : nblk_a;
  const float* part = j.part;
  const int N = j.N, K = j.K, ldc = j.ldc, accumulate = j.accumulate;
  float* dst = j.dst;
  const long long nk4 = (long long)N * (K >> 2);
  const long long NK = (long long)N * K;
  for (long long e = bid * 256ll + threadIdx.x; e < nk4; e += (long long)nb * 256) {
    const int n = (int)(e / (K >> 2)), k = (int)(e - (long long)n * (K >> 2)) * 4;
    f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < nparts; ++i) s += *reinterpret_cast<const f32x4*>(part + i * NK + (size_t)n * K + k);
    f32x4* d = reinterpret_cast<f32x4*>(dst + (size_t)n * ldc + k);
    if (accumulate) s += *d;
    *d = s;
  }
}

// column sums (bias / pos_embed / LayerNorm-parameter gradients): out[chunk][c] (+)= sum over the chunk's rows of
// x[gather(row)][c]; one thread per 4 columns, 16-B (fp32) / 8-B (bf16) row loads.  colsum_launch applies it in
// passes of <= 16 rows per chunk until one row is left, so every pass has parallelism across the rows.
template <typename T>
__global__ __launch_bounds__(256) void colsum4_kernel(const T* x, int ld, int rows, int n4, int rpg, int gs, int off,
                                                      int rpc, float* out, int ldo, int accumulate) {
  const int c4 = blockIdx.x * 256 + threadIdx.x;
  if (c4 >= n4) return;
  const int r0 = blockIdx.y * rpc, r1 = min(rows, r0 + rpc);
  f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int r = r0; r < r1; ++r) {
    const size_t o = (size_t)gather_row(r, rpg, gs, off) * ld + (size_t)c4 * 4;
    if constexpr (sizeof(T) == 4) {
      s += *reinterpret_cast<const f32x4*>(x + o);
    } else {
      const bf16x4 b = *reinterpret_cast<const bf16x4*>(x + o);
      s += f32x4{(float)b[0], (float)b[1], (float)b[2], (float)b[3]};
    }
  }
  f32x4* d = reinterpret_cast<f32x4*>(out + (size_t)blockIdx.y * ldo + (size_t)c4 * 4);
  if (accumulate) s += *d;
  *d = s;
}

// ------------------------------------------------------------------------------------------------
// LayerNorm backward (nn.LayerNorm, libs/uvit.py:100,103,180): one wave per row, mean / rstd recomputed from x
// (two-pass like the forward).  dx = rstd (g - mean(g) - xhat mean(g xhat)), g = dh * gamma; per-wave partial
// sums of dgamma = dh xhat and dbeta = dh go to part[wave][2][D].
template <int NV, typename DT>
__global__ __launch_bounds__(256) void ln_bwd_kernel(LnBwdArgs p, const DT* dh) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + wave, nw = gridDim.x * 4;
  const int nv = p.D >> 2;
  f32x4 dg[NV], db[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) { dg[i] = f32x4{0.f, 0.f, 0.f, 0.f}; db[i] = dg[i]; }
  const f32x4* gm = reinterpret_cast<const f32x4*>(p.gamma);
  for (int r = gw; r < p.rows; r += nw) {
    const int src = gather_row(r, p.rpg, p.gs, p.off);
    const f32x4* xr = reinterpret_cast<const f32x4*>(p.x + (size_t)src * p.ldx);
    f32x4 v[NV], d[NV];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = lane + i * 64;
      if (idx < nv) {
        v[i] = xr[idx];
        if constexpr (sizeof(DT) == 4) {
          d[i] = reinterpret_cast<const f32x4*>(dh + (size_t)r * p.lddh)[idx];
        } else {
          const bf16x4 b = reinterpret_cast<const bf16x4*>(dh + (size_t)r * p.lddh)[idx];
          d[i] = f32x4{(float)b[0], (float)b[1], (float)b[2], (float)b[3]};
        }
        s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
      }
    }
    const float mean = wave_sum(s) / (float)p.D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if (lane + i * 64 < nv) {
        const f32x4 c = v[i] - mean;
        q += (c[0] * c[0] + c[1] * c[1]) + (c[2] * c[2] + c[3] * c[3]);
      }
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)p.D + p.eps);
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = lane + i * 64;
      if (idx < nv) {
        v[i] = (v[i] - mean) * rstd;                // xhat
        const f32x4 gg = d[i] * gm[idx];
        sa += (gg[0] + gg[1]) + (gg[2] + gg[3]);
        const f32x4 gx = gg * v[i];
        sb += (gx[0] + gx[1]) + (gx[2] + gx[3]);
        dg[i] += d[i] * v[i];
        db[i] += d[i];
      }
    }
    const float a = wave_sum(sa) / (float)p.D, b = wave_sum(sb) / (float)p.D;
    f32x4* dxr = reinterpret_cast<f32x4*>(p.dx + (size_t)src * p.lddx);
    bf16x4* dxb = p.dxb ? reinterpret_cast<bf16x4*>(p.dxb + (size_t)src * p.lddx) : nullptr;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = lane + i * 64;
      if (idx < nv) {
        f32x4 o = (d[i] * gm[idx] - a - v[i] * b) * rstd;
        if (p.accumulate) o += dxr[idx];
        dxr[idx] = o;
        if (dxb) dxb[idx] = to_bf16x4(o[0], o[1], o[2], o[3]);
      }
    }
  }
  // the block's four waves' partials summed through LDS: one dgamma / dbeta partial row per block
  // (partials [gridDim.x][2][D]; fewer rows for the column-sum passes that follow)
  __shared__ f32x4 red[4][2][64];
  float* pg = p.part + (size_t)blockIdx.x * 2 * p.D;                      // partials [nblk][2][D]: dgamma
  float* pb = pg + p.D;                                                    //                         dbeta
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    red[wave][0][lane] = dg[i];
    red[wave][1][lane] = db[i];
    __syncthreads();
    if (wave < 2) {
      const f32x4 v = red[0][wave][lane] + red[1][wave][lane] + red[2][wave][lane] + red[3][wave][lane];
      const int idx = lane + i * 64;
      if (idx < nv) reinterpret_cast<f32x4*>(wave == 0 ? pg : pb)[idx] = v;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// exact-erf GELU (nn.GELU, libs/timm.py:102) and its derivative Phi(u) + u phi(u), 8 bf16 per thread
__device__ __forceinline__ float gelu_exact(float u) { return 0.5f * u * (1.0f + erff(u * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad(float u) {
  return 0.5f * (1.0f + erff(u * 0.70710678118654752f)) + u * 0.3989422804014327f * expf(-0.5f * u * u);
}

__global__ __launch_bounds__(256) void gelu_fwd_kernel(const bf16* u, bf16* g, long long n8) {
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n8; e += (long long)gridDim.x * 256) {
    const bf16x8 a = reinterpret_cast<const bf16x8*>(u)[e];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)gelu_exact((float)a[j]);
    reinterpret_cast<bf16x8*>(g)[e] = o;
  }
}

__global__ __launch_bounds__(256) void gelu_bwd_kernel(bf16* dg, const bf16* u, long long n8) {
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n8; e += (long long)gridDim.x * 256) {
    const bf16x8 a = reinterpret_cast<const bf16x8*>(u)[e];
    const bf16x8 d = reinterpret_cast<const bf16x8*>(dg)[e];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)((float)d[j] * gelu_grad((float)a[j]));
    reinterpret_cast<bf16x8*>(dg)[e] = o;
  }
}

// ------------------------------------------------------------------------------------------------
// Attention backward (libs/uvit.py:66-92 with S = Q K^T Dh^-1/2, P = softmax(S), O = P V), Dh = 64, L <= 288.
// One workgroup (16 waves) per (sequence b, head h); Q, K, V and dO of the head live in LDS as [Lp][64] bf16 images
// (128-B rows, 16-B chunk c of row r stored at c ^ (r & 7)), Lp = L rounded up to 32, rows >= L zero.
//   pass 0: lse2[q] = log2 sum_k exp2(S c) (c = Dh^-1/2 log2 e; +inf for padded queries) and
//           delta[q] = sum_d dO[q][d] O[q][d]
//   pass A: per 16-key tile (wave-owned): for every 32-query slice S, P = exp2(S c - lse2), dP = dO V^T,
//           dS = P (dP - delta), dV^T += dO^T P, dK^T += Q^T dS  (P / dS straight from the accumulators as the B
//           operand; the query k-slots of the transposed-read A operands permuted to match, as in attention.hip)
//   pass B: per 16-query tile (wave-owned): over 32-key slices S^T, P^T, dP^T, dS^T, dQ^T += K^T dS^T
// dK, dQ are scaled by Dh^-1/2.  Output: dqkv [b*L + i][3D] in the (3, H, Dh) column layout of the forward's qkv.
constexpr int AB_MAXL = 288;
constexpr int AB_THREADS = 1024;   // one workgroup per (image, head): 16 waves over its 16-key / 16-query tiles

// a head's rows in LDS: NCHR 16-B chunks per row (8: Dh 64; 12: Dh 72 padded to 96 for the 32-deep MFMA k-steps),
// chunks XOR-swizzled by the row within groups of 8 (and of 4 for chunks 8..11)
template <int NCHR>
__device__ __forceinline__ int ab_off(int row, int chunk) {
  if constexpr (NCHR == 8) return row * 128 + ((chunk ^ (row & 7)) << 4);
  else return row * (NCHR * 16) + ((chunk < 8 ? (chunk ^ (row & 7)) : 8 + ((chunk - 8) ^ (row & 3))) << 4);
}

template <int NCHR>
__device__ __forceinline__ bf16x8 ab_row(const char* img, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(img + ab_off<NCHR>(row, chunk));
}

// A-operand fragment of X^T (rows d = d0 + (lane & 15), k-slots = the 8 image rows r0 + 4g + {0..3} and
// r0 + 16 + 4g + {0..3}) by two transposed reads
template <int NCHR>
__device__ __forceinline__ bf16x8 ab_trT(const char* img, int r0, int d0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int ra = r0 + 4 * g + q, rb = ra + 16;
  const int c = (d0 >> 3) + (p >> 1);
  return tr_frag(img + ab_off<NCHR>(ra, c) + (p & 1) * 8, img + ab_off<NCHR>(rb, c) + (p & 1) * 8);
}

// LONG = 1 (288 < L <= 608: the t2i streams, 334 image / 590 mask tokens): the four images do not fit, so LDS holds
// two at a time -- Q and dO for pass 0 / pass A (a wave's own 16 keys' K and V rows sit in its registers; pass 0
// reads K rows from global / L2), then K and V for pass B (a wave's own query's Q and dO rows in registers).  The
// arithmetic (fragments, MFMA order, P / dS rounding) is the resident kernel's, so both give the same bits where
// both apply; 8 waves (2 per SIMD) leave room for the register-resident rows.
constexpr int AB_MAXL_LONG = 608;
constexpr int AB_MAXL_72 = 415;   // Dh 72: 2 x 416 rows x 192 B + lse / delta <= 160 KiB
constexpr int AB_THREADS_LONG = 512;

// DH = 72 (U-ViT-H): rows padded to 96 (12 chunks, zeros past 72): three 32-deep k-steps for S / dP, five 16-wide
// output tiles for dQ / dK / dV (d 72..79 of the last never stored); always the two-images-at-a-time form (L <= 415)
template <int LONG, int DH>
__global__ __launch_bounds__(LONG ? AB_THREADS_LONG : AB_THREADS, 1) void attn_bwd_kernel(AttnBwdArgs p) {
  static_assert(DH == 64 || (DH == 72 && LONG), "head dims 64 / 72 (72: two images at a time)");
  constexpr int NTH = LONG ? AB_THREADS_LONG : AB_THREADS;
  constexpr int NWV = NTH / 64;   // resident: 16 waves = four per SIMD (120 VGPRs each); LONG: 8
  constexpr int NCHR = DH == 64 ? 8 : 12, NCH = DH / 8, KK = NCHR / 4, NDT = (DH + 15) / 16, ROWB = NCHR * 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int L = p.L, Lp = (L + 31) & ~31;
  const int bh = blockIdx.x, b = bh / p.H, h = bh - b * p.H;
  const int D = p.H * DH;
  // resident: [Q | K | V | dO]; LONG: [Q | dO], later [K | V]
  char* Qs = smem;
  char* Ks = LONG ? smem : Qs + Lp * ROWB;
  char* Vs = LONG ? smem + Lp * ROWB : Ks + Lp * ROWB;
  char* Os = LONG ? smem + Lp * ROWB : Vs + Lp * ROWB;   // dO
  float* lse = reinterpret_cast<float*>(smem + (LONG ? 2 : 4) * Lp * ROWB);
  float* dlt = lse + Lp;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t row0 = (size_t)b * L;
  // global row r (clamped to the sequence) of image img: 0 Q, 1 K, 2 V, 3 dO; 16-B chunk c
  auto grow = [&](int img, int r, int c) -> bf16x8 {
    if (c >= NCH) return bf16x8{};   // Dh 72: the padding columns 72..95
    r = r < L ? r : L - 1;
    const bf16* src = img < 3 ? p.qkv + (row0 + r) * p.ldq + img * D + h * DH + c * 8
                              : p.dout + (row0 + r) * p.lddo + h * DH + c * 8;
    return *reinterpret_cast<const bf16x8*>(src);
  };
  // stage images (16-B chunks, rows >= L zero): slot i of LDS <- image imgs[i]
  auto stage = [&](int n, const int* imgs) {
    for (int e = tid; e < Lp * NCHR * n; e += NTH) {
      const int i = e / (Lp * NCHR), r = (e / NCHR) % Lp, c = e % NCHR;
      bf16x8 v = bf16x8{};
      if (r < L) v = grow(imgs[i], r, c);
      *reinterpret_cast<bf16x8*>(smem + i * Lp * ROWB + ab_off<NCHR>(r, c)) = v;
    }
  };
  if constexpr (LONG) {
    const int imgs[2] = {0, 3};
    stage(2, imgs);
  } else {
    const int imgs[4] = {0, 1, 2, 3};
    stage(4, imgs);
  }
  __syncthreads();
  const float cs = p.scale * 1.4426950408889634f;
  const int g = lane >> 4, col = lane & 15;

  // ---- pass 0: lse2 per query (16-query tiles), delta per query
  for (int qt = wave; qt * 16 < Lp; qt += NWV) {
    const int q0 = qt * 16;
    float m = -INFINITY, l = 0.f;
    for (int k0 = 0; k0 < Lp; k0 += 16) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)   // S^T[key][q]: A = K rows, B = Q rows
        s = mfma16x16x32(LONG ? grow(1, k0 + col, kk * 4 + g) : ab_row<NCHR>(Ks, k0 + col, kk * 4 + g),
                         ab_row<NCHR>(Qs, q0 + col, kk * 4 + g), s);
      // lane: q = q0 + col, keys k0 + 4g + j
      float tmax = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[j] = (k0 + 4 * g + j < L) ? s[j] * cs : -INFINITY;
        tmax = fmaxf(tmax, s[j]);
      }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float mn = fmaxf(m, tmax);
      float ts = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) ts += exp2f(s[j] - mn);
      ts += __shfl_xor(ts, 16, 64);
      ts += __shfl_xor(ts, 32, 64);
      l = l * exp2f(m - mn) + ts;
      m = mn;
    }
    if (g == 0) lse[q0 + col] = (q0 + col < L) ? m + log2f(l) : INFINITY;
  }
  for (int q = tid; q < Lp; q += NTH) {
    float d = 0.f;
    if (q < L) {
      const bf16* orow = p.o + (row0 + q) * p.ldo + h * DH;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const bf16x8 ov = *reinterpret_cast<const bf16x8*>(orow + c * 8);
        const bf16x8 dv = ab_row<NCHR>(Os, q, c);
#pragma unroll
        for (int j = 0; j < 8; ++j) d += (float)ov[j] * (float)dv[j];
      }
    }
    dlt[q] = d;
  }
  __syncthreads();

  // ---- pass A: dK, dV per 16-key tile
  for (int kt = wave; kt * 16 < L; kt += NWV) {
    const int k0 = kt * 16;
    f32x4 dv[NDT], dk[NDT];
#pragma unroll
    for (int i = 0; i < NDT; ++i) { dv[i] = f32x4{0.f, 0.f, 0.f, 0.f}; dk[i] = dv[i]; }
    bf16x8 kr[KK], vr[KK];   // LONG: the tile's K / V rows (B operands of every query slice)
    if constexpr (LONG) {
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        kr[kk] = grow(1, k0 + col, kk * 4 + g);
        vr[kk] = grow(2, k0 + col, kk * 4 + g);
      }
    }
    for (int q0 = 0; q0 < Lp; q0 += 32) {
      f32x4 s[2], dp[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {   // S[q][key] / dP[q][key]: A = Q / dO rows (q), B = K / V rows (key)
        s[hh] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp[hh] = s[hh];
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          s[hh] = mfma16x16x32(ab_row<NCHR>(Qs, q0 + hh * 16 + col, kk * 4 + g),
                               LONG ? kr[kk] : ab_row<NCHR>(Ks, k0 + col, kk * 4 + g), s[hh]);
          dp[hh] = mfma16x16x32(ab_row<NCHR>(Os, q0 + hh * 16 + col, kk * 4 + g),
                                LONG ? vr[kk] : ab_row<NCHR>(Vs, k0 + col, kk * 4 + g), dp[hh]);
        }
      }
      // lane: key k0 + col, queries q0 + hh*16 + 4g + j
      bf16x8 pf, sf;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int q = q0 + hh * 16 + 4 * g + j;
          const float pv = exp2f(s[hh][j] * cs - lse[q]);
          pf[hh * 4 + j] = (bf16)pv;
          sf[hh * 4 + j] = (bf16)(pv * (dp[hh][j] - dlt[q]));
        }
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        dv[dt] = mfma16x16x32(ab_trT<NCHR>(Os, q0, dt * 16, lane), pf, dv[dt]);
        dk[dt] = mfma16x16x32(ab_trT<NCHR>(Qs, q0, dt * 16, lane), sf, dk[dt]);
      }
    }
    // lane: key k0 + col, d = dt*16 + 4g + {0..3}
    const int key = k0 + col;
    if (key < L) {
      bf16* drow = p.dqkv + (row0 + key) * p.lddq + h * DH;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const int d = dt * 16 + 4 * g;
        if (d >= DH) break;
        *reinterpret_cast<bf16x4*>(drow + D + d) =
            to_bf16x4(dk[dt][0] * p.scale, dk[dt][1] * p.scale, dk[dt][2] * p.scale, dk[dt][3] * p.scale);
        *reinterpret_cast<bf16x4*>(drow + 2 * D + d) = to_bf16x4(dv[dt][0], dv[dt][1], dv[dt][2], dv[dt][3]);
      }
    }
  }
  if constexpr (LONG) {   // Q / dO -> K / V
    __syncthreads();
    const int imgs[2] = {1, 2};
    stage(2, imgs);
    __syncthreads();
  }

  // ---- pass B: dQ per 16-query tile
  for (int qt = wave; qt * 16 < L; qt += NWV) {
    const int q0 = qt * 16;
    const int q = q0 + col;
    const float lq = lse[q], dq_ = dlt[q];
    f32x4 dq[NDT];
#pragma unroll
    for (int i = 0; i < NDT; ++i) dq[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 qr[KK], orr[KK];   // LONG: the query's Q / dO rows
    if constexpr (LONG) {
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        qr[kk] = grow(0, q, kk * 4 + g);
        orr[kk] = grow(3, q, kk * 4 + g);
      }
    }
    for (int k0 = 0; k0 < Lp; k0 += 32) {
      f32x4 s[2], dp[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {   // S^T[key][q]: A = K / V rows (key), B = Q / dO rows (q)
        s[hh] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp[hh] = s[hh];
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          s[hh] = mfma16x16x32(ab_row<NCHR>(Ks, k0 + hh * 16 + col, kk * 4 + g), LONG ? qr[kk] : ab_row<NCHR>(Qs, q, kk * 4 + g),
                               s[hh]);
          dp[hh] = mfma16x16x32(ab_row<NCHR>(Vs, k0 + hh * 16 + col, kk * 4 + g),
                                LONG ? orr[kk] : ab_row<NCHR>(Os, q, kk * 4 + g), dp[hh]);
        }
      }
      // lane: q, keys k0 + hh*16 + 4g + j
      bf16x8 sf;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int key = k0 + hh * 16 + 4 * g + j;
          const float pv = key < L ? exp2f(s[hh][j] * cs - lq) : 0.f;
          sf[hh * 4 + j] = (bf16)(pv * (dp[hh][j] - dq_));
        }
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) dq[dt] = mfma16x16x32(ab_trT<NCHR>(Ks, k0, dt * 16, lane), sf, dq[dt]);
    }
    if (q < L) {
      bf16* drow = p.dqkv + (row0 + q) * p.lddq + h * DH;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const int d = dt * 16 + 4 * g;
        if (d >= DH) break;
        *reinterpret_cast<bf16x4*>(drow + d) =
            to_bf16x4(dq[dt][0] * p.scale, dq[dt][1] * p.scale, dq[dt][2] * p.scale, dq[dt][3] * p.scale);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// LSimple (sde.py:270-279 / train_ldm_discrete.py:87-90): loss[b] = mean_j (target - pred)^2 (mos), and the
// gradient of gscale * sum_b loss[b] w.r.t. pred: -2 gscale (target - pred) / per
// tanh_bwd: pred = tanh(u) (the t2i mask head, libs/uvit_t2i.py:513) and dpred is the gradient w.r.t. u
__global__ __launch_bounds__(256) void lsimple_kernel(const float* pred, const float* target, float* loss, float* dpred,
                                                      int per, float gscale, int tanh_bwd) {
  const int b = blockIdx.x;
  const float* pr = pred + (size_t)b * per;
  const float* tg = target + (size_t)b * per;
  float* dp = dpred + (size_t)b * per;
  const float k = -2.0f * gscale / (float)per;
  float s = 0.f;
  for (int i = threadIdx.x; i < per; i += 256) {
    const float y = pr[i], d = tg[i] - y;
    s += d * d;
    dp[i] = tanh_bwd ? k * d * (1.0f - y * y) : k * d;
  }
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) loss[b] = (red[0] + red[1] + red[2] + red[3]) / (float)per;
}

// final_layer conv3x3 (pad 1) backward: data gradient (the transposed conv) ...
__global__ __launch_bounds__(256) void conv_bwd_data_kernel(const float* dout, const float* w, float* din, int B, int C,
                                                            int H, int W) {
  const long long per = (long long)C * H * W, n = per * B;
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    const int b = (int)(e / per), r = (int)(e % per);
    const int ci = r / (H * W), y = (r / W) % H, x = r % W;
    float acc = 0.f;
    for (int co = 0; co < C; ++co) {
      const float* dp = dout + ((size_t)b * C + co) * H * W;
      const float* wp = w + ((size_t)co * C + ci) * 9;
      for (int ky = 0; ky < 3; ++ky) {
        const int yy = y + 1 - ky;
        if (yy < 0 || yy >= H) continue;
        for (int kx = 0; kx < 3; ++kx) {
          const int xx = x + 1 - kx;
          if (xx < 0 || xx >= W) continue;
          acc = fmaf(wp[ky * 3 + kx], dp[(size_t)yy * W + xx], acc);
        }
      }
    }
    din[e] = acc;
  }
}

// ... and weight / bias gradients: one workgroup per weight (co, ci, ky, kx), then one per bias co
__global__ __launch_bounds__(256) void conv_bwd_weight_kernel(const float* dout, const float* in, float* dw, float* db,
                                                              int B, int C, int H, int W) {
  const int o = blockIdx.x;
  const int nw = C * C * 9;
  float s = 0.f;
  const long long hw = (long long)H * W;
  if (o < nw) {
    const int co = o / (C * 9), ci = (o / 9) % C, ky = (o % 9) / 3, kx = o % 3;
    for (long long e = threadIdx.x; e < B * hw; e += 256) {
      const int b = (int)(e / hw), yx = (int)(e % hw), y = yx / W, x = yx % W;
      const int yy = y + ky - 1, xx = x + kx - 1;
      if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
      s += dout[((size_t)b * C + co) * hw + yx] * in[((size_t)b * C + ci) * hw + (size_t)yy * W + xx];
    }
  } else {
    const int co = o - nw;
    for (long long e = threadIdx.x; e < B * hw; e += 256) {
      const int b = (int)(e / hw), yx = (int)(e % hw);
      s += dout[((size_t)b * C + co) * hw + yx];
    }
  }
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t = (red[0] + red[1] + red[2] + red[3]);
    if (o < nw) dw[o] = t;
    else db[o - nw] = t;
  }
}

// decoder_pred + unpatchify backward (libs/uvit.py:182,225-228): per patch token (b, i) the P = p*p*C output
// gradients are gathered from dpre [B, C, H, W] in the (p1, p2, C) column order -> dtok bf16 [B*N][P_pad] (the
// weight-gradient operand, zero padded) and dx[token][d] = sum_j dtok[j] W[j][d] (fp32)
__global__ __launch_bounds__(256) void head_bwd_kernel(HeadBwdArgs p) {
  __shared__ float t[16][64];
  const int hp_n = p.Himg / p.p, wp_n = p.Wimg / p.p, N = hp_n * wp_n;
  const int tok0 = blockIdx.x * 16;
  const int ntok = min(16, p.B * N - tok0);
  for (int e = threadIdx.x; e < 16 * p.P_pad; e += 256) {
    const int tk = e / p.P_pad, n = e % p.P_pad;
    float v = 0.f;
    if (tk < ntok && n < p.P) {
      const int m = tok0 + tk, b = m / N, i = m % N, hp = i / wp_n, wq = i % wp_n;
      const int c = n % p.C, p2 = (n / p.C) % p.p, p1 = n / (p.C * p.p);
      v = p.dpre[(((size_t)b * p.C + c) * p.Himg + hp * p.p + p1) * p.Wimg + wq * p.p + p2];
    }
    t[tk][n] = v;
    if (tk < ntok) p.dtok[(size_t)(tok0 + tk) * p.P_pad + n] = (bf16)v;
  }
  __syncthreads();
  for (int d = threadIdx.x; d < p.D; d += 256) {
    for (int tk = 0; tk < ntok; ++tk) {
      float acc = 0.f;
      for (int n = 0; n < p.P; ++n) acc = fmaf(t[tk][n], p.W[(size_t)n * p.D + d], acc);
      p.dx[(size_t)(tok0 + tk) * p.D + d] = acc;
    }
  }
}

// patch vectors of the net input (PatchEmbed's conv as a GEMM operand): pv[b*N + i][k], k = (c, p1, p2), zero padded
__global__ __launch_bounds__(256) void patchify_kernel(const float* img, bf16* pv, int B, int C, int H, int W, int p,
                                                       int ldp) {
  const int wp_n = W / p, N = (H / p) * wp_n, K = C * p * p;
  const long long n = (long long)B * N * ldp;
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    const int m = (int)(e / ldp), k = (int)(e % ldp);
    float v = 0.f;
    if (k < K) {
      const int b = m / N, i = m % N, hp = i / wp_n, wq = i % wp_n;
      const int c = k / (p * p), p1 = (k / p) % p, p2 = k % p;
      v = img[(((size_t)b * C + c) * H + hp * p + p1) * W + wq * p + p2];
    }
    pv[e] = (bf16)v;
  }
}

// label_emb gradient: dlab[y[b]] += dx[b * L + row]  (atomics: a label may repeat in the batch)
__global__ __launch_bounds__(256) void label_scatter_kernel(const float* dx, int L, int row, int D, const int64_t* y,
                                                            float* dlab, int B) {
  const int b = blockIdx.x;
  const int64_t cls = y[b];
  for (int d = threadIdx.x; d < D; d += 256)
    atomicAdd(dlab + (size_t)cls * D + d, dx[((size_t)b * L + row) * D + d]);
}

// dx += add (fp32), dxb = bf16(dx)
// dst[gd(r)] (+)= src[gs(r)], dstb[gd(r)] = bf16(dst[gd(r)]) over `rows` rows of D floats; g(r) = (r / rpg) * gs + off +
// r % rpg (rpg 0: r).  The t2i mask-stream input cat(x, m): its image rows' gradient into x's, the injection's into
// the mask output's image rows, the mask head's into the mask rows.
__global__ __launch_bounds__(256) void rows_add_cast_kernel(float* dst, bf16* dstb, int drpg, int dgs, int doff,
                                                            const float* src, int srpg, int sgs, int soff, int rows,
                                                            int D, int acc) {
  const int d4 = D >> 2;
  const long long n = (long long)rows * d4;
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    const int r = (int)(e / d4), c = (int)(e % d4);
    const size_t rd = drpg > 0 ? (size_t)(r / drpg) * dgs + doff + r % drpg : (size_t)r;
    const size_t rs = srpg > 0 ? (size_t)(r / srpg) * sgs + soff + r % srpg : (size_t)r;
    f32x4 v = reinterpret_cast<const f32x4*>(src + rs * D)[c];
    f32x4* o = reinterpret_cast<f32x4*>(dst + rd * D) + c;
    if (acc) v += *o;
    *o = v;
    reinterpret_cast<bf16x4*>(dstb + rd * D)[c] = to_bf16x4(v[0], v[1], v[2], v[3]);
  }
}

__global__ __launch_bounds__(256) void add_cast_kernel(float* dx, const float* add, bf16* dxb, long long n4) {
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n4; e += (long long)gridDim.x * 256) {
    f32x4 v = reinterpret_cast<f32x4*>(dx)[e];
    if (add) v += reinterpret_cast<const f32x4*>(add)[e];
    reinterpret_cast<f32x4*>(dx)[e] = v;
    reinterpret_cast<bf16x4*>(dxb)[e] = to_bf16x4(v[0], v[1], v[2], v[3]);
  }
}

// W fp32 [N][K] -> W^T bf16 [K][N]: 64 x 64 tiles, 16-B row loads, the tile transposed through LDS, 8-B row stores
// (N, K multiples of 4)
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const float* w, bf16* wt, int N, int K) {
  __shared__ float t[64][65];
  const int n0 = blockIdx.y * 64, k0 = blockIdx.x * 64;
  const int c = (threadIdx.x & 15) * 4, r = threadIdx.x >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + r + 16 * j, k = k0 + c;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (n < N && k < K) v = *reinterpret_cast<const f32x4*>(w + (size_t)n * K + k);
#pragma unroll
    for (int q = 0; q < 4; ++q) t[c + q][r + 16 * j] = v[q];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = k0 + r + 16 * j, n = n0 + c;
    if (k < K && n < N) {
      const float* row = &t[r + 16 * j][c];
      *reinterpret_cast<bf16x4*>(wt + (size_t)k * N + n) = to_bf16x4(row[0], row[1], row[2], row[3]);
    }
  }
}

// torch.optim.AdamW (decoupled weight decay) + EMA (utils.py:339-345) + the bf16 working copy, over the flat
// parameter buffer.  p <- p (1 - lr wd);  m <- b1 m + (1 - b1) g;  v <- b2 v + (1 - b2) g^2;
// p <- p - (lr / bc1) m / (sqrt(v) / sqrt(bc2) + eps);  ema <- rate ema + (1 - rate) p;  pb <- bf16(p)
__global__ __launch_bounds__(256) void adamw_kernel(AdamWArgs a, long long n) {
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    const float g = a.g2 ? a.g[e] + a.g2[e] : a.g[e];
    float pv = a.p[e] * (1.0f - a.lr * a.wd);
    const float m = a.b1 * a.m[e] + (1.0f - a.b1) * g;
    const float v = a.b2 * a.v[e] + (1.0f - a.b2) * g * g;
    a.m[e] = m;
    a.v[e] = v;
    pv -= a.step_size * m / (sqrtf(v) * a.inv_sqrt_bc2 + a.eps);
    a.p[e] = pv;
    if (a.ema) a.ema[e] = a.ema_rate * a.ema[e] + (1.0f - a.ema_rate) * pv;
    if (a.pb) a.pb[e] = (bf16)pv;
  }
}

}  // namespace

// ---------------------------------------------------------------------------------------------------------------
const char* wgrad_check(const WgradArgs& p) {
  if (p.M <= 0 || p.N <= 0 || p.K <= 0) return "wgrad: M, N, K must be positive";
  if (p.K % 4 || p.ldc % 4) return "wgrad: K and ldc must be multiples of 4";
  if (p.bias_out && p.N % 4) return "wgrad: the fused bias gradient needs N % 4 == 0";
  if (p.lda % 8 || p.ldb % 8) return "wgrad: lda / ldb must be multiples of 8 (16-byte rows)";
  if (((uintptr_t)p.A | (uintptr_t)p.B) & 15 || ((uintptr_t)p.C & 15)) return "wgrad: operands must be 16-byte aligned";
  const long long arows = p.a_rpg > 0 ? (long long)((p.M - 1) / p.a_rpg) * p.a_gs + p.a_off + p.a_rpg : p.M;
  const long long brows = p.b_rpg > 0 ? (long long)((p.M - 1) / p.b_rpg) * p.b_gs + p.b_off + p.b_rpg : p.M;
  if (arows * p.lda * 2 >= 0x7fffffffLL || brows * p.ldb * 2 >= 0x7fffffffLL)
    return "wgrad: an operand spans >= 2 GiB (32-bit buffer offsets)";
  return nullptr;
}

int g_wgrad_tile = 0;   // 0 auto, 128 / 256 forced (pdm_set_wgrad_tile, A/B timing)

hipError_t wgrad_launch(const WgradArgs& args, float* part, size_t part_bytes, hipStream_t stream) {
  WgradArgs p = args;
  // the 256 x 128 tile wherever the n extent fills it (every U-ViT Linear), the 128 x 128 one for narrow outputs
  const int TN = g_wgrad_tile ? g_wgrad_tile : (p.N >= 256 ? 256 : 128);
  const int tiles_n = (p.N + TN - 1) / TN, tiles_k = (p.K + 127) / 128;
  const int tiles = tiles_n * tiles_k;
  // split the reduction so that >= ~1024 workgroups run (2 per CU is the residency), >= 512 rows each, and the
  // fp32 partials fit the scratch
  int split = (1024 + tiles - 1) / tiles;
  split = std::min(split, std::max(1, p.M / 512));
  const long long nk = (long long)p.N * p.K;
  const long long nb = p.bias_out ? p.N : 0;   // bias partials follow the dW partials
  if (!part) split = 1;
  else split = (int)std::min<long long>(split, (long long)(part_bytes / ((nk + nb) * 4)));
  if (split < 1) split = 1;
  int mchunk = ((p.M + split - 1) / split + 31) & ~31;
  split = (p.M + mchunk - 1) / mchunk;
  p.mchunk = mchunk;
  if (split > 1) {
    p.C = part;
    p.ldc = p.K;
    p.sC = nk;
    p.accumulate = 0;
    if (p.bias_out) {
      p.bias_out = part + (size_t)split * nk;
      p.sB = p.N;
      p.bias_acc = 0;
    }
  } else {
    p.sC = 0;
    p.sB = 0;
  }
  if (TN == 256)
    hipLaunchKernelGGL(wgrad_kernel<256>, dim3(tiles, split), dim3(256), 3 * (32 * 256 * 2 + 32 * 128 * 2), stream, p,
                       tiles_k);
  else
    hipLaunchKernelGGL(wgrad_kernel<128>, dim3(tiles, split), dim3(256), 3 * (32 * 128 * 2 * 2), stream, p, tiles_k);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || split == 1) return e;
  const PartsJob ja{part, p.N, p.K, args.C, args.ldc, args.accumulate};
  const PartsJob jb{p.bias_out, 1, p.N, args.bias_out, p.N, args.bias_acc};
  const int ga = (int)grid_for(nk / 4), gb = args.bias_out ? (int)grid_for(p.N / 4) : 0;
  hipLaunchKernelGGL(reduce_parts_kernel, dim3(ga + gb), dim3(256), 0, stream, ja, jb, split, ga);
  return hipGetLastError();
}

hipError_t colsum_launch(const void* x, int is_bf16, int ld, int rows, int ncols, int rpg, int gs, int off, float* dst,
                         int accumulate, float* part, size_t part_bytes, hipStream_t stream) {
  if (ncols % 4 || ld % 4 || rows <= 0) return hipErrorInvalidValue;
  const int n4 = ncols / 4;
  const size_t half = part_bytes / 2 / 4;   // floats per ping-pong half
  float* buf[2] = {part, part + half};
  const void* src = x;
  int cur = rows, pass = 0;
  for (;;) {
    int rpc = 16;
    int chunks = (cur + rpc - 1) / rpc;
    if (chunks > 1 && (size_t)chunks * ncols > half) {   // fewer, longer chunks when the partials would not fit
      chunks = (int)std::max<size_t>(1, half / ncols);
      rpc = (cur + chunks - 1) / chunks;
      chunks = (cur + rpc - 1) / rpc;
    }
    const bool last = chunks == 1;
    float* out = last ? dst : buf[pass & 1];
    dim3 grid((n4 + 255) / 256, chunks);
    if (pass == 0 && is_bf16)
      hipLaunchKernelGGL(colsum4_kernel<bf16>, grid, dim3(256), 0, stream, (const bf16*)src, ld, cur, n4, rpg, gs, off,
                         rpc, out, ncols, last ? accumulate : 0);
    else
      hipLaunchKernelGGL(colsum4_kernel<float>, grid, dim3(256), 0, stream, (const float*)src, pass == 0 ? ld : ncols,
                         cur, n4, pass == 0 ? rpg : 0, gs, off, rpc, out, ncols, last ? accumulate : 0);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess || last) return e;
    src = out;
    cur = chunks;
    ++pass;
  }
}

hipError_t ln_bwd_launch(const LnBwdArgs& args, const void* dh, int dh_bf16, float* dgamma, float* dbeta,
                         hipStream_t stream) {
  LnBwdArgs p = args;
  const int nv = p.D >> 2;
  const int NV = (nv + 63) / 64;
  // one wave per row, 4 per block; up to 1024 blocks (16 waves per CU) so row latency (two wave-sum chains per row)
  // overlaps across waves; each wave's dgamma / dbeta partials are summed by colsum_launch afterwards
  int nblk = std::min(1024, (p.rows + 3) / 4);
  // partials [2][4 nblk][D] + at least [2][D] for the column-sum passes must fit the scratch
  if (((size_t)nblk * 4 + 1) * 2 * p.D * 4 > p.part_bytes)
    nblk = (int)((p.part_bytes / ((size_t)2 * p.D * 4) - 1) / 4);
  if (nblk < 1 || p.D % 4 || NV > 8) return hipErrorInvalidValue;
#define PDM_LNB(N)                                                                                                 \
  case N:                                                                                                          \
    if (dh_bf16) hipLaunchKernelGGL((ln_bwd_kernel<N, bf16>), dim3(nblk), dim3(256), 0, stream, p, (const bf16*)dh); \
    else hipLaunchKernelGGL((ln_bwd_kernel<N, float>), dim3(nblk), dim3(256), 0, stream, p, (const float*)dh);     \
    break;
  switch (NV) {
    PDM_LNB(1) PDM_LNB(2) PDM_LNB(3) PDM_LNB(4) PDM_LNB(5) PDM_LNB(6) PDM_LNB(7) PDM_LNB(8)
  }
#undef PDM_LNB
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // partials [nblk][2][D] in the first part of the scratch; the column sums use the rest.  When dbeta follows
  // dgamma in the parameter buffer (the flat layout's norm.weight, norm.bias) one column-sum chain covers both.
  const int nw = nblk;
  float* rest = p.part + (size_t)2 * nw * p.D;
  const size_t rest_bytes = p.part_bytes - (size_t)2 * nw * p.D * 4;
  if (dbeta == dgamma + p.D)
    return colsum_launch(p.part, 0, 2 * p.D, nw, 2 * p.D, 0, 0, 0, dgamma, p.accumulate_params, rest, rest_bytes, stream);
  if ((e = colsum_launch(p.part, 0, 2 * p.D, nw, p.D, 0, 0, 0, dgamma, p.accumulate_params, rest, rest_bytes, stream)) !=
      hipSuccess)
    return e;
  return colsum_launch(p.part + p.D, 0, 2 * p.D, nw, p.D, 0, 0, 0, dbeta, p.accumulate_params, rest, rest_bytes, stream);
}

hipError_t gelu_fwd_launch(const bf16* u, bf16* g, long long n, hipStream_t stream) {
  if (n % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gelu_fwd_kernel, dim3(grid_for(n / 8)), dim3(256), 0, stream, u, g, n / 8);
  return hipGetLastError();
}

hipError_t gelu_bwd_launch(bf16* dg, const bf16* u, long long n, hipStream_t stream) {
  if (n % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(grid_for(n / 8)), dim3(256), 0, stream, dg, u, n / 8);
  return hipGetLastError();
}

const char* attn_bwd_check(const AttnBwdArgs& p) {
  if (p.Dh != 64 && p.Dh != 72) return "attention backward: head dim 64 or 72";
  if (p.L <= 0 || p.L > (p.Dh == 64 ? AB_MAXL_LONG : AB_MAXL_72))
    return "attention backward: 1 <= L <= 608 (head dim 64) / 415 (72): two of the head's Q, K, V, dO in LDS at a time";
  if (p.B <= 0 || p.H <= 0) return "attention backward: B, H must be positive";
  if (p.ldq % 8 || p.ldo % 8 || p.lddo % 8 || p.lddq % 4) return "attention backward: row strides must be 16-byte multiples";
  return nullptr;
}

hipError_t attn_bwd_launch(const AttnBwdArgs& p, hipStream_t stream) {
  const int Lp = (p.L + 31) & ~31;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)attn_bwd_kernel<0, 64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              4 * AB_MAXL * 128 + 2 * AB_MAXL * 4);
    (void)hipFuncSetAttribute((const void*)attn_bwd_kernel<1, 64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * AB_MAXL_LONG * 128 + 2 * AB_MAXL_LONG * 4);
    (void)hipFuncSetAttribute((const void*)attn_bwd_kernel<1, 72>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * 416 * 192 + 2 * 416 * 4);
    attr = true;
  }
  if (p.Dh == 72)
    hipLaunchKernelGGL((attn_bwd_kernel<1, 72>), dim3(p.B * p.H), dim3(AB_THREADS_LONG), 2 * Lp * 192 + 2 * Lp * 4,
                       stream, p);
  else if (p.L <= AB_MAXL)
    hipLaunchKernelGGL((attn_bwd_kernel<0, 64>), dim3(p.B * p.H), dim3(AB_THREADS), 4 * Lp * 128 + 2 * Lp * 4, stream, p);
  else
    hipLaunchKernelGGL((attn_bwd_kernel<1, 64>), dim3(p.B * p.H), dim3(AB_THREADS_LONG), 2 * Lp * 128 + 2 * Lp * 4,
                       stream, p);
  return hipGetLastError();
}

hipError_t lsimple_launch(const float* pred, const float* target, float* loss, float* dpred, int B, int per,
                          float gscale, hipStream_t stream, int tanh_bwd) {
  hipLaunchKernelGGL(lsimple_kernel, dim3(B), dim3(256), 0, stream, pred, target, loss, dpred, per, gscale, tanh_bwd);
  return hipGetLastError();
}

hipError_t conv3x3_bwd_launch(const float* dout, const float* in, const float* w, float* din, float* dw, float* db,
                              int B, int C, int H, int W, hipStream_t stream) {
  hipLaunchKernelGGL(conv_bwd_data_kernel, dim3(grid_for((long long)B * C * H * W)), dim3(256), 0, stream, dout, w, din,
                     B, C, H, W);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(conv_bwd_weight_kernel, dim3(C * C * 9 + C), dim3(256), 0, stream, dout, in, dw, db, B, C, H, W);
  return hipGetLastError();
}

hipError_t head_bwd_launch(const HeadBwdArgs& p, hipStream_t stream) {
  if (p.P > 64 || p.P_pad < p.P || p.P_pad > 64) return hipErrorInvalidValue;
  const int rows = p.B * (p.Himg / p.p) * (p.Wimg / p.p);
  hipLaunchKernelGGL(head_bwd_kernel, dim3((rows + 15) / 16), dim3(256), 0, stream, p);
  return hipGetLastError();
}

hipError_t patchify_launch(const float* img, bf16* pv, int B, int C, int H, int W, int p, int ldp, hipStream_t stream) {
  const long long n = (long long)B * (H / p) * (W / p) * ldp;
  hipLaunchKernelGGL(patchify_kernel, dim3(grid_for(n)), dim3(256), 0, stream, img, pv, B, C, H, W, p, ldp);
  return hipGetLastError();
}

hipError_t label_scatter_launch(const float* dx, int L, int row, int D, const int64_t* y, float* dlab, int B,
                                hipStream_t stream) {
  hipLaunchKernelGGL(label_scatter_kernel, dim3(B), dim3(256), 0, stream, dx, L, row, D, y, dlab, B);
  return hipGetLastError();
}

hipError_t add_cast_launch(float* dx, const float* add, bf16* dxb, long long n, hipStream_t stream) {
  if (n % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(add_cast_kernel, dim3(grid_for(n / 4)), dim3(256), 0, stream, dx, add, dxb, n / 4);
  return hipGetLastError();
}

hipError_t rows_add_cast_launch(float* dst, bf16* dstb, int drpg, int dgs, int doff, const float* src, int srpg, int sgs,
                                int soff, int rows, int D, int accumulate, hipStream_t stream) {
  if (rows <= 0) return hipSuccess;
  if (D % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rows_add_cast_kernel, dim3(grid_for((long long)rows * D / 4)), dim3(256), 0, stream, dst, dstb,
                     drpg, dgs, doff, src, srpg, sgs, soff, rows, D, accumulate);
  return hipGetLastError();
}

hipError_t transpose_bf16_launch(const float* w, bf16* wt, int N, int K, hipStream_t stream) {
  if (N % 4 || K % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3((K + 63) / 64, (N + 63) / 64), dim3(256), 0, stream, w, wt, N, K);
  return hipGetLastError();
}

hipError_t adamw_launch(const AdamWArgs& a, long long n, hipStream_t stream) {
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(n)), dim3(256), 0, stream, a, n);
  return hipGetLastError();
}

}  // namespace pdm

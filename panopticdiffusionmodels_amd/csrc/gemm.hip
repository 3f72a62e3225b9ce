// bf16 MFMA GEMM with fused epilogues for the U-ViT linear layers (gfx950).
//
//   C[m, n] = sum_k A[m, k] * W[n, k]   (+ bias[n])  -> epilogue
//
// W is the nn.Linear weight as stored by the reference ([out, in], libs/uvit.py:61-63, libs/timm.py:101-104),
// so both operands are K-contiguous.  A may be split along K into two row-major operands (the long-skip
// `skip_linear(cat([x, skip]))` of libs/uvit.py:116-117 without materialising the concat).
//
// Tile 128x128x64, 4 waves (2x2), each wave 64x64 = 4x4 mfma_f32_16x16x32_bf16 accumulators.  Operands
// are staged global->LDS with 16-byte LDS-DMA (global_load_lds_dwordx4), two stages; LDS rows are 128 B
// with an XOR swizzle (chunk ^ ((row >> 1) & 7)) applied on the SOURCE address, which makes every
// ds_read_b128 fragment read bank-conflict free.  The MFMA is issued with the weight fragment as the A
// operand so each lane ends up owning 4 consecutive output columns of one row: 8/16-byte epilogue stores.
#include <cstdio>
#include <type_traits>
#include <utility>

#include "pdm_common.h"
#include "pdm_kernels.h"

namespace pdm {

namespace {
constexpr int BM = 128, BN = 128, BK = 64;

template <int... I, class F>
__device__ __forceinline__ void sfor_impl(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  sfor_impl(std::make_integer_sequence<int, N>{}, f);
}
// bf16 / GELU epilogues: one bf16 output row per stored row, bias and the fused-LayerNorm consumer apply
constexpr bool epi_rowout(int e) { return e == EPI_BF16 || e == EPI_GELU; }

// A-operand row pointer for k-columns [k0, k0 + 64): dense rows, or an implicit-GEMM conv3x3 tap.
// (b, y, x) of the row's output pixel is passed in; returns the address of element k0 of that row.
__device__ __forceinline__ const bf16* conv_row_ptr(const GemmArgs& p, const bf16* A1, int b, int y, int x, int k0) {
  const int tap = k0 / p.convC, ci0 = k0 - tap * p.convC;
  const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
  if (yy < 0 || yy >= p.convH || xx < 0 || xx >= p.convW) return p.zero;
  const int sh = p.conv_up, Hs = p.convH >> sh, Ws = p.convW >> sh;
  return A1 + (((size_t)b * Hs + (yy >> sh)) * Ws + (xx >> sh)) * p.convC + ci0;
}
constexpr int TILE_BYTES = BM * BK * 2;           // 16 KiB per operand tile
constexpr int SMEM_BYTES = 2 * 2 * TILE_BYTES;    // 2 stages x (A, W)

__device__ __forceinline__ bf16x8 lds_frag(const char* tile, int row, int chunk) {
  const int off = row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
  return *reinterpret_cast<const bf16x8*>(tile + off);
}

template <int EPI>
__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(GemmArgs p, int tiles_n, int nwg) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap: blocks b and b+8 share an XCD; give each XCD a contiguous tile range so
  // neighbouring tiles (same A row panel) hit the same L2.
  int bid = blockIdx.x;
  {
    const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
  }
  const int tm = bid / tiles_n, tn = bid - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  if (p.batch > 1) {
    const long long z = blockIdx.y;
    p.A1 += z * p.sA;
    p.W += z * p.sW;
    if (p.out_bf16) p.out_bf16 += z * p.sO;
    if (p.out_f32) p.out_f32 += z * p.sR;
  }
  const int ldw = p.ldw > 0 ? p.ldw : p.K;

  auto stage = [&](int kt, int buf) {
    const int k0 = kt * BK;
    const bf16* Ab;
    int lda, ka;
    if (k0 < p.K1) { Ab = p.A1; lda = p.lda1; ka = k0; }
    else { Ab = p.A2; lda = p.lda2; ka = k0 - p.K1; }
    char* sa = smem + buf * (2 * TILE_BYTES);
    char* sw = sa + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rg = wave * 4 + i;               // group of 8 tile rows = one 1 KiB LDS-DMA
      const int row = rg * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      int gm = m0 + row;
      gm = gm < p.M ? gm : p.M - 1;
      const bf16* arow;
      if (p.conv) {
        const int hw = p.convH * p.convW, b = gm / hw, r = gm - b * hw;
        arow = conv_row_ptr(p, Ab, b, r / p.convW, r % p.convW, ka);
      } else {
        if (p.a_rows_per_group > 0 && k0 < p.K1) gm = (gm / p.a_rows_per_group) * p.a_group_stride + gm % p.a_rows_per_group;
        arow = Ab + (size_t)gm * lda + ka;
      }
      glds16(arow + c * 8, (PDM_LDS void*)(sa + rg * 1024));
      int gn = n0 + row;
      gn = gn < p.N ? gn : p.N - 1;
      glds16(p.W + (size_t)gn * ldw + k0 + c * 8, (PDM_LDS void*)(sw + rg * 1024));
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const char* sa = smem + cur * (2 * TILE_BYTES);
    const char* sw = sa + TILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + (lane >> 4);
      bf16x8 af[4], wf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = lds_frag(sa, wm * 64 + i * 16 + (lane & 15), chunk);
#pragma unroll
      for (int i = 0; i < 4; ++i) wf[i] = lds_frag(sw, wn * 64 + i * 16 + (lane & 15), chunk);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) acc[ni][mi] = mfma16x16x32(wf[ni], af[mi], acc[ni][mi]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: lane owns rows m = .. + (lane & 15), columns n .. n+3
  const bool ln = epi_rowout(EPI) && p.ln_stats != nullptr;
  float2 mr[4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    mr[mi] = make_float2(0.f, 1.f);
    if (ln) {
      const int m = min(m0 + wm * 64 + mi * 16 + (lane & 15), p.M - 1);
      mr[mi] = ln_merge(p.ln_stats + (size_t)m * p.ln_ld * 2, p.ln_ld, p.ln_D, p.ln_eps);
    }
  }
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = n0 + wn * 64 + ni * 16 + (lane >> 4) * 4;
    if (n >= p.N) continue;  // N % 4 == 0: a lane's 4 columns are all in or all out
    f32x4 b = f32x4{0.f, 0.f, 0.f, 0.f};
    if (p.bias) b = *reinterpret_cast<const f32x4*>(p.bias + n);
    f32x4 c = f32x4{0.f, 0.f, 0.f, 0.f};
    if (ln) c = *reinterpret_cast<const f32x4*>(p.ln_colsum + n);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int m = m0 + wm * 64 + mi * 16 + (lane & 15);
      if (m >= p.M) continue;
      f32x4 v = acc[ni][mi];
      if (ln) v = (v - mr[mi].x * c) * mr[mi].y;
      v += b;
      if constexpr (EPI == EPI_BF16) {
        *reinterpret_cast<bf16x4*>(p.out_bf16 + (size_t)m * p.ldo + n) = to_bf16x4(v[0], v[1], v[2], v[3]);
      } else if constexpr (EPI == EPI_GELU) {
        *reinterpret_cast<bf16x4*>(p.out_bf16 + (size_t)m * p.ldo + n) =
            to_bf16x4(gelu_act(p.act, v[0]), gelu_act(p.act, v[1]), gelu_act(p.act, v[2]), gelu_act(p.act, v[3]));
      } else if constexpr (EPI == EPI_RES) {
        if (p.accumulate) {
          const bf16x4 r = *reinterpret_cast<const bf16x4*>(p.res_in + (size_t)m * p.ldri + n);
          v += f32x4{(float)r[0], (float)r[1], (float)r[2], (float)r[3]};
        }
        *reinterpret_cast<bf16x4*>(p.out_bf16 + (size_t)m * p.ldo + n) = to_bf16x4(v[0], v[1], v[2], v[3]);
      } else {
        f32x4* r = reinterpret_cast<f32x4*>(p.out_f32 + (size_t)m * p.ldr + n);
        if (p.accumulate)
          v += p.res_f32 ? *reinterpret_cast<const f32x4*>(p.res_f32 + (size_t)m * p.ldrf + n) : *r;
        *r = v;
        if (p.out_bf16)
          *reinterpret_cast<bf16x4*>(p.out_bf16 + (size_t)m * p.ldo + n) = to_bf16x4(v[0], v[1], v[2], v[3]);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// 256x256 tile, 8 waves (2 along M x 4 along N, 128x64 per wave = 8x4 MFMA 16x16x32 accumulators).
// K streams through an NS-slot LDS ring of BK-deep sub-tiles (slot = A 256xBK + W 256xBK; BK*2-byte rows
// with an XOR chunk swizzle that makes the fragment ds_read_b128 conflict-free).  NS-1 sub-tiles are kept
// in flight with LDS-DMA; each iteration waits with a COUNTED vmcnt for its own sub-tile only and passes
// one raw s_barrier, so the loads of the next sub-tiles overlap this one's MFMAs.
// Arithmetic intensity per CU: 128 FLOP per staged byte (the 128x128 tile above: 64).
//   BK = 32, NS = 4: 32 KiB slots, 3 in flight, 64-byte rows (half cache lines per load)
//   BK = 64, NS = 2: 64 KiB slots, 1 in flight, 128-byte rows (full lines)
constexpr int BM2 = 256, BN2 = 256;
constexpr int EPI_LDS = 128 * 1024;             // the 256-tile epilogue's staging area; LN row stats follow it
constexpr int EPI_LDS_EXTRA = 256 * 8;
constexpr int COL_LDS = EPI_LDS + EPI_LDS_EXTRA;   // gemm8d: the tile's bias [256] and LN colsum [256] (fp32)
constexpr int COL_LDS_BYTES = 2 * 256 * 4;

template <int BK>
__device__ __forceinline__ int swz_off(int row, int chunk) {
  if constexpr (BK == 32) return row * 64 + ((chunk ^ ((row >> 1) & 3)) << 4);
  else return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
}

// Fragment f of a 256x256 tile's accumulators -> (row, column) of its 16x4 piece within the tile.
//   MAP 0 (gemm256_kernel): wave (wm, wn) owns rows wm*128 + [0,128), columns wn*64 + [0,64); f = ni*8 + mi
//   MAP 1 (gemm8p_kernel):  quadrant (qi, qj) of the tile, wave owns rows qi*128 + wm*64 + [0,64),
//                            columns qj*128 + wn*32 + [0,32); f = ((qi*2 + qj)*2 + ni)*4 + mi
template <int MAP>
__device__ __forceinline__ void frag_pos(int f, int lane, int wm, int wn, int& ml, int& nl) {
  if constexpr (MAP == 0) {
    const int ni = f / 8, mi = f % 8;
    ml = wm * 128 + mi * 16 + (lane & 15);
    nl = wn * 64 + ni * 16 + (lane >> 4) * 4;
  } else {
    const int qi = f / 16, qj = (f / 8) & 1, ni = (f / 4) & 1, mi = f & 3;
    ml = qi * 128 + wm * 64 + mi * 16 + (lane & 15);
    nl = qj * 128 + wn * 32 + ni * 16 + (lane >> 4) * 4;
  }
}

// (mean, rstd) of a row from its <= 8 LayerNorm partials (sum, M2 per 256-column group; Chan's merge, the
// arithmetic of ln_merge in the same order) and, when mu != nullptr, every group's mean mu[t] = sum_t / width_t
// (the centre the producing epilogue subtracted: GemmArgs::mx_center)
__device__ __forceinline__ float2 ln_from_partials(const float2 (&lst)[8], int ld, int D, float eps, float* mu) {
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < 8; ++t) if (t < ld) sum += lst[t].x;
  const float mean = sum / (float)D;
  float m2 = 0.f;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const float n = (float)min(256, D - 256 * t);
    if (mu) mu[t] = t < ld ? lst[t].x / n : 0.f;
    if (t < ld) {
      const float d = lst[t].x / n - mean;
      m2 += lst[t].y + n * d * d;
    }
  }
  return make_float2(mean, 1.0f / sqrtf(m2 / (float)D + eps));
}

// Sum over each 32-lane half of the wave, bitwise the same in every lane (each step adds two equal-valued partners,
// so the commuted sums agree): two quad_perm butterflies, row_half_mirror (quad 0 <-> 1, 2 <-> 3) and row_mirror
// (8-lane halves) as VALU adds with a DPP source (no LDS traffic) for the 16-lane rows, then one swizzle across the
// two rows of each half (v_permlane16_swap measured wrong for this: tools/probes/dpp_probe.hip).
template <int CTRL>
__device__ __forceinline__ float dpp_add(float x) {
  return x + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float sum32(float x) {
  x = dpp_add<0xb1>(x);    // quad_perm [1,0,3,2]
  x = dpp_add<0x4e>(x);    // quad_perm [2,3,0,1]
  x = dpp_add<0x141>(x);   // row_half_mirror
  x = dpp_add<0x140>(x);   // row_mirror
  return x + __shfl_xor(x, 16, 64);
}

// GroupNorm partials in the 256-tile epilogue (GemmArgs::gn_part): a thread stores 8 consecutive columns
// n0 + (tid & 31) * 8 of 16 rows of the tile; gn_cpg >= 8 puts them in one group (slot 0), gn_cpg = 4 in two.
__device__ __forceinline__ void gn_acc(const GemmArgs& p, const float (&f)[8], float (&gs)[2], float (&gq)[2]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int sl = p.gn_cpg == 4 ? (j >> 2) : 0;
    gs[sl] += f[j];
    gq[sl] = fmaf(f[j], f[j], gq[sl]);
  }
}
// the 16 row-threads of each column octet and the octets of a group combine through LDS in fp64 (as
// gn_partial_kernel's per-group pass); one thread per group of the tile writes its 256-row chunk's partial.
// Callers: after a barrier behind the tile's last LDS read; the caller's next LDS write follows a barrier.
__device__ __forceinline__ void gn_store(const GemmArgs& p, char* smem, int tid, int m0, int n0, const float (&gs)[2],
                                         const float (&gq)[2]) {
  float2* red = reinterpret_cast<float2*>(smem);   // [16 row-threads][32 octets][2 slots]
  red[((tid >> 5) * 32 + (tid & 31)) * 2] = make_float2(gs[0], gq[0]);
  red[((tid >> 5) * 32 + (tid & 31)) * 2 + 1] = make_float2(gs[1], gq[1]);
  __syncthreads();
  const int cpg = p.gn_cpg, ngr = min(256, p.N - n0) / cpg;
  if (tid < ngr) {
    double s = 0.0, q = 0.0;
    const int c0 = tid * cpg / 8, nc = cpg >= 8 ? cpg / 8 : 1, sl = cpg >= 8 ? 0 : (tid & 1);
    for (int c = c0; c < c0 + nc; ++c)
      for (int r = 0; r < 16; ++r) {
        const float2 v = red[(r * 32 + c) * 2 + sl];
        s += v.x;
        q += v.y;
      }
    const int b = m0 / p.gn_P, chunk = (m0 - b * p.gn_P) >> 8, g = n0 / cpg + tid;
    double* o = p.gn_part + (((size_t)b * (p.gn_P >> 8) + chunk) * 32 + g) * 2;
    o[0] = s;
    o[1] = q;
  }
  __syncthreads();
}

// Epilogue of a 256x256 tile (needs 128 KiB of LDS; the staging ring is free by then).
//  EPI_RES: the fp32 path below with a bf16 residual stream (res_in read, bf16 out_bf16 written, 16-byte rows).
//  bf16 / GELU: the bf16 tile is written to LDS with a row-XOR chunk swizzle, then stored row-contiguously
//    with 16-byte stores (full lines, half the store instructions of the per-lane 8-byte scatter).  Non-temporal
//    (streaming) stores measured neutral (profiles/r03nt/: qkv 149.1 vs 149.0 us, L/2 bench 57.9 vs 58.0 img/s).
//  fp32 residual: two 128-row passes through LDS; every thread then owns 8 consecutive columns of a row:
//    2 x 16-byte residual loads, 2 x 16-byte stores and one 16-byte bf16 copy store per row chunk.
template <int EPI, int MAP>
__device__ __forceinline__ void epilogue256(const GemmArgs& p, const f32x4 (&acc)[32], char* smem, int m0, int n0,
                                            int tid, int lane, int wm, int wn, bool ln_ready = false,
                                            bool cols_ready = false, int col_off = COL_LDS) {
  // bias of the lane's 4 column groups, loaded up front with one wave-uniform branch (columns past N read a
  // clamped address and are never stored)
  f32x4 bv[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) bv[g] = f32x4{0.f, 0.f, 0.f, 0.f};
  // cols_ready: the kernel staged the tile's bias / colsum (zeros past N or when absent) at COL_LDS in its prologue
  const float* lcol = reinterpret_cast<const float*>(smem + col_off);
  if (epi_rowout(EPI) && cols_ready) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      int ml, nl;
      frag_pos<MAP>(MAP == 0 ? g * 8 : (g >> 1) * 8 + (g & 1) * 4, lane, wm, wn, ml, nl);
      bv[g] = *reinterpret_cast<const f32x4*>(lcol + nl);
    }
  } else if (epi_rowout(EPI) && p.bias) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      int ml, nl;
      frag_pos<MAP>(MAP == 0 ? g * 8 : (g >> 1) * 8 + (g & 1) * 4, lane, wm, wn, ml, nl);
      const int n = min(n0 + nl, p.N - 4);
      bv[g] = *reinterpret_cast<const f32x4*>(p.bias + n);
    }
  }
  const bool full = (m0 + 256 <= p.M) && (n0 + 256 <= p.N);
  // fused LayerNorm consumer: per-row (mean, rstd) of the tile's 256 rows into LDS past the 128 KiB staging
  // area, per-column sums of the gamma-scaled weight like the bias
  float2* lnrow = reinterpret_cast<float2*>(smem + EPI_LDS);
  f32x4 cs[4];
  const bool ln = epi_rowout(EPI) && p.ln_stats != nullptr;
  if (ln) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      int ml, nl;
      frag_pos<MAP>(MAP == 0 ? g * 8 : (g >> 1) * 8 + (g & 1) * 4, lane, wm, wn, ml, nl);
      cs[g] = cols_ready ? *reinterpret_cast<const f32x4*>(lcol + 256 + nl)
                         : *reinterpret_cast<const f32x4*>(p.ln_colsum + min(n0 + nl, p.N - 4));
    }
    if (tid < 256 && !ln_ready) {   // ln_ready: the kernel merged them into lnrow during its prologue
      const int m = min(m0 + tid, p.M - 1);
      lnrow[tid] = ln_merge(p.ln_stats + (size_t)m * p.ln_ld * 2, p.ln_ld, p.ln_D, p.ln_eps);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU) {
    auto stage = [&](auto with_ln) {
#pragma unroll
      for (int f = 0; f < 32; ++f) {
        int ml, nl;
        frag_pos<MAP>(f, lane, wm, wn, ml, nl);
        const int gi = MAP == 0 ? f / 8 : (f / 8 & 1) * 2 + (f / 4 & 1);
        f32x4 v = acc[f];
        if constexpr (decltype(with_ln)::value) {
          const float2 mr = lnrow[ml];
          v = (v - mr.x * cs[gi]) * mr.y;
        }
        v += bv[gi];
        if constexpr (EPI == EPI_GELU) {
          if (p.act) {
            v[0] = gelu_quick(v[0]); v[1] = gelu_quick(v[1]); v[2] = gelu_quick(v[2]); v[3] = gelu_quick(v[3]);
          } else {
            const f32x2 lo = gelu_erf2(f32x2{v[0], v[1]}), hi = gelu_erf2(f32x2{v[2], v[3]});
            v = f32x4{lo[0], lo[1], hi[0], hi[1]};
          }
        }
        const int off = ml * 512 + ((((nl >> 3) ^ (ml & 31)) << 4) | ((nl & 4) << 1));
        *reinterpret_cast<bf16x4*>(smem + off) = to_bf16x4(v[0], v[1], v[2], v[3]);
      }
    };
    if (ln) stage(std::true_type{});
    else stage(std::false_type{});
    __syncthreads();
    i32x4 v[16];
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int idx = it * 512 + tid;
      const int ml = idx >> 5, ch = idx & 31;
      v[it] = *reinterpret_cast<const i32x4*>(smem + ml * 512 + ((ch ^ (ml & 31)) << 4));
    }
    if (p.out_fp8) {   // MXFP8 copy: 4 consecutive lanes hold one 32-column block of a row
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int idx = it * 512 + tid;
        const int m = m0 + (idx >> 5), n = n0 + (idx & 31) * 8;
        const bf16x8 b8 = __builtin_bit_cast(bf16x8, v[it]);
        float f[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = (float)b8[j];
        unsigned e8;
        const uint2 q = mx_quant8(f, &e8);
        if (m < p.M && n < p.N) mx_store8(p.out_fp8, p.ldo8, p.out_scale, p.out_scale_ld, m, n, q, e8, (tid & 3) == 0);
      }
    }
    if (p.gn_part) {   // GroupNorm partials of the rounded values (exactly what the GroupNorm reads)
      float gs[2] = {0.f, 0.f}, gq[2] = {0.f, 0.f};
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const bf16x8 b8 = __builtin_bit_cast(bf16x8, v[it]);
        float f[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = (float)b8[j];
        gn_acc(p, f, gs, gq);
      }
      __syncthreads();   // every thread's LDS read-back is done: the reduction reuses the staging area
      gn_store(p, smem, tid, m0, n0, gs, gq);
    }
    if (!p.out_bf16) return;
    if ((p.dbg_tile0 & 4) && ((n0 >> 8) & 1)) return;   // timing experiment: odd column tiles store nothing
    if (full) {
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int idx = it * 512 + tid;
        const int mr = (p.dbg_tile0 & 8) ? (idx >> 5) : m0 + (idx >> 5);   // timing experiment: bit 3 = every
        *reinterpret_cast<i32x4*>(p.out_bf16 + (size_t)mr * p.ldo + n0 + (idx & 31) * 8) = v[it];   // row tile -> rows 0..255
      }
    } else {
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int idx = it * 512 + tid;
        const int m = m0 + (idx >> 5), n = n0 + (idx & 31) * 8;
        if (m < p.M && n < p.N) *reinterpret_cast<i32x4*>(p.out_bf16 + (size_t)m * p.ldo + n) = v[it];
      }
    }
    return;
  }
  // fp32: the thread's 8 store columns n0 + (tid & 31) * 8 are the same in every row it stores; the 32
  // threads of a half-wave hold one whole 256-column row, so the LayerNorm partials of the row are two
  // half-wave reductions (sum, then M2 about the group mean)
  const int ncols = min(256, p.N - n0);
  auto row_stats = [&](const f32x4& a, const f32x4& b, int m, int n) -> float {   // returns the group mean
    float sv = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sv += n + j < p.N ? a[j] : 0.f;
      sv += n + 4 + j < p.N ? b[j] : 0.f;
    }
    sv = sum32(sv);
    const float mu = sv / (float)ncols;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float d0 = a[j] - mu, d1 = b[j] - mu;
      q += n + j < p.N ? d0 * d0 : 0.f;
      q += n + 4 + j < p.N ? d1 * d1 : 0.f;
    }
    q = sum32(q);
    if ((tid & 31) == 0 && m < p.M) {
      *reinterpret_cast<float2*>(p.stats_out + ((size_t)m * p.stats_ld + (n0 >> 8)) * 2) = make_float2(sv, q);
      if (EPI == EPI_RES && p.stats_out2) {
        const size_t m2 = (size_t)(m / p.out2_rpg) * p.out2_gs + m % p.out2_rpg;
        *reinterpret_cast<float2*>(p.stats_out2 + (m2 * p.stats_ld + (n0 >> 8)) * 2) = make_float2(sv, q);
      }
    }
    return mu;
  };
  // MXFP8 copy of the stored fp32 row piece, minus its 256-column group mean c (mx_center; 0 otherwise)
  auto mx_row = [&](const f32x4& a, const f32x4& b, int m, int n, float c) {
    const float f[8] = {a[0] - c, a[1] - c, a[2] - c, a[3] - c, b[0] - c, b[1] - c, b[2] - c, b[3] - c};
    unsigned e8;
    const uint2 q = mx_quant8(f, &e8);
    if (m < p.M && n < p.N) mx_store8(p.out_fp8, p.ldo8, p.out_scale, p.out_scale_ld, m, n, q, e8, (tid & 3) == 0);
  };
  f32x4 b0 = f32x4{0.f, 0.f, 0.f, 0.f}, b1 = b0;
  if (cols_ready) {
    b0 = *reinterpret_cast<const f32x4*>(lcol + (tid & 31) * 8);
    b1 = *reinterpret_cast<const f32x4*>(lcol + (tid & 31) * 8 + 4);
  } else if (p.bias) {
    const int n = min(n0 + (tid & 31) * 8, p.N - 8 >= 0 ? p.N - 8 : 0);
    b0 = *reinterpret_cast<const f32x4*>(p.bias + n);
    if (n + 4 < p.N) b1 = *reinterpret_cast<const f32x4*>(p.bias + n + 4);
  }
  float gs[2] = {0.f, 0.f}, gq[2] = {0.f, 0.f};   // GroupNorm partials (p.gn_part) of the thread's stored rows
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int f = 0; f < 32; ++f) {
      int ml, nl;
      frag_pos<MAP>(f, lane, wm, wn, ml, nl);
      if ((ml >> 7) != pass) continue;   // compile-time for MAP 1; wave-uniform for MAP 0
      ml &= 127;
      *reinterpret_cast<f32x4*>(smem + ml * 1024 + (((nl >> 2) ^ (ml & 63)) << 4)) = acc[f];
    }
    __syncthreads();
#pragma unroll 1
    for (int g = 0; g < 2; ++g) {   // not unrolled: keeps the staged rows + residual loads within the VGPR budget
      f32x4 v0[4], v1[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int idx = (g * 4 + i) * 512 + tid;
        const int ml = idx >> 5, c8 = idx & 31;
        v0[i] = *reinterpret_cast<const f32x4*>(smem + ml * 1024 + (((2 * c8) ^ (ml & 63)) << 4)) + b0;
        v1[i] = *reinterpret_cast<const f32x4*>(smem + ml * 1024 + (((2 * c8 + 1) ^ (ml & 63)) << 4)) + b1;
      }
      if constexpr (EPI == EPI_RES) {
        // bf16 residual stream (GemmArgs::res_in): v += res_in, out = bf16(v); the LayerNorm partials and the MXFP8
        // copy are taken from the rounded values (exactly what the next GEMM reads)
        if (p.accumulate) {
          i32x4 rr[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int idx = (g * 4 + i) * 512 + tid;
            const int m = min(m0 + pass * 128 + (idx >> 5), p.M - 1), n = min(n0 + (idx & 31) * 8, p.N - 8);
            rr[i] = *reinterpret_cast<const i32x4*>(p.res_in + (size_t)m * p.ldri + n);
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const bf16x8 r = __builtin_bit_cast(bf16x8, rr[i]);
#pragma unroll
            for (int j = 0; j < 4; ++j) { v0[i][j] += (float)r[j]; v1[i][j] += (float)r[4 + j]; }
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int idx = (g * 4 + i) * 512 + tid;
          const int m = m0 + pass * 128 + (idx >> 5), n = n0 + (idx & 31) * 8;
          bf16x8 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) { o[j] = (bf16)v0[i][j]; o[4 + j] = (bf16)v1[i][j]; }
          if (full || (m < p.M && n < p.N)) {
            *reinterpret_cast<bf16x8*>(p.out_bf16 + (size_t)m * p.ldo + n) = o;
            if (p.out2)
              *reinterpret_cast<bf16x8*>(p.out2 + ((size_t)(m / p.out2_rpg) * p.out2_gs + m % p.out2_rpg) * p.ldo + n) = o;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) { v0[i][j] = (float)o[j]; v1[i][j] = (float)o[4 + j]; }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int idx = (g * 4 + i) * 512 + tid;
          const int m = m0 + pass * 128 + (idx >> 5), n = n0 + (idx & 31) * 8;
          const float mu = p.stats_out ? row_stats(v0[i], v1[i], m, n) : 0.f;
          if (p.out_fp8) mx_row(v0[i], v1[i], m, n, p.mx_center ? mu : 0.f);
        }
      } else if (full) {
        if (p.accumulate) {
          f32x4 r0[4], r1[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int idx = (g * 4 + i) * 512 + tid;
            const size_t mr = (size_t)(m0 + pass * 128 + (idx >> 5));
            const f32x4* r = reinterpret_cast<const f32x4*>(p.res_f32 ? p.res_f32 + mr * p.ldrf : p.out_f32 + mr * p.ldr) +
                             (n0 + (idx & 31) * 8) / 4;
            r0[i] = r[0];
            r1[i] = r[1];
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) { v0[i] += r0[i]; v1[i] += r1[i]; }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int idx = (g * 4 + i) * 512 + tid;
          const size_t m = m0 + pass * 128 + (idx >> 5);
          const int n = n0 + (idx & 31) * 8;
          f32x4* r = reinterpret_cast<f32x4*>(p.out_f32 + m * p.ldr + n);
          r[0] = v0[i];
          r[1] = v1[i];
          if (p.gn_part) {
            const float f[8] = {v0[i][0], v0[i][1], v0[i][2], v0[i][3], v1[i][0], v1[i][1], v1[i][2], v1[i][3]};
            gn_acc(p, f, gs, gq);
          }
          if (p.out_bf16) {
            bf16x8 o;
#pragma unroll
            for (int j = 0; j < 4; ++j) { o[j] = (bf16)v0[i][j]; o[4 + j] = (bf16)v1[i][j]; }
            *reinterpret_cast<bf16x8*>(p.out_bf16 + m * p.ldo + n) = o;
          }
        }
        float mu[4] = {0.f, 0.f, 0.f, 0.f};
        if (p.stats_out) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int idx = (g * 4 + i) * 512 + tid;
            mu[i] = row_stats(v0[i], v1[i], m0 + pass * 128 + (idx >> 5), n0 + (idx & 31) * 8);
          }
        }
        if (p.out_fp8) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int idx = (g * 4 + i) * 512 + tid;
            mx_row(v0[i], v1[i], m0 + pass * 128 + (idx >> 5), n0 + (idx & 31) * 8, p.mx_center ? mu[i] : 0.f);
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int idx = (g * 4 + i) * 512 + tid;
          const int m = m0 + pass * 128 + (idx >> 5), n = n0 + (idx & 31) * 8;
          if (m < p.M && n < p.N) {
            f32x4* r = reinterpret_cast<f32x4*>(p.out_f32 + (size_t)m * p.ldr + n);
            f32x4 a = v0[i], b = v1[i];
            if (p.accumulate) {
              const f32x4* rs = p.res_f32 ? reinterpret_cast<const f32x4*>(p.res_f32 + (size_t)m * p.ldrf + n) : r;
              a += rs[0];
              b += rs[1];
            }
            r[0] = a;
            r[1] = b;
            if (p.gn_part) {   // (gn_part tiles are whole: gemm_gn_fusable)
              const float f[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
              gn_acc(p, f, gs, gq);
            }
            if (p.out_bf16) {
              bf16x8 o;
#pragma unroll
              for (int j = 0; j < 4; ++j) { o[j] = (bf16)a[j]; o[4 + j] = (bf16)b[j]; }
              *reinterpret_cast<bf16x8*>(p.out_bf16 + (size_t)m * p.ldo + n) = o;
            }
            v0[i] = a;
            v1[i] = b;
          }
          const float mu = p.stats_out ? row_stats(v0[i], v1[i], m, n) : 0.f;
          if (p.out_fp8) mx_row(v0[i], v1[i], m, n, p.mx_center ? mu : 0.f);
        }
      }
    }
    __syncthreads();
  }
  if constexpr (EPI == EPI_F32) {
    if (p.gn_part) gn_store(p, smem, tid, m0, n0, gs, gq);
  }
}

template <int EPI, int BK, int NS>
__global__ __launch_bounds__(512, 1) void gemm256_kernel(GemmArgs p, int tiles_n, int nwg) {
  constexpr int ROWB = BK * 2;                 // bytes per LDS row
  constexpr int RPP = 1024 / ROWB;             // rows per 1 KiB LDS-DMA piece
  constexpr int CPR = ROWB / 16;               // 16-byte chunks per row
  constexpr int PPW = 256 / RPP / 8;           // pieces per wave per operand per sub-tile
  constexpr int LPS = 2 * PPW;                 // LDS-DMA instructions per wave per sub-tile
  constexpr int SLOT = (BM2 + BN2) * ROWB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  int bid = blockIdx.x;
  {
    const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
  }
  const int tm = bid / tiles_n, tn = bid - tm * tiles_n;
  const int m0 = tm * BM2, n0 = tn * BN2;
  if (p.batch > 1) {
    const long long z = blockIdx.y;
    p.A1 += z * p.sA;
    p.W += z * p.sW;
    if (p.out_bf16) p.out_bf16 += z * p.sO;
    if (p.out_f32) p.out_f32 += z * p.sR;
  }
  const int ldw = p.ldw > 0 ? p.ldw : p.K;

  const int prow = lane / CPR;
  const int pch = lane % CPR;
  const bf16* asrc[PPW];
  const bf16* a2src[PPW];
  const bf16* wsrc[PPW];
  int soff[PPW];
  int cb[PPW], cy[PPW], cx[PPW];   // conv mode: output pixel of each piece row
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int row = (wave * PPW + i) * RPP + prow;
    const int c = (swz_off<BK>(row, pch) - row * ROWB) >> 4;   // logical chunk stored at physical pch
    soff[i] = c * 8;
    int gm = m0 + row;
    gm = gm < p.M ? gm : p.M - 1;
    const int gm1 = p.a_rows_per_group > 0 ? (gm / p.a_rows_per_group) * p.a_group_stride + gm % p.a_rows_per_group : gm;
    asrc[i] = p.A1 + (size_t)gm1 * p.lda1;
    a2src[i] = p.A2 ? p.A2 + (size_t)gm * p.lda2 : nullptr;
    if (p.conv) {
      const int hw = p.convH * p.convW;
      cb[i] = gm / hw;
      const int r = gm - cb[i] * hw;
      cy[i] = r / p.convW;
      cx[i] = r - cy[i] * p.convW;
    }
    int gn = n0 + row;
    gn = gn < p.N ? gn : p.N - 1;
    wsrc[i] = p.W + (size_t)gn * ldw;
  }

  auto issue = [&](int j) {
    const int k0 = j * BK;
    char* slot = smem + (j % NS) * SLOT;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int piece = wave * PPW + i;
      const bf16* src;
      if (p.conv) src = conv_row_ptr(p, p.A1, cb[i], cy[i], cx[i], k0) + soff[i];
      else src = (k0 < p.K1) ? asrc[i] + k0 + soff[i] : a2src[i] + (k0 - p.K1) + soff[i];
      glds16(src, (PDM_LDS void*)(slot + piece * 1024));
      glds16(wsrc[i] + k0 + soff[i], (PDM_LDS void*)(slot + BM2 * ROWB + piece * 1024));
    }
  };

  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nsub = p.K / BK;
#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (j < nsub) issue(j);
  for (int j = 0; j < nsub; ++j) {
    const int ahead = min(nsub - 1 - j, NS - 2);
    if (ahead >= 3) wait_vmcnt<3 * LPS>();
    else if (ahead == 2) wait_vmcnt<2 * LPS>();
    else if (ahead == 1) wait_vmcnt<LPS>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (j + NS - 1 < nsub) issue(j + NS - 1);
    const char* slot = smem + (j % NS) * SLOT;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int chunk = kk * 4 + (lane >> 4);
      bf16x8 wf[4], af[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wn * 64 + i * 16 + (lane & 15);
        wf[i] = *reinterpret_cast<const bf16x8*>(slot + BM2 * ROWB + swz_off<BK>(row, chunk));
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = wm * 128 + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(slot + swz_off<BK>(row, chunk));
      }
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[ni][mi] = mfma16x16x32(wf[ni], af[mi], acc[ni][mi]);
    }
  }

  f32x4 flat[32];
#pragma unroll
  for (int f = 0; f < 32; ++f) flat[f] = acc[f / 8][f % 8];
  epilogue256<EPI, 0>(p, flat, smem, m0, n0, tid, lane, wm, wn);
}

// ------------------------------------------------------------------------------------------------
// 256x256x64 tile, 8 waves, 8-phase schedule (2 LDS buffers x 4 half-tiles).  Each K-tile is staged as four
// 16 KiB half-tiles (A rows 0-127 / 128-255, W rows 0-127 / 128-255), one per phase, two K-tiles' worth of
// buffers; the block's 256x256 output is cut into quadrants (qi = A half, qj = W half) and every wave owns a
// 64x32 piece of each quadrant, so phase q needs only the two half-tiles of its quadrant.  Phase order
// (0,0) (0,1) (1,1) (1,0) reads 12 / 4 / 8 / 0 fragments (W fragments of both halves stay in registers).
// Each phase: fragment reads, one half-tile LDS-DMA of the next K-tile, counted vmcnt (2 half-tiles stay
// in flight), barrier, 16 MFMAs at raised priority, barrier.  Waves 4-7 run one barrier behind waves 0-3
// (one extra barrier up front), so on every SIMD one wave computes while its partner reads/stages.
// Requires K % 128 == 0 (an even number of K-tiles).
__device__ __forceinline__ void bar_raw() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int EPI, int CONV>
__global__ __launch_bounds__(512, 1) void gemm8p_kernel(GemmArgs p, int tiles_n, int nwg) {
  constexpr int ROWB = 128;                     // 64 bf16 per LDS row
  constexpr int HALF = 128 * ROWB;              // 16 KiB half-tile
  constexpr int BUF = 4 * HALF;                 // A0 A1 W0 W1
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  int bid = blockIdx.x;
  {
    const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
  }
  const int tm = bid / tiles_n, tn = bid - tm * tiles_n;
  const int m0 = tm * BM2, n0 = tn * BN2;
  if (p.batch > 1) {
    const long long z = blockIdx.y;
    p.A1 += z * p.sA;
    p.W += z * p.sW;
    if (p.out_bf16) p.out_bf16 += z * p.sO;
    if (p.out_f32) p.out_f32 += z * p.sR;
  }
  const int ldw = p.ldw > 0 ? p.ldw : p.K;

  // this lane's LDS-DMA sources: half h, piece i (8 rows x 128 B per wave-instruction), lane -> (row, chunk)
  const int prow = lane >> 3, pch = lane & 7;
  const bf16* a1src[2][2];
  const bf16* a2src[2][2];
  const bf16* wsrc[2][2];
  int soff[2];
  int cpix[2][2], cb[2][2];   // conv: packed (y << 16 | x) and image of the piece row
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 8 + prow;           // row within the half-tile (0..127)
    soff[i] = (pch ^ ((row >> 1) & 7)) * 8;               // logical chunk stored at physical pch
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int gm = m0 + h * 128 + row;
      gm = gm < p.M ? gm : p.M - 1;
      const int gm1 = (!CONV && p.a_rows_per_group > 0) ? (gm / p.a_rows_per_group) * p.a_group_stride + gm % p.a_rows_per_group : gm;
      a1src[h][i] = p.A1 + (size_t)gm1 * p.lda1;
      a2src[h][i] = p.A2 ? p.A2 + (size_t)gm * p.lda2 : p.A1;
      if constexpr (CONV) {
        const int hw = p.convH * p.convW;
        cb[h][i] = gm / hw;
        const int r = gm - cb[h][i] * hw;
        const int y = r / p.convW;
        cpix[h][i] = (y << 16) | (r - y * p.convW);
      }
      int gn = n0 + h * 128 + row;
      gn = gn < p.N ? gn : p.N - 1;
      wsrc[h][i] = p.W + (size_t)gn * ldw;
    }
  }

  // half-tile kinds: 0 = A rows 0-127, 1 = A rows 128-255, 2 = W rows 0-127, 3 = W rows 128-255
  auto issue = [&](int kt, int kind) {
    const int k0 = kt * 64;
    char* dst = smem + (kt & 1) * BUF + kind * HALF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int piece = wave * 2 + i;
      const bf16* src;
      if (kind >= 2) {
        src = wsrc[kind - 2][i] + k0 + soff[i];
      } else if constexpr (CONV) {
        const int pix = cpix[kind][i];
        src = conv_row_ptr(p, p.A1, cb[kind][i], pix >> 16, pix & 0xffff, k0) + soff[i];
      } else {
        src = (k0 < p.K1) ? a1src[kind][i] + k0 + soff[i] : a2src[kind][i] + (k0 - p.K1) + soff[i];
      }
      glds16(src, (PDM_LDS void*)(dst + piece * 1024));
    }
  };

  f32x4 acc[32];
#pragma unroll
  for (int f = 0; f < 32; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2];      // A fragments of the current A half: [mi][k-sub]
  bf16x8 wf[2][2][2];   // W fragments of both W halves: [qj][ni][k-sub]

  auto read_a = [&](const char* buf, int qi) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int row = qi * 128 + wm * 64 + mi * 16 + (lane & 15);   // row within the 256-row A image
        af[mi][ks] = *reinterpret_cast<const bf16x8*>(buf + (row >> 7) * HALF + swz_off<64>(row & 127, ks * 4 + (lane >> 4)));
      }
  };
  auto read_w = [&](const char* buf, int qj) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int row = wn * 32 + ni * 16 + (lane & 15);
        wf[qj][ni][ks] = *reinterpret_cast<const bf16x8*>(buf + (2 + qj) * HALF + swz_off<64>(row, ks * 4 + (lane >> 4)));
      }
  };
  auto mma = [&](int qi, int qj) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          f32x4& c = acc[((qi * 2 + qj) * 2 + ni) * 4 + mi];
          c = mfma16x16x32(wf[qj][ni][ks], af[mi][ks], c);
        }
    __builtin_amdgcn_s_setprio(0);
  };

  const int nk = p.K / 64;
  issue(0, 0);
  issue(0, 2);
  issue(0, 3);
  issue(0, 1);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // A0, W0 of K-tile 0 landed (this wave's share)
  bar_raw();
  if (wave >= 4) bar_raw();                            // stagger: waves 4-7 one barrier behind

  for (int kt = 0; kt < nk; ++kt) {
    const char* buf = smem + (kt & 1) * BUF;
    const bool more = kt + 1 < nk;
    // phase 1: quadrant (0,0)
    read_a(buf, 0);
    read_w(buf, 0);
    if (more) { issue(kt + 1, 0); asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); }   // W1(kt) landed
    else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    bar_raw();
    mma(0, 0);
    bar_raw();
    // phase 2: quadrant (0,1)
    read_w(buf, 1);
    if (more) { issue(kt + 1, 2); asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); }   // A1(kt) landed
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar_raw();
    mma(0, 1);
    bar_raw();
    // phase 3: quadrant (1,1)
    read_a(buf, 1);
    if (more) issue(kt + 1, 3);
    bar_raw();
    mma(1, 1);
    bar_raw();
    // phase 4: quadrant (1,0) on fragments already in registers
    if (more) { issue(kt + 1, 1); asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); }   // A0, W0(kt+1) landed
    bar_raw();
    mma(1, 0);
    bar_raw();
  }
  if (wave < 4) bar_raw();                             // rejoin the stagger

  epilogue256<EPI, 1>(p, acc, smem, m0, n0, tid, lane, wm, wn);
}

// ------------------------------------------------------------------------------------------------
// 256x256x64 tile, 8 waves, 8-phase schedule with a deep LDS-DMA pipeline (algo 5).
// Same quadrant decomposition and stagger as gemm8p_kernel, but every half-tile slot is refilled as soon as
// its last fragment read is two phases old, so four half-tiles (8 LDS-DMA per wave) stay in flight and each
// half-tile has four phases (~2k cycles) to land instead of one or two:
//   phase (reads)        issues           waits for (vmcnt 8 in steady state)
//   P1 q(0,0) (A0, W0)   W1 of tile k+1   W1(k)
//   P2 q(0,1) (W1)       A1 of tile k+1   A1(k)
//   P3 q(1,1) (A1)       A0 of tile k+2   -
//   P4 q(1,0) (-)        W0 of tile k+2   A0(k+1), W0(k+1)
// Operands are addressed through buffer descriptors (32-bit per-lane offsets, K offset in the scalar
// offset): rows past M / N and padded conv taps take an out-of-range offset and the hardware returns zeros,
// so neither tail clamping nor a zero page is needed.
constexpr unsigned OOB = 0x80000000u;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff, PDM_LDS void* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, lds, 16, (int)voff, soff, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
  const unsigned n = bytes >= 0x7fffffffLL ? 0x7fffffffu : (unsigned)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)n, 0x00020000);
}

// HN (half-N, N <= 128, SCHED 2 only): a 256 x 128 tile -- the W1 half is never loaded and only the qj = 0
// quadrants are computed (the decoder's 128-channel 512^2 convs would otherwise waste half of every 256 x 256
// tile or run on the 128-tile kernel); the epilogue is the 256-wide one, columns >= N are never stored.
// implicit-GEMM conv: byte offset of tap (dy, dx) of the output pixel packed in pix (b << 18 | y << 9 | x, -1 past
// M) in the NHWC source (nearest-upsampled by conv_up), OOB in the zero padding.  No division: 24-bit multiplies only
// (fits_rsrc: H, W <= 512, b < 8192, and every byte offset < 2^31, so the pixel index stays below 2^24).
__device__ __forceinline__ unsigned conv_off(const GemmArgs& p, int pix, int dy, int dx, unsigned sb) {
  // the decode of pix stays in the loop: hoisted per piece (y, x, b * H) it cost 16 more VGPRs and the 512-row tile
  // kernel spilled inside its K-loop (a scratch reload + vmcnt(0) drain per K-tile)
  asm volatile("" : "+v"(pix));
  const int yy = ((pix >> 9) & 511) + dy, xx = (pix & 511) + dx;
  if (pix < 0 || (unsigned)yy >= (unsigned)p.convH || (unsigned)xx >= (unsigned)p.convW) return OOB;
  const int sh = p.conv_up;
  const unsigned row = __umul24((unsigned)(pix >> 18), (unsigned)(p.convH >> sh)) + (unsigned)(yy >> sh);
  const unsigned px = __umul24(row, (unsigned)(p.convW >> sh)) + (unsigned)(xx >> sh);
  return __umul24(px, (unsigned)(p.convC * 2)) + sb;
}

template <int EPI, int CONV, int SCHED, int HN = 0>
__global__ __launch_bounds__(512, 1) void gemm8d_kernel(GemmArgs p, int tiles_n, int nwg) {
  static_assert(!HN || SCHED == 2, "the half-N tile exists in the SCHED 2 schedule only");
  constexpr int ROWB = 128;
  constexpr int HALF = 128 * ROWB;              // 16 KiB half-tile
  constexpr int BUF = 4 * HALF;                 // A0 A1 W0 W1
  enum { KA0 = 0, KA1 = 1, KW0 = 2, KW1 = 3 };
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  int bid = blockIdx.x;
  {
    const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
  }
  int tm, tn;
  if (p.raster > 0) {   // groups of `raster` row panels, column-major inside a group (L2 reuse of A and W)
    const int tiles_m = (p.M + BM2 - 1) / BM2;
    const int grp = bid / (p.raster * tiles_n);
    const int rows_in = min(p.raster, tiles_m - grp * p.raster);
    const int r = bid - grp * p.raster * tiles_n;
    tm = grp * p.raster + r % rows_in;
    tn = r / rows_in;
  } else {
    tm = bid / tiles_n;
    tn = bid - tm * tiles_n;
  }
  const int m0 = tm * BM2, n0 = tn * BN2;
  const int lm0 = (p.dbg_tile0 & 1) ? 0 : m0, ln0 = (p.dbg_tile0 & 1) ? 0 : n0;   // operand origin of the staging loads
  if (p.batch > 1) {
    const long long z = blockIdx.y;
    p.A1 += z * p.sA;
    p.W += z * p.sW;
    if (p.out_bf16) p.out_bf16 += z * p.sO;
    if (p.out_f32) p.out_f32 += z * p.sR;
  }
  const int ldw = p.ldw > 0 ? p.ldw : p.K;

  // descriptor extents (bytes) of the three operands
  long long a1_rows;
  if (CONV) a1_rows = (long long)(p.M / (p.convH * p.convW)) * (p.convH >> p.conv_up) * (p.convW >> p.conv_up);
  else if (p.a_rows_per_group > 0)
    a1_rows = (long long)((p.M - 1) / p.a_rows_per_group) * p.a_group_stride + p.a_rows_per_group;
  else a1_rows = p.M;
  const __amdgpu_buffer_rsrc_t ra1 = make_rsrc(p.A1, a1_rows * (CONV ? p.convC : p.lda1) * 2);
  const __amdgpu_buffer_rsrc_t ra2 = make_rsrc(p.A2 ? p.A2 : p.A1, p.A2 ? (long long)p.M * p.lda2 * 2 : 0);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.W, (long long)(p.N - 1) * ldw * 2 + (long long)p.K * 2);

  // per-lane offsets of this wave's two 1 KiB pieces (8 rows x 128 B) in each half (h) of A and W
  const int prow = lane >> 3, pch = lane & 7;
  unsigned a1off[2][2], a2off[2][2], woff[2][2];
  int cpix[2][2];   // conv: b << 18 | y << 9 | x of the piece row's output pixel, -1 past M (fits_rsrc: H, W <= 512)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 8 + prow;
    const unsigned sb = (unsigned)((pch ^ ((row >> 1) & 7)) * 16);   // logical chunk stored at physical pch
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int gm = lm0 + h * 128 + row;
      if constexpr (CONV) {
        if (gm < p.M) {
          const int hw = p.convH * p.convW, b = gm / hw, r = gm - b * hw, y = r / p.convW;
          cpix[h][i] = (b << 18) | (y << 9) | (r - y * p.convW);
        } else {
          cpix[h][i] = -1;
        }
        a1off[h][i] = sb;
        a2off[h][i] = 0;
      } else {
        const int gm1 = p.a_rows_per_group > 0 ? (gm / p.a_rows_per_group) * p.a_group_stride + gm % p.a_rows_per_group : gm;
        a1off[h][i] = gm < p.M ? (unsigned)gm1 * (unsigned)(p.lda1 * 2) + sb : OOB;
        a2off[h][i] = gm < p.M ? (unsigned)gm * (unsigned)(p.lda2 * 2) + sb : OOB;
        cpix[h][i] = 0;
      }
      const int gn = ln0 + h * 128 + row;
      woff[h][i] = gn < p.N ? (unsigned)gn * (unsigned)(ldw * 2) + sb : OOB;
    }
  }

  auto issue = [&](int kt, int kind) {
    const int k0 = kt * 64;
    char* dst = smem + (kt & 1) * BUF + kind * HALF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      PDM_LDS void* d = (PDM_LDS void*)(dst + (wave * 2 + i) * 1024);
      if (kind >= KW0) {
        dma16(rw, woff[kind - KW0][i], k0 * 2, d);
      } else if constexpr (CONV) {
        const int tap = k0 / p.convC, ci0 = k0 - tap * p.convC;
        const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
        dma16(ra1, conv_off(p, cpix[kind][i], dy, dx, a1off[kind][i]), ci0 * 2, d);
      } else {
        if (k0 < p.K1) dma16(ra1, a1off[kind][i], k0 * 2, d);
        else dma16(ra2, a2off[kind][i], (k0 - p.K1) * 2, d);
      }
    }
  };

  // fused-LayerNorm consumer: the tile's 256 row-statistics partials (<= 8 per row) are loaded before the first
  // operand DMA, so the prologue's vmcnt wait covers them, and merged into the epilogue's LDS row table right
  // after it -- their latency hides under the prologue instead of opening the epilogue (measured: the LN
  // consumer cost +19 us on qkv and +31 us on fc1 at the L/2 shapes when merged in the epilogue)
  const bool ln_pre = (EPI == EPI_BF16 || EPI == EPI_GELU) && p.ln_stats != nullptr && p.ln_ld <= 8;
  float2 lst[8];
  if (ln_pre && tid < 256) {
    const float2* st = reinterpret_cast<const float2*>(p.ln_stats) + (size_t)min(m0 + tid, p.M - 1) * p.ln_ld;
#pragma unroll
    for (int t = 0; t < 8; ++t) lst[t] = t < p.ln_ld ? st[t] : make_float2(0.f, 0.f);
  }
  // the same for the tile's bias and LN column sums (waves 4-7, one column each) -> COL_LDS, so no epilogue
  // opens with a global-load round trip
  float cb = 0.f, cc = 0.f;
  if (tid >= 256) {
    const int n = n0 + tid - 256;
    if (p.bias && n < p.N) cb = p.bias[n];
    if (epi_rowout(EPI) && p.ln_stats && n < p.N) cc = p.ln_colsum[n];   // staged even when ln_D > 2048
  }
  auto ln_prologue = [&]() {
    if (tid >= 256) {
      reinterpret_cast<float*>(smem + COL_LDS)[tid - 256] = cb;
      reinterpret_cast<float*>(smem + COL_LDS)[tid] = cc;   // colsum at +256
    }
    if (ln_pre && tid < 256)
      reinterpret_cast<float2*>(smem + EPI_LDS)[tid] = ln_from_partials(lst, p.ln_ld, p.ln_D, p.ln_eps, nullptr);
  };

  f32x4 acc[32];
#pragma unroll
  for (int f = 0; f < 32; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2];      // A fragments of the current A half: [mi][k-sub]
  bf16x8 wf[2][2][2];   // W fragments of both W halves: [qj][ni][k-sub]

  auto read_a = [&](const char* buf, int qi) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int row = wm * 64 + mi * 16 + (lane & 15);
        af[mi][ks] = *reinterpret_cast<const bf16x8*>(buf + qi * HALF + swz_off<64>(row, ks * 4 + (lane >> 4)));
      }
  };
  auto read_w = [&](const char* buf, int qj) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int row = wn * 32 + ni * 16 + (lane & 15);
        wf[qj][ni][ks] = *reinterpret_cast<const bf16x8*>(buf + (2 + qj) * HALF + swz_off<64>(row, ks * 4 + (lane >> 4)));
      }
  };
  // SCHED 1/2: the fragment reads of a phase are retired before its first barrier, so the MFMAs start on
  // data already in registers and a slot is free for refill one phase after its last read.
  auto lds_done = [&]() {
    if constexpr (SCHED != 0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto mma = [&](int qi, int qj) {
    if constexpr (SCHED == 0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          f32x4& c = acc[((qi * 2 + qj) * 2 + ni) * 4 + mi];
          c = mfma16x16x32(wf[qj][ni][ks], af[mi][ks], c);
        }
    __builtin_amdgcn_s_setprio(0);
  };

  const int nk = p.K / 64;
  if constexpr (HN) {
    // SCHED 2 with the W1 half dropped: phase A reads A0 W0 (quadrant (0,0)) and issues A1 of tile k+1, phase
    // B reads A1 (quadrant (1,0)) and issues A0 W0 of tile k+2; every wait leaves the 6 youngest LDS-DMA
    // (3 half-tiles) in flight.
    issue(0, KA0);
    issue(0, KW0);
    issue(0, KA1);
    if (nk > 1) {
      issue(1, KA0);
      issue(1, KW0);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    }
    ln_prologue();
    bar_raw();
    if (wave >= 4) bar_raw();
    for (int kt = 0; kt < nk; ++kt) {
      const char* buf = smem + (kt & 1) * BUF;
      const bool m1 = kt + 1 < nk, m2 = kt + 2 < nk;
      read_a(buf, 0);
      read_w(buf, 0);
      if (m1) { issue(kt + 1, KA1); lds_done(); asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); }   // A1(kt)
      else { lds_done(); asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
      bar_raw();
      mma(0, 0);
      bar_raw();
      read_a(buf, 1);
      if (m2) {
        issue(kt + 2, KA0);
        issue(kt + 2, KW0);
        lds_done();
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // A0 W0 (kt+1)
      } else {
        lds_done();
        if (m1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      }
      bar_raw();
      mma(1, 0);
      bar_raw();
    }
  } else if constexpr (SCHED == 2) {
    // 2 phases per K-tile: A (reads A0 W0 W1, quadrants (0,0) (0,1)) and B (reads A1, quadrants (1,0) (1,1)),
    // 32 MFMAs each.  Issue order: A0 W0 W1 of tile k+2 in B(k), A1 of tile k+1 in A(k); every wait leaves
    // the 8 youngest LDS-DMA (4 half-tiles) in flight.
    issue(0, KA0);
    issue(0, KW0);
    issue(0, KW1);
    issue(0, KA1);
    if (nk > 1) {
      issue(1, KA0);
      issue(1, KW0);
      issue(1, KW1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    }
    ln_prologue();
    bar_raw();
    if (wave >= 4) bar_raw();
    for (int kt = 0; kt < nk; ++kt) {
      const char* buf = smem + (kt & 1) * BUF;
      const bool m1 = kt + 1 < nk, m2 = kt + 2 < nk;
      // phase A
      read_a(buf, 0);
      read_w(buf, 0);
      read_w(buf, 1);
      if (m1) { issue(kt + 1, KA1); lds_done(); asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }   // A1(kt)
      else { lds_done(); asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
      bar_raw();
      mma(0, 0);
      mma(0, 1);
      bar_raw();
      // phase B
      read_a(buf, 1);
      if (m2) {
        issue(kt + 2, KA0);
        issue(kt + 2, KW0);
        issue(kt + 2, KW1);
        lds_done();
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // A0 W0 W1 (kt+1)
      } else {
        lds_done();
        if (m1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      }
      bar_raw();
      mma(1, 0);
      mma(1, 1);
      bar_raw();
    }
  } else {
    issue(0, KA0);
    issue(0, KW0);
    issue(0, KW1);
    issue(0, KA1);
    if (nk > 1) {
      issue(1, KA0);
      issue(1, KW0);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    ln_prologue();
    bar_raw();
    if (wave >= 4) bar_raw();                            // stagger: waves 4-7 one barrier behind

    for (int kt = 0; kt < nk; ++kt) {
      const char* buf = smem + (kt & 1) * BUF;
      const bool m1 = kt + 1 < nk, m2 = kt + 2 < nk;
      // P1: quadrant (0,0)
      read_a(buf, 0);
      read_w(buf, 0);
      lds_done();
      if (m1) { issue(kt + 1, KW1); asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }
      else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      bar_raw();
      mma(0, 0);
      bar_raw();
      // P2: quadrant (0,1)
      read_w(buf, 1);
      lds_done();
      if (m1) { issue(kt + 1, KA1); asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar_raw();
      mma(0, 1);
      bar_raw();
      // P3: quadrant (1,1)
      read_a(buf, 1);
      lds_done();
      if (m2) issue(kt + 2, KA0);
      bar_raw();
      mma(1, 1);
      bar_raw();
      // P4: quadrant (1,0) on fragments already in registers
      if (m2) { issue(kt + 2, KW0); asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }
      else if (m1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      bar_raw();
      mma(1, 0);
      bar_raw();
    }
  }
  if (wave < 4) bar_raw();                             // rejoin the stagger

  if (p.dbg_tile0 & 16) {   // timing experiment: no epilogue at all (the accumulators are kept live, nothing is written)
#pragma unroll
    for (int f = 0; f < 32; ++f) asm volatile("" ::"v"(acc[f]));
    return;
  }
  epilogue256<EPI, 1>(p, acc, smem, m0, n0, tid, lane, wm, wn, ln_pre, true);
}

// ------------------------------------------------------------------------------------------------
// Persistent 256 x 256 kernel (algo 11, the default for the U-ViT block GEMMs: bf16 / GELU outputs with or
// without the fused-LayerNorm consumer, and the bf16 residual epilogue with its LayerNorm partials).
//
// gemm8d's main loop (SCHED 2) runs unchanged, but a workgroup owns one CU for the whole launch and walks its
// XCD's tile range in a static round robin, and the LDS-DMA ring runs on across tile boundaries: the K-tiles are
// numbered continuously over the workgroup's tiles (ring slot = global K-tile & 1), so the last K-tile's phases
// already issue the next tile's K-tile 0 and the A0 W0 W1 halves of its K-tile 1 exactly as they would issue
// K-tiles of the same tile.  The next tile's main loop therefore starts on landed operands instead of an empty
// pipeline.  That needs an epilogue that leaves the ring alone, so nothing is staged through LDS:
//  * bf16 / GELU: the accumulator fragment holds 4 consecutive columns of one row per lane; two fragments 16
//    columns apart are converted to bf16 and exchanged between the lane rows {0,1} and {2,3} with
//    v_permlane16_swap, after which every lane holds 8 consecutive columns (16 bytes) of its row and stores them
//    with one buffer store (16 rows x 64 B per instruction);
//  * residual: the bf16 residual is loaded in that 16-byte layout (buffer loads, zeros out of range), swapped
//    back into the fragment layout, added in fp32 (acc + bias + residual, rounded once, as EPI_RES), and the
//    LayerNorm partials (sum, M2 about the 256-column group mean) of the rounded rows are reduced per wave
//    (permlane swaps across the 4 lane rows holding a row's columns) and across the 4 column waves in LDS.
// Small per-tile tables (the LN consumer's raw row partials, bias, LN column sums) are LDS-DMA'd for the next
// tile while the current epilogue runs.  Every store is a buffer store with out-of-range offsets dropped, so a
// lane issues the same number of VMEM ops on every tile; the first K-tile after an epilogue waits with the
// epilogue's E stores excluded from the count (they retire one phase later), so the stores overlap the next
// tile's first MFMAs.
constexpr int S_RING = 2 * 4 * 128 * 128;      // 128 KiB ring (as gemm8d)
constexpr int S_RAW = S_RING;                  // raw LN partials of a tile's 256 rows: 256 x ln_ld float2 (<= 16 KiB)
constexpr int S_LNROW = S_RAW + 256 * 8 * 8;   // merged (mean, rstd) per row (2 KiB)
constexpr int S_COL = S_LNROW + 256 * 8;       // bias [256] | LN colsum [256] (2 KiB)
constexpr int S_STAT = S_COL + 2 * 256 * 4;    // residual epilogue: per (row, column wave) sum / M2 (8 KiB)
constexpr int S_FLAG = S_STAT + 256 * 4 * 8;   // stream-K: the polled hand-off result, broadcast to the waves (16 B)
constexpr int S_SMEM = S_FLAG + 16;             // 156 KiB + 16 B
// MXFP8 operands (FP8 = 1, no stream-K): the E8M0 block scales of the ring's two K-tiles (A rows | W rows, 2 KiB
// per slot) take the stream-K flag's place; 160 KiB in all.  The centred LayerNorm's per-row table (bf16 hi / lo of
// mu_t - mean, 32 B per row) uses S_STAT, which only the residual epilogue needs otherwise.
constexpr int S_MXS = S_FLAG;
constexpr int S_SMEM_MX = S_MXS + 2 * 2048;

template <int N>
__device__ __forceinline__ void wait_vmcnt_n() {   // s_waitcnt vmcnt(N), N < 64
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  bf16x2 r;
  r[0] = (bf16)a;
  r[1] = (bf16)b;
  return __builtin_bit_cast(unsigned, r);
}
__device__ __forceinline__ float bf16lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

// sum over the 4 lanes l, l ^ 16, l ^ 32, l ^ 48 (the four 16-lane rows of one fragment column), in every lane
__device__ __forceinline__ float xrow_sum4(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// LDS accesses the compiler does not see: hipcc drains vmcnt before a visible LDS access while an LDS-DMA may be
// pending, which would wait for the epilogue's stores and the next tile's prefetch.  Reads are issued together
// with their lgkmcnt wait in ONE asm statement (early-clobber outputs): an asm output counts as written at the end
// of its statement, and hipcc does copy such registers right behind the statement (measured: a copy of a
// ds_read result before a separate wait read stale data).  The data read were retired by earlier counted waits
// + barriers.
__device__ __forceinline__ unsigned lds_addr(const void* p) { return (unsigned)(uintptr_t)(PDM_LDS const void*)p; }
// 8 x 16 B at base + {0, 64, 512, 576, 1024, 1088, 1536, 1600} (a lane's bias / LN-colsum fragments)
__device__ __forceinline__ void lds_rd_cols(const void* p, f32x4 (&b)[2][2], f32x4 (&c)[2][2]) {
  asm volatile(
      "ds_read_b128 %0, %8\n\tds_read_b128 %1, %8 offset:64\n\tds_read_b128 %2, %8 offset:512\n\t"
      "ds_read_b128 %3, %8 offset:576\n\tds_read_b128 %4, %8 offset:1024\n\tds_read_b128 %5, %8 offset:1088\n\t"
      "ds_read_b128 %6, %8 offset:1536\n\tds_read_b128 %7, %8 offset:1600\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(b[0][0]), "=&v"(b[0][1]), "=&v"(b[1][0]), "=&v"(b[1][1]), "=&v"(c[0][0]), "=&v"(c[0][1]), "=&v"(c[1][0]),
        "=&v"(c[1][1])
      : "v"(lds_addr(p))
      : "memory");
}
// 8 x 8 B at base + 8 * {0..7} (a row's raw LN partials)
__device__ __forceinline__ void lds_rd_raw(const void* p, f32x2 (&v)[8]) {
  asm volatile(
      "ds_read_b64 %0, %8\n\tds_read_b64 %1, %8 offset:8\n\tds_read_b64 %2, %8 offset:16\n\t"
      "ds_read_b64 %3, %8 offset:24\n\tds_read_b64 %4, %8 offset:32\n\tds_read_b64 %5, %8 offset:40\n\t"
      "ds_read_b64 %6, %8 offset:48\n\tds_read_b64 %7, %8 offset:56\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
      : "v"(lds_addr(p))
      : "memory");
}
// 8 x 8 B at base + {0, 128, 256, 384, 1024, 1152, 1280, 1408} (the (mean, rstd) of a lane's 8 rows)
__device__ __forceinline__ void lds_rd_rows(const void* p, f32x2 (&v)[8]) {
  asm volatile(
      "ds_read_b64 %0, %8\n\tds_read_b64 %1, %8 offset:128\n\tds_read_b64 %2, %8 offset:256\n\t"
      "ds_read_b64 %3, %8 offset:384\n\tds_read_b64 %4, %8 offset:1024\n\tds_read_b64 %5, %8 offset:1152\n\t"
      "ds_read_b64 %6, %8 offset:1280\n\tds_read_b64 %7, %8 offset:1408\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
      : "v"(lds_addr(p))
      : "memory");
}
// 4 x 8 B at base + {0, 8, 16, 24} (one row's per-wave (sum, M2) pairs)
__device__ __forceinline__ void lds_rd_stat2(const void* p, f32x2 (&v)[4]) {
  asm volatile(
      "ds_read_b64 %0, %4\n\tds_read_b64 %1, %4 offset:8\n\tds_read_b64 %2, %4 offset:16\n\t"
      "ds_read_b64 %3, %4 offset:24\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
      : "v"(lds_addr(p))
      : "memory");
}
__device__ __forceinline__ void lds_wr64(void* p, float2 v) {
  const f32x2 w = f32x2{v.x, v.y};
  asm volatile("ds_write_b64 %0, %1" ::"v"(lds_addr(p)), "v"(w) : "memory");
}
__device__ __forceinline__ void lds_wr128(void* p, i32x4 v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
// 8 x 16 B at base + {0, 512, 1024, 1536, 4096, 4608, 5120, 5632} (a lane's 8 rows of the centred-LN row table)
__device__ __forceinline__ void lds_rd_rowc(const void* p, i32x4 (&v)[8]) {
  asm volatile(
      "ds_read_b128 %0, %8\n\tds_read_b128 %1, %8 offset:512\n\tds_read_b128 %2, %8 offset:1024\n\t"
      "ds_read_b128 %3, %8 offset:1536\n\tds_read_b128 %4, %8 offset:4096\n\tds_read_b128 %5, %8 offset:4608\n\t"
      "ds_read_b128 %6, %8 offset:5120\n\tds_read_b128 %7, %8 offset:5632\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
      : "v"(lds_addr(p))
      : "memory");
}
// stream-K diagnostics (pdm_set_gemm_tuning bit 8): tails run, hand-offs not taken, summed poll time
__device__ unsigned long long g_sk_stats[4];
// -DPDM_G8S_SEG diagnostic builds: shader cycles per main-loop segment, summed over workgroups for wave 0 [0..11] and
// wave 4 [12..23] (A: reads, refill issue, vmcnt wait, barrier, MFMAs, barrier; B: the same) + workgroups [24]
__device__ unsigned long long g_seg_stats[25];

// a copy of x the compiler cannot see through: values derived from it are computed where they are used instead of
// being hoisted and held in registers across loops
__device__ __forceinline__ int opaque_i(int x) {
  asm volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// lanes of rows {0,1} and {2,3} exchange: returns (a', b') with a' = [a.r0, b.r0, a.r2, b.r2], b' = [a.r1, b.r1,
// a.r3, b.r3] (16-lane rows r0..r3); its own inverse
__device__ __forceinline__ void pl16swap(unsigned& a, unsigned& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  a = r[0];
  b = r[1];
}

// MXO = 1 (bf16 / GELU only): the output is the MXFP8 copy alone (out_fp8 + out_scale, no bf16 rows): the H/4 bf16
// fc1 whose GELU epilogue emits the fp8 fc2 operand (capi.hip run_block8)
// Grouped launch (nt0 < ntiles): tiles [0, nt0) are problem p, [nt0, ntiles) problem p2 -- two GEMMs of the same
// N / K / epilogue whose operands, rows and outputs differ (the t2i image- and mask-stream block Linears of one layer,
// capi.hip run_block16_pair), walked as one tile list so a layer's two small launches fill the CUs together.  Every
// per-problem field is read through the tile's view (TV); the shared ones (N, K, strides, flags) come from p.
struct TV {
  const bf16* A1;
  const bf16* A2;
  const bf16* W;
  const float* bias;
  const float* ln_stats;
  const float* ln_colsum;
  bf16* out;
  const bf16* res;
  float* st;
  int M;
};
__host__ __device__ __forceinline__ TV view_of(const GemmArgs& q) {
  return TV{q.A1, q.A2 ? q.A2 : q.A1, q.W, q.bias, q.ln_stats, q.ln_colsum, q.out_bf16, q.res_in, q.stats_out, q.M};
}
// the view of a tile's problem: p's fields, or the second problem's (t2) -- a field-wise select on a small by-value
// struct (a whole second GemmArgs bound by reference made hipcc copy both to scratch: 784 B per lane)
__device__ __forceinline__ TV tile_view(const GemmArgs& p, const TV& t2, bool second) {
  TV v;
  v.A1 = second ? t2.A1 : p.A1;
  v.A2 = second ? t2.A2 : (p.A2 ? p.A2 : p.A1);
  v.W = second ? t2.W : p.W;
  v.bias = second ? t2.bias : p.bias;
  v.ln_stats = second ? t2.ln_stats : p.ln_stats;
  v.ln_colsum = second ? t2.ln_colsum : p.ln_colsum;
  v.out = second ? t2.out : p.out_bf16;
  v.res = second ? t2.res : p.res_in;
  v.st = second ? t2.st : p.stats_out;
  v.M = second ? t2.M : p.M;
  return v;
}

// GRP = 1: the grouped kernel (a second problem p2 from tile nt0 on, gemm8g_kernel); GRP = 0 compiles the one-problem
// kernel with every view resolved to p at compile time
//
// SK = 1: stream-K (one problem).  A partly filled last wave of tiles (the U-ViT's N = 1024 Linears at 100 rows:
// 404 tiles on 256 CUs = a makespan of 2 tiles for 1.58 tiles of work) is removed by giving every workgroup an equal
// share of the group's K-steps instead of whole tiles.  Workgroup j of an XCD group owns the K-step range
// [B(j), B(j+1)) of the group's tile order (tile-major, 64-deep K-steps; boundaries on even K-steps), i.e. the tail
// (K-steps s..nk) of a tile T0 whose head (0..s) the group's workgroup j-1 owns, whole tiles, and the head of a tile
// T1 whose tail workgroup j+1 owns.  It runs them in the order head, whole tiles, tail:
//  * head: the K-steps 0..s of T1 run as usual, then the fp32 accumulators go to this workgroup's slab (write-through
//    sc1 stores, overlapped with the next segment's first K-steps like an epilogue's stores) and a flag is raised
//    once every wave's stores have retired (one lane, relaxed agent-scope store behind a workgroup barrier);
//  * tail: every wave drains, one lane polls the predecessor's flag (sc1 loads, bounded by 20 us), the waves load its
//    slab straight into the accumulators (sc1 loads) and CONTINUE the MFMA chain from K-step s -- the same sequence
//    of accumulations as one workgroup running the whole tile, so the result is bit-identical to SK = 0 and to the
//    batch-size-independent tile arithmetic the sampler relies on.  Should the flag not come (the producer not yet
//    resident, e.g. beside another lane's kernel), the tail is recomputed from K-step 0 instead: no workgroup ever
//    waits unboundedly on another, and both branches give the same bits.
// The producer's head runs first and needs nothing, so the flag is normally up long before the consumer's tail
// (margin = share - nk K-steps); gemm_launch takes SK only where every workgroup's share is >= nk + 4 K-steps.
//
// FP8 = 1: MXFP8 operands (GemmArgs::fp8; gemm_mx_kernel's math on this ring): a K-tile is 128 e4m3 = the same
// 128-byte rows, staged, swizzled and read exactly as the bf16 K-tile, one v_mfma_scale_f32_16x16x128_f8f6f4 per
// fragment pair instead of two bf16 MFMAs, plus one 4-byte-per-lane LDS-DMA of E8M0 scales per wave and K-tile
// (waves 0-3: the tile's A rows, 4-7: its W rows) issued with A0 W0 W1, so the ring waits count 9 ops instead of 8.
// bf16 epilogue only, with the centred LayerNorm consumer (ln_gcol: acc += sum_t (mu_t - mean) c_t as one bf16 MFMA
// per accumulator, as gemm_mx_kernel) or the plain one: the U-ViT-H/4 qkv.
// DUAL = 0: no split-K second A operand (A2 / K1 < K: the long-skip concat of skip_linear only): the refill issue then
// has no per-piece operand test and descriptor select -- measured 4-7 % on the single-operand Linears at 50 rows
// (profiles/r06n: proj 39.5 -> 37.8, fc1 131.7 -> 123.7, fc2 99.2 -> 94.8 us), whose load segments are issue-bound
template <int EPI, int MXO, int GRP, int SK = 0, int FP8 = 0, int DUAL = 1>
__device__ __forceinline__ void gemm8s_body(const GemmArgs& p, int tiles_n, int ntiles, const TV& p2, int nt0) {
  static_assert(EPI == EPI_BF16 || EPI == EPI_GELU || EPI == EPI_RES, "persistent kernel epilogues");
  static_assert(!FP8 || ((EPI == EPI_BF16 || EPI == EPI_RES) && !MXO && !GRP && !SK),
                "MXFP8 operands: one problem, the bf16 or the bf16-residual epilogue");
  static_assert(!MXO || EPI != EPI_RES, "MXFP8 output: bf16 / GELU epilogues");
  static_assert(!SK || !GRP, "stream-K: one problem");
  constexpr int ROWB = 128;
  constexpr int HALF = 128 * ROWB;
  constexpr int BUF = 4 * HALF;
  enum { KA0 = 0, KA1 = 1, KW0 = 2, KW1 = 3 };
  // VMEM ops every lane issues in an epilogue after its last wait: 16 output stores (+ 1 LN-partial store; MXO:
  // 16 fp8 row stores + 4 scale-byte stores)
  constexpr int E = EPI == EPI_RES ? 17 : MXO ? 20 : 16;
  constexpr int ES = FP8 ? 1 : 2;   // operand bytes per element
  constexpr int RW = FP8 ? 9 : 8;   // ring VMEM ops a lane leaves in flight at a phase wait (FP8: + the scale piece)

  typedef int v8i __attribute__((ext_vector_type(8)));
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int g4 = lane >> 4, r16 = lane & 15;

  // this workgroup's tiles: the XCD label x = blockIdx % 8 owns a contiguous range of the tile order (gemm8d's
  // bijective remap), walked by its nx workgroups round robin
  const int G = gridDim.x, x = blockIdx.x & 7, jw = blockIdx.x >> 3;
  const int q8 = ntiles >> 3, r8 = ntiles & 7;
  const int tstart = x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8;
  const int tcnt = q8 + (x < r8 ? 1 : 0);
  const int nx = (G >> 3) + (x < (G & 7) ? 1 : 0);
  const int nk = p.K / (FP8 ? 128 : 64);   // >= 4 (gemm_launch: fits_8s / fits_8s_mx)
  // segments: SK = 0 the tiles tstart + jw + i * nx (whole); SK = 1 [head of tile ht] [whole tiles tf0 ..] [tail]
  int ntl;
  int ht = 0, hke = 0, tf0 = 0, nf = 0, tt = 0, tkb = 0;
  bool has_head = false, has_tail = false;
  if constexpr (SK) {
    const long long I = (long long)tcnt * nk;
    auto bnd = [&](int j) {   // boundary j of the group's K-step range, on an even K-step, no piece shorter than 2
      const long long b = I * j / nx;
      int t = (int)(b / nk), o = (int)(b - (long long)t * nk);
      o &= ~1;
      if (nk - o < 2) {
        o = 0;
        ++t;
      }
      return t * nk + o;
    };
    const int sa = bnd(jw), sb = bnd(jw + 1);
    const int ta = sa / nk, oa = sa - ta * nk, tb = sb / nk, ob = sb - tb * nk;
    has_tail = oa > 0;
    tt = ta;
    tkb = oa;
    tf0 = has_tail ? ta + 1 : ta;
    nf = tb - tf0;
    has_head = ob > 0;
    ht = tb;
    hke = ob;
    ntl = (has_head ? 1 : 0) + nf + (has_tail ? 1 : 0);
  } else {
    ntl = tcnt > jw ? (tcnt - jw + nx - 1) / nx : 0;
  }
  if (ntl == 0) return;
  // segment i: group-global tile u, K-steps [kb, ke), kind 0 whole / 1 head (-> slab) / 2 tail (<- slab)
  auto seg = [&](int i, int& u, int& kb_, int& ke_, int& kd) {
    if constexpr (SK) {
      const int j = i - (has_head ? 1 : 0);
      if (has_head && i == 0) {
        u = tstart + ht; kb_ = 0; ke_ = hke; kd = 1;
      } else if (j < nf) {
        u = tstart + tf0 + j; kb_ = 0; ke_ = nk; kd = 0;
      } else {
        u = tstart + tt; kb_ = tkb; ke_ = nk; kd = 2;
      }
    } else {
      u = tstart + jw + i * nx; kb_ = 0; ke_ = nk; kd = 0;
    }
  };
  auto tile_mn = [&](int u, int& m0_, int& n0_, bool& second) {
    second = GRP && u >= nt0;
    if (second) u -= nt0;
    const int tiles_m = ((GRP && second ? p2.M : p.M) + BM2 - 1) / BM2;
    int tm, tn;
    if (p.raster > 0) {
      const int grp = u / (p.raster * tiles_n);
      const int rows_in = min(p.raster, tiles_m - grp * p.raster);
      const int r = u - grp * p.raster * tiles_n;
      tm = grp * p.raster + r % rows_in;
      tn = r / rows_in;
    } else {
      tm = u / tiles_n;
      tn = u - tm * tiles_n;
    }
    m0_ = tm * BM2;
    n0_ = tn * BN2;
  };

  // operand descriptors of one tile, based at its first row / column: rows past M (N) lie past num_records and
  // come back as zeros, so the per-lane offsets below are the same for every tile
  const int ldw = p.ldw > 0 ? p.ldw : p.K;
  __amdgpu_buffer_rsrc_t ra1, ra2, rw;
  // FP8: this wave's scale piece -- A rows (waves 0-3) or W rows (4-7) (wave & 3) * 64 + lane of the tile, zero past
  // M / N (an E8M0 byte of 0xff would be NaN)
  const bool s_is_a = wave < 4;
  const int srow = (wave & 3) * 64 + lane;
  unsigned soff = OOB;
  auto set_tile = [&](const TV& v, int m0_, int n0_) {
    ra1 = make_rsrc(reinterpret_cast<const char*>(v.A1) + (size_t)m0_ * p.lda1 * ES, (long long)(v.M - m0_) * p.lda1 * ES);
    ra2 = make_rsrc(reinterpret_cast<const char*>(v.A2) + (size_t)m0_ * p.lda1 * ES, (long long)(v.M - m0_) * p.lda1 * ES);
    rw = make_rsrc(reinterpret_cast<const char*>(v.W) + (size_t)n0_ * ldw * ES,
                   (long long)(p.N - n0_ - 1) * ldw * ES + (long long)p.K * ES);
    if constexpr (FP8)
      soff = s_is_a ? (m0_ + srow < v.M ? (unsigned)(m0_ + srow) * 4u : OOB)
                    : (n0_ + srow < p.N ? (unsigned)(n0_ + srow) * 4u : OOB);
  };
  // output / residual / partials descriptors of the current tile's problem (rebuilt per tile: scalar work)
  __amdgpu_buffer_rsrc_t rout, rres, rst;
  const __amdgpu_buffer_rsrc_t rsc =
      make_rsrc(MXO ? (const void*)p.out_scale : (const void*)p.W, MXO ? (long long)((p.N + 127) >> 7) * p.out_scale_ld * 4 : 0);
  const bool ln = epi_rowout(EPI) && p.ln_stats != nullptr;
  const bool stats = EPI == EPI_RES && p.stats_out != nullptr;
  auto set_out = [&](const TV& v) {
    rout = MXO ? make_rsrc(p.out_fp8, (long long)v.M * p.ldo8) : make_rsrc(v.out, (long long)v.M * p.ldo * 2);
    rres = make_rsrc(EPI == EPI_RES && p.accumulate ? (const void*)v.res : (const void*)v.out,
                     EPI == EPI_RES && p.accumulate ? (long long)v.M * p.ldri * 2 : 0);
    rst = make_rsrc(stats ? (const void*)v.st : (const void*)v.W, stats ? (long long)v.M * p.stats_ld * 8 : 0);
  };

  // per-lane offsets (tile relative) of this wave's two 1 KiB pieces (8 rows x 128 B) in each half (h) of A and W
  const int prow = lane >> 3, pch = lane & 7;
  unsigned aoff[2][2], woff[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 8 + prow;
    const unsigned sb = (unsigned)((pch ^ ((row >> 1) & 7)) * 16);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      aoff[h][i] = (unsigned)(h * 128 + row) * (unsigned)(p.lda1 * ES) + sb;
      woff[h][i] = (unsigned)(h * 128 + row) * (unsigned)(ldw * ES) + sb;
    }
  }
  auto issue = [&](int slot, int kt, int kind) {
    const int k0 = kt * 64;
    char* dst = smem + slot * BUF + kind * HALF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      PDM_LDS void* d = (PDM_LDS void*)(dst + (wave * 2 + i) * 1024);
      if (kind >= KW0) dma16(rw, woff[kind - KW0][i], k0 * 2, d);
      else if (!DUAL || k0 < p.K1) dma16(ra1, aoff[kind][i], k0 * 2, d);
      else dma16(ra2, aoff[kind][i], (k0 - p.K1) * 2, d);
    }
  };
  // FP8: the E8M0 scales of K-tile kt into ring slot `slot` (one 4-byte piece per lane: 256 rows per wave group)
  const __amdgpu_buffer_rsrc_t rsa =
      make_rsrc(FP8 ? (const void*)p.a_scale : (const void*)p.W, FP8 ? (long long)nk * p.a_scale_ld * 4 : 0);
  const __amdgpu_buffer_rsrc_t rsw =
      make_rsrc(FP8 ? (const void*)p.w_scale : (const void*)p.W, FP8 ? (long long)nk * p.w_scale_ld * 4 : 0);
  auto issue_scales = [&](int slot, int kt) {
    if constexpr (FP8) {
      PDM_LDS void* d = (PDM_LDS void*)(smem + S_MXS + slot * 2048 + (s_is_a ? 0 : 1024) + (wave & 3) * 256);
      if (s_is_a) __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, d, 4, (int)soff, kt * p.a_scale_ld * 4, 0, 0);
      else __builtin_amdgcn_raw_ptr_buffer_load_lds(rsw, d, 4, (int)soff, kt * p.w_scale_ld * 4, 0, 0);
    }
  };
  // a tile's small tables -> LDS by buffer LDS-DMA (zeros past M / N; hipcc orders LDS reads behind these without
  // draining vmcnt, unlike the global-address form): the raw LN partials of its 256 rows (contiguous in
  // ln_stats), bias, LN column sums
  auto issue_tables = [&](const TV& v, int m0_, int n0_) {
    if (ln) {
      const int pieces = p.ln_ld * 2;   // KiB
      const __amdgpu_buffer_rsrc_t rr = make_rsrc(v.ln_stats + (size_t)m0_ * p.ln_ld * 2, (long long)(v.M - m0_) * p.ln_ld * 8);
      for (int pc = wave; pc < pieces; pc += 8)
        dma16(rr, (unsigned)(pc * 1024 + lane * 16), 0, (PDM_LDS void*)(smem + S_RAW + pc * 1024));
      if (wave == 7)
        dma16(make_rsrc(v.ln_colsum + n0_, (long long)(p.N - n0_) * 4), (unsigned)(lane * 16), 0,
              (PDM_LDS void*)(smem + S_COL + 1024));
    }
    if (wave == 6)   // no bias: an empty descriptor stages zeros, so the epilogues add it unconditionally
      dma16(v.bias ? make_rsrc(v.bias + n0_, (long long)(p.N - n0_) * 4) : make_rsrc(p.W, 0), (unsigned)(lane * 16), 0,
            (PDM_LDS void*)(smem + S_COL));
  };

  bf16x8 af[4][2];
  bf16x8 wf[2][2][2];
  auto read_a = [&](const char* buf, int qi) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int row = wm * 64 + mi * 16 + r16;
        af[mi][ks] = *reinterpret_cast<const bf16x8*>(buf + qi * HALF + swz_off<64>(row, ks * 4 + g4));
      }
  };
  auto read_w = [&](const char* buf, int qj) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int row = wn * 32 + ni * 16 + r16;
        wf[qj][ni][ks] = *reinterpret_cast<const bf16x8*>(buf + (2 + qj) * HALF + swz_off<64>(row, ks * 4 + g4));
      }
  };
  // FP8: the same chunks read straight into 8-VGPR operands (the scaled MFMA takes 32 bytes per lane; two bf16x8
  // halves would need copies into adjacent registers)
  v8i af8[4], wf8[2][2];
  auto frag8 = [&](v8i& dst, const char* base, int row) {
    i32x4* h = reinterpret_cast<i32x4*>(&dst);
    h[0] = *reinterpret_cast<const i32x4*>(base + swz_off<64>(row, g4));
    h[1] = *reinterpret_cast<const i32x4*>(base + swz_off<64>(row, 4 + g4));
  };
  auto read_a8 = [&](const char* buf, int qi) {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) frag8(af8[mi], buf + qi * HALF, wm * 64 + mi * 16 + r16);
  };
  auto read_w8 = [&](const char* buf) {
#pragma unroll
    for (int qj = 0; qj < 2; ++qj)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) frag8(wf8[qj][ni], buf + (2 + qj) * HALF, wn * 32 + ni * 16 + r16);
  };
  auto lds_done = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  f32x4 acc[32];
  auto mma = [&](int qi, int qj) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          f32x4& c = acc[((qi * 2 + qj) * 2 + ni) * 4 + mi];
          c = mfma16x16x32(wf[qj][ni][ks], af[mi][ks], c);
        }
    __builtin_amdgcn_s_setprio(0);
  };
  // FP8: a lane's packed E8M0 bytes (gemm_mx_kernel's read_scales): sa[qi] byte mi, sw byte qj * 2 + ni, each the
  // lane's k-block g4 of its row
  unsigned sa[2] = {0u, 0u}, sw = 0u;
  auto read_scales = [&](int slot) {
    const unsigned* sl = reinterpret_cast<const unsigned*>(smem + S_MXS + slot * 2048);
#pragma unroll
    for (int qi = 0; qi < 2; ++qi) {
      unsigned v = 0;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) v |= ((sl[qi * 128 + wm * 64 + mi * 16 + r16] >> (8 * g4)) & 0xffu) << (8 * mi);
      sa[qi] = v;
    }
    unsigned v = 0;
#pragma unroll
    for (int qj = 0; qj < 2; ++qj)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
        v |= ((sl[256 + qj * 128 + wn * 32 + ni * 16 + r16] >> (8 * g4)) & 0xffu) << (8 * (qj * 2 + ni));
    sw = v;
    asm volatile("" : "+v"(sa[0]), "+v"(sa[1]), "+v"(sw));
  };
  // FP8: one scaled MFMA per fragment pair (the lane's 32-byte fragments = chunks g4 and 4 + g4 of its row)
  auto mma8 = [&](auto qic, auto qjc) {
    constexpr int qi = decltype(qic)::value, qj = decltype(qjc)::value;
    __builtin_amdgcn_s_setprio(1);
    static_for<2>([&](auto nic) {
      constexpr int ni = decltype(nic)::value;
      static_for<4>([&](auto mic) {
        constexpr int mi = decltype(mic)::value;
        f32x4& c = acc[((qi * 2 + qj) * 2 + ni) * 4 + mi];
        c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wf8[qj][ni], af8[mi], c, 0, 0, qj * 2 + ni, sw, mi,
                                                             sa[qi]);
        asm volatile("" : "+v"(c));   // keep the MFMA in this phase (as gemm_mx_kernel)
      });
    });
    __builtin_amdgcn_s_setprio(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  int m0, n0;
  bool sec;
  int u0, kb, ke, kind;
  seg(0, u0, kb, ke, kind);
  tile_mn(u0, m0, n0, sec);
  TV cv = tile_view(p, p2, GRP && sec), nv = cv;
  set_tile(cv, m0, n0);
  set_out(cv);   // one problem: the output descriptors are built once (grouped: again per tile)
  // prologue of the first segment: tables, K-tile kb, A0 W0 W1 of K-tile kb+1; the wait retires the tables and
  // A0 W0 W1(kb)
  issue_tables(cv, m0, n0);
  issue_scales(0, kb);
  issue(0, kb, KA0);
  issue(0, kb, KW0);
  issue(0, kb, KW1);
  issue(0, kb, KA1);
  issue_scales(1, kb + 1);
  issue(1, kb + 1, KA0);
  issue(1, kb + 1, KW0);
  issue(1, kb + 1, KW1);
  wait_vmcnt_n<RW>();
  bar_raw();

#ifdef PDM_G8S_CLK
  // diagnostic builds only: the in-kernel clock (shader-clock ticks / 100 MHz real-time ticks, summed over workgroups
  // into g_sk_stats[0..2], read by pdm_gemm_sk_stats; MI355X_MICROARCH DVFS item 6; tools/g8s_clock.py)
  const unsigned long long clk_t0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();
#endif
  int g = 0;                  // K-steps run so far: the ring slot of the next one is g & 1
#if defined(PDM_G8S_SEG) || defined(PDM_G8S_ESEG)
  unsigned seg_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif
  bool pub_pending = false;   // SK: this workgroup's head slab stored, its flag not yet raised
  // Ordering of the hand-off (relaxed atomics by design): publish() runs only after EVERY wave of this
  // workgroup has drained its slab stores (wait_vmcnt_n<0> + barrier in the tail branch below; the stores are sc1
  // write-through, so vmcnt 0 means they reached this XCD's L2), and the consumer is workgroup blockIdx + 8, which
  // the round-robin dispatch places on the SAME XCD (blockIdx % 8) and hence the same L2; it polls with agent-scope
  // loads and reads the slab with sc1 (L1-bypassing) loads after a barrier.  An __ATOMIC_RELEASE store at agent scope
  // would add an L2 writeback (buffer_wbl2) of every dirty line for other XCDs that never read the slab.  If the
  // workgroup -> XCD mapping ever changes, switch to release / acquire.  Off by default (pdm_set_gemm_sk).
  auto publish = [&]() {
    if (tid == 0) __hip_atomic_store(p.sk_flags + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pub_pending = false;
  };
  for (int it = 0; it < ntl; ++it) {
    const bool has_next = it + 1 < ntl;
    int m0n = 0, n0n = 0, kbn = 0, ken = 0, kindn = 0;
    if (has_next) {
      bool secn;
      int un;
      seg(it + 1, un, kbn, ken, kindn);
      tile_mn(un, m0n, n0n, secn);
      if constexpr (GRP) nv = tile_view(p, p2, secn);   // one problem: nv == cv throughout
    }
#pragma unroll
    for (int f = 0; f < 32; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the previous segment's epilogue stores (E per lane; a head's slab: 32) are younger than the ring loads the
    // first K-tile waits for
    bool after_epi = it > 0;
    const bool after_slab = SK && it == 1 && has_head;
    if constexpr (SK) {
      if (kind == 2) {
        // tail: every wave drains (ring prefetch of this tile, the previous epilogue's / slab's stores), so the own
        // head's flag can go up now; then take over the predecessor's accumulators
        wait_vmcnt_n<0>();
        bar_raw();
        if (pub_pending) publish();
        if (tid == 0) {
          const unsigned* fl = p.sk_flags + blockIdx.x - 8;
          const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
          unsigned ok = 0;
          for (; !(p.dbg_tile0 & 128);) {   // dbg bit 7 (tests): never take the hand-off, recompute the tile
            if (__hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
              ok = 1;
              break;
            }
            if (__builtin_amdgcn_s_memrealtime() - t0 > 2000ull) break;   // 20 us (100 MHz)
            __builtin_amdgcn_s_sleep(2);
          }
          if (p.dbg_tile0 & 256) {   // diagnostics: tails, hand-offs not taken, poll time (10 ns ticks)
            atomicAdd(&g_sk_stats[0], 1ull);
            if (!ok) atomicAdd(&g_sk_stats[1], 1ull);
            atomicAdd(&g_sk_stats[2], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - t0));
          }
          asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(lds_addr(smem + S_FLAG)), "v"(ok) : "memory");
        }
        bar_raw();
        unsigned okv;
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(okv) : "v"(lds_addr(smem + S_FLAG)) : "memory");
        if (p.dbg_tile0 & 512) {   // timing experiment: the hand-off without its slab traffic (wrong results)
        } else if (__builtin_amdgcn_readfirstlane(okv)) {
          // sc1 loads (L1 bypassed) of the sc1-stored slab, behind the polling wave's match + the barrier
          const __amdgpu_buffer_rsrc_t rsl = make_rsrc(p.sk_slab + (size_t)(blockIdx.x - 8) * 65536, 262144);
#pragma unroll
          for (int f = 0; f < 32; ++f) {
            const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsl, opaque_i(tid) * 16, f * 8192, 16);
            acc[f] = __builtin_bit_cast(f32x4, v);
          }
          // consume them here: the compiler's own waits for these loads then sit in this branch, not in front of
          // every segment's first MFMAs (its wait tracking merges the branches)
#pragma unroll
          for (int f = 0; f < 32; ++f) asm volatile("" : "+v"(acc[f]));
        } else {
          // no hand-off: the whole tile here.  The ring's K-tiles kb, kb+1 have landed (drained above) and nobody
          // reads them: re-prime the same slots with K-tiles 0, 1 as the kernel prologue does
          kb = 0;
          issue(g & 1, 0, KA0);
          issue(g & 1, 0, KW0);
          issue(g & 1, 0, KW1);
          issue(g & 1, 0, KA1);
          issue((g + 1) & 1, 1, KA0);
          issue((g + 1) & 1, 1, KW0);
          issue((g + 1) & 1, 1, KW1);
          wait_vmcnt_n<8>();
          bar_raw();
        }
        after_epi = false;
      }
    }
    if (wave >= 4) bar_raw();        // stagger: waves 4-7 one barrier behind
#ifdef PDM_G8S_DIAG
    // diagnostic builds only (tools/build_variant.sh TAG -DPDM_G8S_DIAG=bits, tools/g8s_diag.py): bits 1 / 2 / 4 drop
    // the main loop's LDS-DMA refills / fragment reads / MFMAs (wrong results; timing of what bounds the loop)
    constexpr bool d_nodma = PDM_G8S_DIAG & 1, d_noread = PDM_G8S_DIAG & 2, d_nomma = PDM_G8S_DIAG & 4;
#else
    constexpr bool d_nodma = false, d_noread = false, d_nomma = false;
#endif
#ifdef PDM_G8S_SEG
    unsigned long long seg_t = __builtin_amdgcn_s_memtime();
    auto seg = [&](int i) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      seg_acc[i] += (unsigned)(t - seg_t);
      seg_t = t;
    };
#else
    auto seg = [](int) {};
#endif
    // one K-tile (two phases); ST = the steady state kb < kt < ke - 2 (not a segment's first K-tile, K-tiles g+1 and
    // g+2 in this segment), where every test below folds at compile time: the loading wave's segment is issue-bound,
    // so its branches and selects cost time (the first and the last two K-tiles keep the general form)
    auto ktile = [&](const int kt, auto stc) {
      constexpr bool ST = decltype(stc)::value;
      const int slot = g & 1;
      const char* buf = smem + slot * BUF;
      const bool first = !ST && kt == kb && after_epi;
      const bool m1 = ST || kt + 1 < ke || has_next;   // K-tile g+1 exists (this segment's kt+1 or the next one's kbn)
      const bool m2 = ST || kt + 2 < ke || has_next;   // K-tile g+2 (segments >= 2 K-tiles: the next one's kbn + {0, 1})
      // phase A: quadrants (0,0) (0,1); issues A1 of K-tile g+1
      if constexpr (FP8) {
        read_a8(buf, 0);
        read_w8(buf);
        read_scales(slot);
      } else if (!d_noread) {
        read_a(buf, 0);
        read_w(buf, 0);
        read_w(buf, 1);
      }
      // a phase's refills issue behind its fragment reads and before their lgkmcnt wait: they write ring halves no
      // wave reads in this phase, and their issue (the TA takes one 1 KiB piece at a time) overlaps the reads'
      // latency (L/2 bench 63.7 -> 64.5 img/s same box, profiles/r06q; issued before the reads: 63.6)
      seg(0);
      if (m1) {
        if (!d_nodma) issue(slot ^ 1, ST || kt + 1 < ke ? kt + 1 : kbn, KA1);
        lds_done();
        seg(1);
        if (first && after_slab) wait_vmcnt_n<8 + 32>();
        else if (first) wait_vmcnt_n<RW + E>();
        else wait_vmcnt_n<RW>();
      } else {
        lds_done();
        wait_vmcnt_n<0>();
      }
      seg(2);
      bar_raw();
      seg(3);
      if constexpr (FP8) {
        mma8(I0{}, I0{});
        mma8(I0{}, I1{});
      } else if (!d_nomma) {
        mma(0, 0);
        mma(0, 1);
      }
      seg(4);
      bar_raw();
      seg(5);
      // phase B: quadrants (1,0) (1,1); issues A0 W0 W1 of K-tile g+2 (the next segment's from kt = ke-2 on)
      if (!ST && kt == ke - 2 && has_next) set_tile(nv, m0n, n0n);
      const int k2 = ST || kt + 2 < ke ? kt + 2 : kbn + (kt + 2 - ke);
      if constexpr (FP8) read_a8(buf, 1);
      else if (!d_noread) read_a(buf, 1);
      seg(6);
      if (m2) {
        issue_scales(slot, k2);
        if (!d_nodma) {
          issue(slot, k2, KA0);
          issue(slot, k2, KW0);
          issue(slot, k2, KW1);
        }
        lds_done();
        seg(7);
        if (first && after_slab) wait_vmcnt_n<8 + 32>();
        else if (first) wait_vmcnt_n<RW + E>();
        else wait_vmcnt_n<RW>();
      } else {
        lds_done();
        if (m1) wait_vmcnt_n<2>();
      }
      seg(8);
      bar_raw();
      seg(9);
      // SK: the head slab's stores are older than everything this K-tile's phase-A wait left in flight, and by this
      // barrier every wave (4-7 one barrier behind) has passed that wait: raise the flag
      if constexpr (SK) {
        if (pub_pending && kt == kb + 1) publish();
      }
      if constexpr (FP8) {
        mma8(I1{}, I0{});
        mma8(I1{}, I1{});
      } else if (!d_nomma) {
        mma(1, 0);
        mma(1, 1);
      }
      seg(10);
      bar_raw();
      seg(11);
    };
    using STF = std::false_type;
    using STT = std::true_type;
    if constexpr (SK) {
      for (int kt = kb; kt < ke; ++kt, ++g) ktile(kt, STF{});
    } else {
      int kt = kb;
      ktile(kt, STF{});   // nk >= 4 (fits_8s / fits_8s_mx): the first K-tile, then the steady ones
      ++kt;
      ++g;
      for (; kt + 2 < ke; ++kt, ++g) ktile(kt, STT{});
      for (; kt < ke; ++kt, ++g) ktile(kt, STF{});
    }
#ifdef PDM_G8S_ESEG
    // diagnostic builds only (-DPDM_G8S_ESEG, tools/g8s_eseg.py): shader cycles of the epilogue's parts per tile
    unsigned long long eseg_t = __builtin_amdgcn_s_memtime();
    auto eseg = [&](int i) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      seg_acc[i] += (unsigned)(t - eseg_t);
      eseg_t = t;
    };
#else
    auto eseg = [](int) {};
#endif
    if (wave < 4) bar_raw();   // rejoin the stagger
    eseg(0);

    if constexpr (SK) {
      if (kind == 1) {   // head: accumulators -> slab (sc1 write-through), the next tile's tables
        if (has_next) issue_tables(nv, m0n, n0n);
        const __amdgpu_buffer_rsrc_t rsl = make_rsrc(p.sk_slab + (size_t)blockIdx.x * 65536, 262144);
#pragma unroll
        for (int f = 0; f < 32; ++f)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, acc[f]), rsl,
                                                 (p.dbg_tile0 & 512) ? (int)OOB : opaque_i(tid) * 16, f * 8192, 16);
        pub_pending = true;
        m0 = m0n;
        n0 = n0n;
        kb = kbn;
        ke = ken;
        kind = kindn;
        continue;
      }
    }

    if (p.dbg_tile0 & 16) {    // timing experiment: no epilogue (its E stores still issued, to nowhere)
#pragma unroll
      for (int f = 0; f < 32; ++f) asm volatile("" ::"v"(acc[f]));
      if (has_next) issue_tables(nv, m0n, n0n);
      if constexpr (GRP) set_out(cv);
#pragma unroll
      for (int s = 0; s < E; ++s) __builtin_amdgcn_raw_buffer_store_b32(0, rout, (int)OOB, 0, 0);
      m0 = m0n;
      n0 = n0n;
      kb = kbn;
      ke = ken;
      kind = kindn;
      if constexpr (GRP) cv = nv;
      continue;
    }

    // ---- epilogue of tile (m0, n0) of problem cv ----
    if constexpr (GRP) set_out(cv);
    const int M = cv.M;
    // this lane's columns: fragment (qj, ni) covers n0 + qj*128 + wn*32 + ni*16 + g4*4 + [0, 4)
    f32x4 bv[2][2], cs[2][2];
    // lane-derived LDS addresses recomputed here from an opaque copy of tid, not held across the K-loop (the
    // residual epilogue runs at the 256-VGPR limit)
    const int tid_e = opaque_i(tid), g4e = (tid_e & 63) >> 4, r16e = tid_e & 15;
    lds_rd_cols(smem + S_COL + (wn * 32 + g4e * 4) * 4, bv, cs);
    char* lnrow = smem + S_LNROW;
    // FP8 centred LayerNorm (ln_gcol): rows carry mean 0 and the table of (mu_t - mean) as bf16 hi / lo
    const bool lnc = FP8 && ln && p.ln_gcol != nullptr;
    if (ln && tid < 256) {
      f32x2 raw[8];
      lds_rd_raw(smem + S_RAW + tid_e * p.ln_ld * 8, raw);
      float2 lst[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) lst[t] = t < p.ln_ld ? make_float2(raw[t][0], raw[t][1]) : make_float2(0.f, 0.f);
      if (lnc) {
        float mu[8];
        const float2 mr = ln_from_partials(lst, p.ln_ld, p.ln_D, p.ln_eps, mu);
        unsigned hl[8];   // hi pairs 0..3, lo pairs 4..7
#pragma unroll
        for (int t = 0; t < 8; t += 2) {
          const float d0 = mu[t] - mr.x, d1 = mu[t + 1] - mr.x;
          const unsigned h = pack_bf16x2(d0, d1);
          hl[t >> 1] = h;
          hl[4 + (t >> 1)] = pack_bf16x2(d0 - bf16lo(h), d1 - bf16hi(h));
        }
        lds_wr128(smem + S_STAT + tid * 32, i32x4{(int)hl[0], (int)hl[1], (int)hl[2], (int)hl[3]});
        lds_wr128(smem + S_STAT + tid * 32 + 16, i32x4{(int)hl[4], (int)hl[5], (int)hl[6], (int)hl[7]});
        lds_wr64(lnrow + tid * 8, make_float2(0.f, mr.y));
      } else {
        lds_wr64(lnrow + tid * 8, ln_from_partials(lst, p.ln_ld, p.ln_D, p.ln_eps, nullptr));
      }
    }
    lds_sync();
#pragma unroll
    for (int qj = 0; qj < 2; ++qj)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        if (!ln || lnc) cs[qj][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    eseg(1);
    bar_raw();   // lnrow complete; the raw / column tables are free for the next tile's
    if constexpr (FP8) {
      if (lnc) {
        // acc += sum_t (mu_t - mean) c_t[n] as one bf16 16x16x32 MFMA per accumulator (gemm_mx_kernel's correction):
        // K lanes 0-7 carry hi * hi, 8-15 hi * lo, 16-23 lo * hi, 24-31 zeros.  Column tables c_t (hi | lo, 32 B per
        // column) come straight from ln_gcol, the row tables from S_STAT.
        const __amdgpu_buffer_rsrc_t rg = make_rsrc(p.ln_gcol, (long long)p.N * 32);
        i32x4 gv[2][2];
#pragma unroll
        for (int qj = 0; qj < 2; ++qj)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni) {
            const int col = n0 + qj * 128 + wn * 32 + ni * 16 + r16e;
            const unsigned off = (g4e == 3 || col >= p.N) ? OOB : (unsigned)col * 32u + (g4e == 1 ? 16u : 0u);
            gv[qj][ni] = __builtin_amdgcn_raw_buffer_load_b128(rg, (int)off, 0, 0);
          }
        i32x4 rv[8];
        lds_rd_rowc(smem + S_STAT + (wm * 64 + r16e) * 32 + (g4e == 2 ? 16 : 0), rv);
        wait_vmcnt_n<0>();
        asm volatile("" : "+v"(gv[0][0]), "+v"(gv[0][1]), "+v"(gv[1][0]), "+v"(gv[1][1]));
        const i32x4 z4 = i32x4{0, 0, 0, 0};
#pragma unroll
        for (int qi = 0; qi < 2; ++qi)
#pragma unroll
          for (int qj = 0; qj < 2; ++qj)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
              for (int mi = 0; mi < 4; ++mi) {
                f32x4& c = acc[((qi * 2 + qj) * 2 + ni) * 4 + mi];
                const i32x4 a = g4e == 3 ? z4 : rv[qi * 4 + mi];
                c = mfma16x16x32(__builtin_bit_cast(bf16x8, gv[qj][ni]), __builtin_bit_cast(bf16x8, a), c);
              }
      }
    }
    if (has_next) issue_tables(nv, m0n, n0n);
    const int offg = (g4 & 1) * 16 + (g4 >> 1) * 8;   // post-swap column offset of the lane's 8 columns
    float2 mrow[2][4];   // (mean, rstd) of the lane's 8 rows
    {
      f32x2 mr8[8];
      lds_rd_rows(lnrow + (wm * 64 + r16e) * 8, mr8);
#pragma unroll
      for (int qi = 0; qi < 2; ++qi)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
          mrow[qi][mi] = ln ? make_float2(mr8[qi * 4 + mi][0], mr8[qi * 4 + mi][1]) : make_float2(0.f, 1.f);
    }

    eseg(2);
    if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU) {
      unsigned e8[16];   // MXO: E8M0 scale of block (qi, mi, qj) at [qi * 8 + mi * 2 + qj]
#pragma unroll
      for (int qi = 0; qi < 2; ++qi)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          const int ml = qi * 128 + wm * 64 + mi * 16 + r16;
          const float2 mr = mrow[qi][mi];
          const int m = m0 + ml;
#pragma unroll
          for (int qj = 0; qj < 2; ++qj) {
            unsigned u[2][2];
            f32x4 v[2];
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
              v[ni] = acc[((qi * 2 + qj) * 2 + ni) * 4 + mi];
              // rstd * (acc - mean * colsum) + bias as acc * rstd + (bias - mean * rstd * colsum): 2 FMAs per value
              if (ln) v[ni] = v[ni] * mr.y + (bv[qj][ni] - (mr.x * mr.y) * cs[qj][ni]);
              else v[ni] += bv[qj][ni];
            }
            if constexpr (EPI == EPI_GELU && MXO && SK) {   // (the stream-K MXFP8-output form spills with 4 pairs)
#pragma unroll
              for (int ni = 0; ni < 2; ++ni) {
                const f32x2 lo = gelu_erf2(f32x2{v[ni][0], v[ni][1]}), hi = gelu_erf2(f32x2{v[ni][2], v[ni][3]});
                v[ni] = f32x4{lo[0], lo[1], hi[0], hi[1]};
              }
            } else if constexpr (EPI == EPI_GELU) {   // exact-erf GELU only (quick GELU: gemm8d, fits_8s); 4 pairs interleaved
              f32x2 x2[4] = {f32x2{v[0][0], v[0][1]}, f32x2{v[0][2], v[0][3]}, f32x2{v[1][0], v[1][1]},
                             f32x2{v[1][2], v[1][3]}};
              gelu_erf2x4(x2);
              v[0] = f32x4{x2[0][0], x2[0][1], x2[1][0], x2[1][1]};
              v[1] = f32x4{x2[2][0], x2[2][1], x2[3][0], x2[3][1]};
            }
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
              u[ni][0] = pack_bf16x2(v[ni][0], v[ni][1]);
              u[ni][1] = pack_bf16x2(v[ni][2], v[ni][3]);
            }
            if constexpr (MXO) {
              // MXFP8 of the bf16-rounded values (as gemm8d's staged epilogue): the 32-column block qj*128 + wn*32
              // of row m is fragments ni 0/1 of the 4 lane rows g4, so its |max| is the lane's 8 values reduced
              // over l ^ 16, l ^ 32; after the quantisation a permlane16 swap gives every lane 8 consecutive bytes
              const float f[8] = {bf16lo(u[0][0]), bf16hi(u[0][0]), bf16lo(u[0][1]), bf16hi(u[0][1]),
                                  bf16lo(u[1][0]), bf16hi(u[1][0]), bf16lo(u[1][1]), bf16hi(u[1][1])};
              float am = 0.f;
#pragma unroll
              for (int j = 0; j < 8; ++j) am = fmaxf(am, fabsf(f[j]));
              const auto a32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(am), __float_as_uint(am), false, false);
              am = fmaxf(__uint_as_float(a32[0]), __uint_as_float(a32[1]));
              const auto a16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(am), __float_as_uint(am), false, false);
              am = fmaxf(__uint_as_float(a16[0]), __uint_as_float(a16[1]));
              const unsigned bits = __float_as_uint(am * (1.0f / 448.0f));
              unsigned e = (bits >> 23) & 0xffu;
              e += (bits & 0x7fffffu) ? 1u : 0u;
              e = e > 254u ? 254u : e;
              const float inv = __uint_as_float((254u - e) << 23);   // 2^(127 - e)
              int w0 = 0, w1 = 0;
              w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[0] * inv, f[1] * inv, w0, false);
              w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[2] * inv, f[3] * inv, w0, true);
              w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[4] * inv, f[5] * inv, w1, false);
              w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[6] * inv, f[7] * inv, w1, true);
              unsigned q0 = (unsigned)w0, q1 = (unsigned)w1;
              pl16swap(q0, q1);
              e8[qi * 8 + mi * 2 + qj] = e;
              const int n = n0 + qj * 128 + wn * 32 + offg;
              const unsigned off = (m < M && n < p.N && !(p.dbg_tile0 & 32)) ? (unsigned)m * (unsigned)p.ldo8 + (unsigned)n : OOB;
              __builtin_amdgcn_raw_buffer_store_b64(i32x2{(int)q0, (int)q1}, rout, (int)off, 0, 0);
            } else {
              pl16swap(u[0][0], u[1][0]);
              pl16swap(u[0][1], u[1][1]);
              const int n = n0 + qj * 128 + wn * 32 + offg;
              const unsigned off = (m < M && n < p.N && !(p.dbg_tile0 & 32)) ? ((unsigned)m * (unsigned)p.ldo + (unsigned)n) * 2u : OOB;
              __builtin_amdgcn_raw_buffer_store_b128(i32x4{(int)u[0][0], (int)u[0][1], (int)u[1][0], (int)u[1][1]},
                                                     rout, (int)off, 0, 0);
            }
          }
        }
      if constexpr (MXO) {
        // scale bytes: block (row m, 32 columns at n) -> byte ((n >> 7) * out_scale_ld + m) * 4 + ((n >> 5) & 3) =
        // ((n0 / 128 + qj) * ld + m) * 4 + wn; the 4 lane rows hold equal scales, so store j takes block
        // gi = j * 4 + g4 in lane row g4 (4 byte stores instead of 16)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const unsigned ev = g4 == 0 ? e8[j * 4] : g4 == 1 ? e8[j * 4 + 1] : g4 == 2 ? e8[j * 4 + 2] : e8[j * 4 + 3];
          const int qi = j >> 1, mi = (j & 1) * 2 + (g4 >> 1), qj = g4 & 1;
          const int m = m0 + qi * 128 + wm * 64 + mi * 16 + r16;
          const int nb = n0 + qj * 128 + wn * 32;
          const unsigned off = (m < M && nb < p.N && !(p.dbg_tile0 & 32))
                                   ? ((unsigned)((n0 >> 7) + qj) * (unsigned)p.out_scale_ld + (unsigned)m) * 4u + (unsigned)wn : OOB;
          __builtin_amdgcn_raw_buffer_store_b8((unsigned char)ev, rsc, (int)off, 0, 0);
        }
      }
    } else {   // EPI_RES
      // Residual rows in the 16-byte layout, all issued before the first use.  No per-value masks: rows past M fall
      // past the descriptors' num_records (the hardware reads zeros and drops the stores), and a column past N holds
      // exactly 0 (zero W rows, zero-staged bias, a masked residual load), so it adds nothing to a row's sum and
      // (0 - mu)^2 to its M2, which is subtracted per row below.  Only the column test stays on each 16-byte access.
      i32x4 rr[2][4][2];
      const bool acc_res = p.accumulate != 0;
      const bool drop_st = p.dbg_tile0 & 32, drop_res = !acc_res || (p.dbg_tile0 & 64);
#pragma unroll
      for (int qi = 0; qi < 2; ++qi)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int qj = 0; qj < 2; ++qj) {
            const unsigned m = (unsigned)(m0 + qi * 128 + wm * 64 + mi * 16 + r16);
            const int n = n0 + qj * 128 + wn * 32 + offg;
            const unsigned off = (!drop_res && n < p.N) ? (m * (unsigned)p.ldri + (unsigned)n) * 2u : OOB;
            rr[qi][mi][qj] = __builtin_amdgcn_raw_buffer_load_b128(rres, (int)off, 0, 0);
          }
      const int ncols = min(256, p.N - n0);
      float rsum[2][4];
#pragma unroll
      for (int qi = 0; qi < 2; ++qi)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          const unsigned m = (unsigned)(m0 + qi * 128 + wm * 64 + mi * 16 + r16);
          f32x2 s2 = f32x2{0.f, 0.f};
#pragma unroll
          for (int qj = 0; qj < 2; ++qj) {
            unsigned r0 = (unsigned)rr[qi][mi][qj][0], r1 = (unsigned)rr[qi][mi][qj][1];
            unsigned r2 = (unsigned)rr[qi][mi][qj][2], r3 = (unsigned)rr[qi][mi][qj][3];
            pl16swap(r0, r2);   // back to the fragment layout: (r0, r1) = fragment ni 0, (r2, r3) = ni 1
            pl16swap(r1, r3);
            const unsigned rs[2][2] = {{r0, r1}, {r2, r3}};
            unsigned u[2][2];
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
              f32x4& v = acc[((qi * 2 + qj) * 2 + ni) * 4 + mi];
              v += bv[qj][ni];
              v += f32x4{bf16lo(rs[ni][0]), bf16hi(rs[ni][0]), bf16lo(rs[ni][1]), bf16hi(rs[ni][1])};
              u[ni][0] = pack_bf16x2(v[0], v[1]);
              u[ni][1] = pack_bf16x2(v[2], v[3]);
              // the rounded values feed the partials (exactly what the next GEMM reads)
              v = f32x4{bf16lo(u[ni][0]), bf16hi(u[ni][0]), bf16lo(u[ni][1]), bf16hi(u[ni][1])};
              s2 += f32x2{v[0], v[1]};
              s2 += f32x2{v[2], v[3]};
            }
            pl16swap(u[0][0], u[1][0]);
            pl16swap(u[0][1], u[1][1]);
            const int n = n0 + qj * 128 + wn * 32 + offg;
            const unsigned off = (!drop_st && n < p.N) ? (m * (unsigned)p.ldo + (unsigned)n) * 2u : OOB;
            __builtin_amdgcn_raw_buffer_store_b128(i32x4{(int)u[0][0], (int)u[0][1], (int)u[1][0], (int)u[1][1]},
                                                   rout, (int)off, 0, 0);
          }
          rsum[qi][mi] = s2[0] + s2[1];
        }
      eseg(3);
      // LayerNorm partials of the 256-column group (sum, M2 about the group mean): every wave reduces its own 64
      // columns of a row (sum over the 4 lane rows, M2 about the wave's own mean) and the 4 column waves (wn) are
      // merged with Chan's update through LDS -- one barrier.  Without stats_out the store still issues (to
      // nowhere), so every epilogue has E VMEM ops.
      char* tab = smem + S_STAT;   // [row][wn][sum, m2] fp32
      auto wave_cols = [&](int w) { return max(0, min(32, ncols - w * 32)) + max(0, min(32, ncols - 128 - w * 32)); };
      if (stats) {
        const int nw = wave_cols(wn);
        const float inv_w = nw > 0 ? 1.0f / (float)nw : 0.f;
        const float nzero = (float)(64 - nw);   // the wave's columns past N: exact zeros, (0 - mu)^2 each in q
#pragma unroll
        for (int qi = 0; qi < 2; ++qi)
#pragma unroll
          for (int mi = 0; mi < 4; ++mi) {
            const float sw = xrow_sum4(rsum[qi][mi]);
            const float mu = sw * inv_w;
            f32x2 q2 = f32x2{0.f, 0.f};
#pragma unroll
            for (int qj = 0; qj < 2; ++qj)
#pragma unroll
              for (int ni = 0; ni < 2; ++ni) {
                const f32x4 a = acc[((qi * 2 + qj) * 2 + ni) * 4 + mi];
                const f32x2 d0 = f32x2{a[0], a[1]} - mu, d1 = f32x2{a[2], a[3]} - mu;
                q2 += d0 * d0;
                q2 += d1 * d1;
              }
            const float q = xrow_sum4(q2[0] + q2[1]) - nzero * mu * mu;
            if (g4 == 0) lds_wr64(tab + ((qi * 128 + wm * 64 + mi * 16 + r16) * 4 + wn) * 8, make_float2(sw, q));
          }
      }
      eseg(4);
      lds_sync();
      bar_raw();
      eseg(5);
      {   // one float per thread: row tid >> 1, component tid & 1 (sum, M2)
        const int tid_s = opaque_i(tid), ml = tid_s >> 1, c = tid_s & 1;
        f32x2 t4[4];
        lds_rd_stat2(tab + ml * 32, t4);
        const float S = (t4[0][0] + t4[1][0]) + (t4[2][0] + t4[3][0]);
        float v = S;
        if (c) {
          const float mean = S / (float)ncols;
          v = 0.f;
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const int nw = wave_cols(w);
            const float d = nw > 0 ? t4[w][0] / (float)nw - mean : 0.f;
            v += t4[w][1] + (float)nw * d * d;
          }
        }
        const int m = m0 + ml;
        const unsigned off = (stats && m < M) ? (unsigned)((m * p.stats_ld + (n0 >> 8)) * 2 + c) * 4u : OOB;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(v), rst, (int)off, 0, 0);
      }
      eseg(6);
    }
    if constexpr (EPI != EPI_RES) eseg(6);
    m0 = m0n;
    n0 = n0n;
    kb = kbn;
    ke = ken;
    kind = kindn;
    if constexpr (GRP) cv = nv;
  }
#if defined(PDM_G8S_SEG) || defined(PDM_G8S_ESEG)
  if (lane == 0 && (wave == 0 || wave == 4)) {
#pragma unroll
    for (int i = 0; i < 12; ++i) atomicAdd(&g_seg_stats[(wave == 4 ? 12 : 0) + i], (unsigned long long)seg_acc[i]);
    if (wave == 0) atomicAdd(&g_seg_stats[24], 1ull);
  }
#endif
#ifdef PDM_G8S_CLK
  if (tid == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    atomicAdd(&g_sk_stats[0], t1 - clk_t0);
    atomicAdd(&g_sk_stats[1], r1 - clk_r0);
    atomicAdd(&g_sk_stats[2], 1ull);
  }
#endif
}

// the one-problem kernel keeps its own signature (a second by-value GemmArgs in every launch measured +0.7 % on the
// L/2 forward); the grouped kernel takes both problems
template <int EPI, int MXO = 0, int SK = 0, int FP8 = 0, int DUAL = 1>
__global__ __launch_bounds__(512, 1) void gemm8s_kernel(GemmArgs p, int tiles_n, int ntiles) {
  gemm8s_body<EPI, MXO, 0, SK, FP8, DUAL>(p, tiles_n, ntiles, TV{}, ntiles);
}
template <int EPI, int DUAL = 1>
__global__ __launch_bounds__(512, 1) void gemm8g_kernel(GemmArgs p, int tiles_n, int ntiles, TV p2, int nt0) {
  gemm8s_body<EPI, 0, 1, 0, 0, DUAL>(p, tiles_n, ntiles, p2, nt0);
}

// ------------------------------------------------------------------------------------------------
// Tall tile for N <= 128 (algo 9; the decoder's 128-channel 512^2 convs): 512 x 128 per workgroup, 8 waves.
// A 256 x 128 tile re-fetches its 32 KiB A K-tile for half the MFMA work of a 256 x 256 one and runs at the
// same time per K-tile (tools/conv_bench.py: algo 8 ~ algo 1 ~ 0.58 PF on these convs), so the N = 128 GEMM
// needs more rows per W panel instead: four 128-row A quarters share one W half-tile.  Every wave owns a 64 x 32
// piece of each quarter -- the same 32 accumulators and fragment reads per MFMA as gemm8d.  Ring: 2 slots x
// (A0 A1 A2 A3 W) x 16 KiB = the whole 160 KiB LDS (no LN / prologue-staged columns: bias is read in the
// epilogue).  Per K-tile:
//   phase A(k): reads A0 W A1 of tile k, issues A2 A3 of tile k+1        wait: A2 A3 (k)
//   phase B(k): reads A2 A3 of tile k,   issues A0 W A1 of tile k+2      wait: A0 W A1 (k+1)
// every wait leaving the 10 youngest LDS-DMA (5 16-KiB pieces) in flight.  Quarter q accumulates into the
// 256x256 layout's quadrant slot (q & 1, q >> 1), so the epilogue runs twice through the 256-tile epilogue: rows
// 0-255 from slots (*, 0) (slots (*, 1) sit at columns >= 128 >= N and are never stored), then, with the two
// slot halves swapped, rows 256-511.
template <int EPI, int CONV>
__global__ __launch_bounds__(512, 1) void gemm8t_kernel(GemmArgs p, int nwg) {
  constexpr int ROWB = 128;
  constexpr int HALF = 128 * ROWB;              // 16 KiB piece
  constexpr int BUF = 5 * HALF;                 // A0 A1 A2 A3 W
  constexpr int KW = 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  int bid = blockIdx.x;
  {
    const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
  }
  const int m0 = bid * 512;
  const int ldw = p.ldw > 0 ? p.ldw : p.K;
  long long a1_rows;
  if (CONV) a1_rows = (long long)(p.M / (p.convH * p.convW)) * (p.convH >> p.conv_up) * (p.convW >> p.conv_up);
  else a1_rows = p.M;
  const __amdgpu_buffer_rsrc_t ra1 = make_rsrc(p.A1, a1_rows * (CONV ? p.convC : p.lda1) * 2);
  const __amdgpu_buffer_rsrc_t ra2 = make_rsrc(p.A2 ? p.A2 : p.A1, p.A2 ? (long long)p.M * p.lda2 * 2 : 0);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.W, (long long)(p.N - 1) * ldw * 2 + (long long)p.K * 2);

  const int prow = lane >> 3, pch = lane & 7;
  unsigned a1off[4][2], a2off[4][2], woff[2], sbv[2];   // conv: only sbv (the swizzled chunk) and cpix
  int cpix[4][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 8 + prow;
    const unsigned sb = (unsigned)((pch ^ ((row >> 1) & 7)) * 16);
    sbv[i] = sb;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int gm = m0 + h * 128 + row;
      if constexpr (CONV) {
        if (gm < p.M) {
          const int hw = p.convH * p.convW, b = gm / hw, r = gm - b * hw, y = r / p.convW;
          cpix[h][i] = (b << 18) | (y << 9) | (r - y * p.convW);
        } else {
          cpix[h][i] = -1;
        }
        a1off[h][i] = 0;
        a2off[h][i] = 0;
      } else {
        a1off[h][i] = gm < p.M ? (unsigned)gm * (unsigned)(p.lda1 * 2) + sb : OOB;
        a2off[h][i] = gm < p.M ? (unsigned)gm * (unsigned)(p.lda2 * 2) + sb : OOB;
        cpix[h][i] = 0;
      }
    }
    woff[i] = row < p.N ? (unsigned)row * (unsigned)(ldw * 2) + sb : OOB;
  }

  auto issue = [&](int kt, int kind) {
    const int k0 = kt * 64;
    char* dst = smem + (kt & 1) * BUF + kind * HALF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      PDM_LDS void* d = (PDM_LDS void*)(dst + (wave * 2 + i) * 1024);
      if (kind == KW) {
        dma16(rw, woff[i], k0 * 2, d);
      } else if constexpr (CONV) {
        const int tap = k0 / p.convC, ci0 = k0 - tap * p.convC;
        const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
        dma16(ra1, conv_off(p, cpix[kind][i], dy, dx, sbv[i]), ci0 * 2, d);
      } else {
        if (k0 < p.K1) dma16(ra1, a1off[kind][i], k0 * 2, d);
        else dma16(ra2, a2off[kind][i], (k0 - p.K1) * 2, d);
      }
    }
  };

  f32x4 acc[32];
#pragma unroll
  for (int f = 0; f < 32; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
  // every fragment a phase uses is read before its first barrier (waves 4-7 run one barrier behind, so a read
  // after it could race the other half's refill of the slot): two quarters' A fragments + the W fragments
  bf16x8 af[2][4][2];   // A fragments of the phase's two quarters: [quarter & 1][mi][k-sub]
  bf16x8 wf[2][2];      // W fragments: [ni][k-sub]
  auto read_a = [&](const char* buf, int q) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int row = wm * 64 + mi * 16 + (lane & 15);
        af[q & 1][mi][ks] = *reinterpret_cast<const bf16x8*>(buf + q * HALF + swz_off<64>(row, ks * 4 + (lane >> 4)));
      }
  };
  auto read_w = [&](const char* buf) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int row = wn * 32 + ni * 16 + (lane & 15);
        wf[ni][ks] = *reinterpret_cast<const bf16x8*>(buf + KW * HALF + swz_off<64>(row, ks * 4 + (lane >> 4)));
      }
  };
  auto lds_done = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mma = [&](int q) {   // quarter q -> quadrant slot (q & 1, q >> 1)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          f32x4& c = acc[(((q & 1) * 2 + (q >> 1)) * 2 + ni) * 4 + mi];
          c = mfma16x16x32(wf[ni][ks], af[q & 1][mi][ks], c);
        }
    __builtin_amdgcn_s_setprio(0);
  };

  const int nk = p.K / 64;
  issue(0, 0);
  issue(0, KW);
  issue(0, 1);
  issue(0, 2);
  issue(0, 3);
  if (nk > 1) {
    issue(1, 0);
    issue(1, KW);
    issue(1, 1);
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");   // A0 W A1 (0)
  } else {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  bar_raw();
  if (wave >= 4) bar_raw();
  for (int kt = 0; kt < nk; ++kt) {
    const char* buf = smem + (kt & 1) * BUF;
    const bool m1 = kt + 1 < nk, m2 = kt + 2 < nk;
    // phase A
    read_a(buf, 0);
    read_w(buf);
    read_a(buf, 1);
    if (m1) {
      issue(kt + 1, 2);
      issue(kt + 1, 3);
      lds_done();
      asm volatile("s_waitcnt vmcnt(10)" ::: "memory");   // A2 A3 (kt)
    } else {
      lds_done();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar_raw();
    mma(0);
    mma(1);
    bar_raw();
    // phase B
    read_a(buf, 2);
    read_a(buf, 3);
    if (m2) {
      issue(kt + 2, 0);
      issue(kt + 2, KW);
      issue(kt + 2, 1);
      lds_done();
      asm volatile("s_waitcnt vmcnt(10)" ::: "memory");   // A0 W A1 (kt+1)
    } else {
      lds_done();
      if (m1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    bar_raw();
    mma(2);
    mma(3);
    bar_raw();
  }
  if (wave < 4) bar_raw();

  epilogue256<EPI, 1>(p, acc, smem, m0, 0, tid, lane, wm, wn);
  if (m0 + 256 < p.M) {
    __syncthreads();   // the first half's LDS read-back is done before the second half is staged
#pragma unroll
    for (int f = 0; f < 32; ++f)
      if (f & 8) {
        const f32x4 t = acc[f];
        acc[f] = acc[f ^ 8];
        acc[f ^ 8] = t;
      }
    epilogue256<EPI, 1>(p, acc, smem, m0 + 256, 0, tid, lane, wm, wn);
  }
}

// ------------------------------------------------------------------------------------------------
// MXFP8 GEMM (algo 7 schedule, e4m3 operands with E8M0 block scales) on v_mfma_scale_f32_16x16x128_f8f6f4:
// twice the bf16 MFMA rate.  A K-tile is 128 fp8 = 128-byte LDS rows, so staging, swizzle and fragment reads
// are byte-for-byte those of the bf16 kernel (a lane's 32-byte fragment = chunks g and 4+g, g = lane >> 4,
// exactly the operand layout the scaled MFMA expects: tools/probes/mx_layout.hip).  Per K-tile each wave also
// stages 256 B of block scales (waves 0-3: A rows, waves 4-7: W rows) into a 2 KiB slot; a lane packs the four
// E8M0 bytes it needs per operand half into one VGPR and the MFMA selects them with opsel.
//   phase A(k): reads A0 W0 W1 + scales of tile k, issues A1(k+1)          wait: A1(k)
//   phase B(k): reads A1,      issues S A0 W0 W1 of tile k+2               wait: S A0 W0 W1 (k+1)

constexpr int MX_SCALE_LDS = EPI_LDS + EPI_LDS_EXTRA;   // 2 x 2 KiB of staged block scales
constexpr int MX_COL_LDS = MX_SCALE_LDS + 2 * 2048;      // the tile's bias [256] + LN colsum [256] (fp32)
constexpr int MX_ROWC_LDS = MX_COL_LDS + COL_LDS_BYTES;  // centred LN: per row (mu_t - mean) as bf16 hi[8] lo[8]
constexpr int MX_GCOL_LDS = MX_ROWC_LDS + 256 * 32;      // centred LN: per column c_t as bf16 hi[8] lo[8]
constexpr int MX_SMEM = MX_GCOL_LDS + 256 * 32;          // 152 KiB

template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm_mx_kernel(GemmArgs p, int tiles_n, int nwg) {
  constexpr int HALF = 128 * 128;
  constexpr int BUF = 4 * HALF;
  enum { KA0 = 0, KA1 = 1, KW0 = 2, KW1 = 3 };
  typedef int v8i __attribute__((ext_vector_type(8)));
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably uniform: scalar descriptor choice
  const int wm = wave >> 2, wn = wave & 3, g = lane >> 4;
  int bid = blockIdx.x;
  {
    const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
  }
  int tm, tn;
  if (p.raster > 0) {
    const int tiles_m = (p.M + BM2 - 1) / BM2;
    const int grp = bid / (p.raster * tiles_n);
    const int rows_in = min(p.raster, tiles_m - grp * p.raster);
    const int r = bid - grp * p.raster * tiles_n;
    tm = grp * p.raster + r % rows_in;
    tn = r / rows_in;
  } else {
    tm = bid / tiles_n;
    tn = bid - tm * tiles_n;
  }
  const int m0 = tm * BM2, n0 = tn * BN2;
  const int ldw = p.ldw > 0 ? p.ldw : p.K;
  const int nk = p.K / 128;
  const unsigned char* A8 = reinterpret_cast<const unsigned char*>(p.A1);
  const unsigned char* W8 = reinterpret_cast<const unsigned char*>(p.W);
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(A8, (long long)p.M * p.lda1);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(W8, (long long)(p.N - 1) * ldw + p.K);
  const __amdgpu_buffer_rsrc_t rsa = make_rsrc(p.a_scale, (long long)nk * p.a_scale_ld * 4);
  const __amdgpu_buffer_rsrc_t rsw = make_rsrc(p.w_scale, (long long)nk * p.w_scale_ld * 4);

  const int prow = lane >> 3, pch = lane & 7;
  unsigned aoff[2][2], woff[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 8 + prow;
    const unsigned sb = (unsigned)((pch ^ ((row >> 1) & 7)) * 16);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int gm = m0 + h * 128 + row, gn = n0 + h * 128 + row;
      aoff[h][i] = gm < p.M ? (unsigned)gm * (unsigned)p.lda1 + sb : OOB;
      woff[h][i] = gn < p.N ? (unsigned)gn * (unsigned)ldw + sb : OOB;
    }
  }
  // block-scale staging: wave w < 4 stages A rows m0 + 64 w + lane, waves 4-7 W rows n0 + 64 (w - 4) + lane
  const bool s_is_a = wave < 4;
  const int srow = (wave & 3) * 64 + lane;
  const unsigned soff = s_is_a ? (m0 + srow < p.M ? (unsigned)(m0 + srow) * 4u : OOB)
                               : (n0 + srow < p.N ? (unsigned)(n0 + srow) * 4u : OOB);

  auto issue = [&](int kt, int kind) {
    char* dst = smem + (kt & 1) * BUF + kind * HALF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      PDM_LDS void* d = (PDM_LDS void*)(dst + (wave * 2 + i) * 1024);
      if (kind >= KW0) dma16(rw, woff[kind - KW0][i], kt * 128, d);
      else dma16(ra, aoff[kind][i], kt * 128, d);
    }
  };
  auto issue_scales = [&](int kt) {
    PDM_LDS void* d = (PDM_LDS void*)(smem + MX_SCALE_LDS + (kt & 1) * 2048 + (s_is_a ? 0 : 1024) + (wave & 3) * 256);
    if (s_is_a) __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, d, 4, (int)soff, kt * p.a_scale_ld * 4, 0, 0);
    else __builtin_amdgcn_raw_ptr_buffer_load_lds(rsw, d, 4, (int)soff, kt * p.w_scale_ld * 4, 0, 0);
  };

  f32x4 acc[32];
#pragma unroll
  for (int f = 0; f < 32; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
  v8i af[4];        // A fragments of the current A half: [mi], 32 fp8 each
  v8i wf[2][2];     // W fragments of both W halves: [qj][ni]
  unsigned sa[2], sw = 0;   // packed E8M0: sa[qi] byte mi, sw byte qj*2 + ni

  // a lane's 32-byte fragment = its row's 16-byte chunks g and 4 + g, read straight into the 8-VGPR operand
  auto frag = [&](v8i& dst, const char* base, int row) {
    i32x4* h = reinterpret_cast<i32x4*>(&dst);
    h[0] = *reinterpret_cast<const i32x4*>(base + swz_off<64>(row, g));
    h[1] = *reinterpret_cast<const i32x4*>(base + swz_off<64>(row, 4 + g));
  };
  auto read_a = [&](const char* buf, int qi) {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) frag(af[mi], buf + qi * HALF, wm * 64 + mi * 16 + (lane & 15));
  };
  auto read_w = [&](const char* buf) {
#pragma unroll
    for (int qj = 0; qj < 2; ++qj)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) frag(wf[qj][ni], buf + (2 + qj) * HALF, wn * 32 + ni * 16 + (lane & 15));
  };
  auto read_scales = [&](int kt) {
    const unsigned* sl = reinterpret_cast<const unsigned*>(smem + MX_SCALE_LDS + (kt & 1) * 2048);
#pragma unroll
    for (int qi = 0; qi < 2; ++qi) {
      unsigned v = 0;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
        v |= ((sl[qi * 128 + wm * 64 + mi * 16 + (lane & 15)] >> (8 * g)) & 0xffu) << (8 * mi);
      sa[qi] = v;
    }
    unsigned v = 0;
#pragma unroll
    for (int qj = 0; qj < 2; ++qj)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
        v |= ((sl[256 + qj * 128 + wn * 32 + ni * 16 + (lane & 15)] >> (8 * g)) & 0xffu) << (8 * (qj * 2 + ni));
    sw = v;
    asm volatile("" : "+v"(sa[0]), "+v"(sa[1]), "+v"(sw));
  };
  auto lds_done = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mma = [&](auto qic, auto qjc) {
    constexpr int qi = decltype(qic)::value, qj = decltype(qjc)::value;
    __builtin_amdgcn_s_setprio(1);
    static_for<2>([&](auto nic) {
      constexpr int ni = decltype(nic)::value;
      static_for<4>([&](auto mic) {
        constexpr int mi = decltype(mic)::value;
        f32x4& c = acc[((qi * 2 + qj) * 2 + ni) * 4 + mi];
        c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wf[qj][ni], af[mi], c, 0, 0, qj * 2 + ni, sw, mi,
                                                             sa[qi]);
        // pin the MFMA inside this phase: IR-level sinking otherwise moves whole MFMA clusters (and the scale
        // packing feeding them) across the barriers into the next phase
        asm volatile("" : "+v"(c));
      });
    });
    __builtin_amdgcn_s_setprio(0);
  };

  // epilogue inputs fetched ahead of the first operand DMA (as gemm8d_kernel): the tile's LayerNorm row partials
  // (waves 0-3, one row each), its bias / LN column sums or, for the centred LayerNorm (GemmArgs::ln_gcol), the
  // bf16 hi / lo group sums of its columns (waves 4-7, one column each); the prologue's vmcnt wait covers them
  const bool ln_pre = epi_rowout(EPI) && p.ln_stats != nullptr && p.ln_ld <= 8;
  const bool lnc = ln_pre && p.ln_gcol != nullptr;
  float2 lst[8];
  if (ln_pre && tid < 256) {
    const float2* st = reinterpret_cast<const float2*>(p.ln_stats) + (size_t)min(m0 + tid, p.M - 1) * p.ln_ld;
#pragma unroll
    for (int t = 0; t < 8; ++t) lst[t] = t < p.ln_ld ? st[t] : make_float2(0.f, 0.f);
  }
  float cb = 0.f, cc = 0.f;
  i32x4 gc[2] = {i32x4{0, 0, 0, 0}, i32x4{0, 0, 0, 0}};
  if (tid >= 256) {
    const int n = n0 + tid - 256;
    if (n < p.N) {
      if (p.bias) cb = p.bias[n];
      if (epi_rowout(EPI) && p.ln_stats && !lnc) cc = p.ln_colsum[n];
      if (lnc) {
        const i32x4* src = reinterpret_cast<const i32x4*>(p.ln_gcol + (size_t)n * 16);
        gc[0] = src[0];
        gc[1] = src[1];
      }
    }
  }

  issue_scales(0);
  issue(0, KA0);
  issue(0, KW0);
  issue(0, KW1);
  issue(0, KA1);
  if (nk > 1) {
    issue_scales(1);
    issue(1, KA0);
    issue(1, KW0);
    issue(1, KW1);
    asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  }
  if (tid >= 256) {
    reinterpret_cast<float*>(smem + MX_COL_LDS)[tid - 256] = cb;
    reinterpret_cast<float*>(smem + MX_COL_LDS)[tid] = cc;   // colsum at +256 (zero for the centred form)
    if (lnc) {
      i32x4* dst = reinterpret_cast<i32x4*>(smem + MX_GCOL_LDS + (tid - 256) * 32);
      dst[0] = gc[0];
      dst[1] = gc[1];
    }
  }
  if (ln_pre && tid < 256) {
    float mu[8];
    const float2 mr = ln_from_partials(lst, p.ln_ld, p.ln_D, p.ln_eps, lnc ? mu : nullptr);
    if (lnc) {   // rows carry (mu_t - mean) as a bf16 pair; the epilogue then sees mean 0
      bf16x8 hi, lo;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const float d = mu[t] - mr.x;
        hi[t] = (bf16)d;
        lo[t] = (bf16)(d - (float)hi[t]);
      }
      bf16x8* dst = reinterpret_cast<bf16x8*>(smem + MX_ROWC_LDS + tid * 32);
      dst[0] = hi;
      dst[1] = lo;
      reinterpret_cast<float2*>(smem + EPI_LDS)[tid] = make_float2(0.f, mr.y);
    } else {
      reinterpret_cast<float2*>(smem + EPI_LDS)[tid] = mr;
    }
  }
  bar_raw();
  if (wave >= 4) bar_raw();
  for (int kt = 0; kt < nk; ++kt) {
    const char* buf = smem + (kt & 1) * BUF;
    const bool m1 = kt + 1 < nk, m2 = kt + 2 < nk;
    // phase A
    read_a(buf, 0);
    read_w(buf);
    read_scales(kt);
    if (m1) { issue(kt + 1, KA1); lds_done(); asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); }   // A1(kt)
    else { lds_done(); asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
    bar_raw();
    mma(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
    mma(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
    bar_raw();
    // phase B
    read_a(buf, 1);
    if (m2) {
      issue_scales(kt + 2);
      issue(kt + 2, KA0);
      issue(kt + 2, KW0);
      issue(kt + 2, KW1);
      lds_done();
      asm volatile("s_waitcnt vmcnt(9)" ::: "memory");   // S A0 W0 W1 (kt+1)
    } else {
      lds_done();
      if (m1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    }
    bar_raw();
    mma(std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{});
    mma(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});
    bar_raw();
  }
  if (wave < 4) bar_raw();
  if (lnc) {
    // centred LayerNorm: acc += sum_t (mu_t - mean) c_t as one bf16 MFMA per accumulator; K lanes 0-7 carry
    // hi * hi, 8-15 hi * lo, 16-23 lo * hi, 24-31 zeros (tables written before the prologue barrier)
    const int kg = lane >> 4;
    const bf16x8 z8 = __builtin_bit_cast(bf16x8, i32x4{0, 0, 0, 0});
    bf16x8 wc[2][2];
#pragma unroll
    for (int qj = 0; qj < 2; ++qj)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int col = qj * 128 + wn * 32 + ni * 16 + (lane & 15);
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(smem + MX_GCOL_LDS + col * 32 + (kg == 1 ? 16 : 0));
        wc[qj][ni] = kg == 3 ? z8 : v;
      }
#pragma unroll
    for (int qi = 0; qi < 2; ++qi) {
      bf16x8 ac[4];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int row = qi * 128 + wm * 64 + mi * 16 + (lane & 15);
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(smem + MX_ROWC_LDS + row * 32 + (kg == 2 ? 16 : 0));
        ac[mi] = kg == 3 ? z8 : v;
      }
#pragma unroll
      for (int qj = 0; qj < 2; ++qj)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int mi = 0; mi < 4; ++mi) {
            f32x4& c = acc[((qi * 2 + qj) * 2 + ni) * 4 + mi];
            c = mfma16x16x32(wc[qj][ni], ac[mi], c);
          }
    }
  }
  epilogue256<EPI, 1>(p, acc, smem, m0, n0, tid, lane, wm, wn, ln_pre, true, MX_COL_LDS);
}
}  // namespace

static int g_gemm_raster = 0, g_gemm_dbg = 0;   // tuning knobs (pdm_set_gemm_tuning)

static bool fits_rsrc(const GemmArgs& p);

const char* gemm_check(const GemmArgs& p, int epi) {
  if (p.M <= 0 || p.N <= 0 || p.K <= 0) return "gemm: M, N, K must be positive";
  if (p.N % 4) return "gemm: N must be a multiple of 4";
  if (p.K % BK) return "gemm: K must be a multiple of 64";
  if (p.K1 % BK || p.K1 <= 0 || p.K1 > p.K) return "gemm: K1 must be a positive multiple of 64 and <= K";
  if (p.K1 < p.K && !p.A2) return "gemm: split-K operand A2 missing";
  if (p.a_rows_per_group < 0 || (p.a_rows_per_group > 0 && p.a_group_stride < p.a_rows_per_group))
    return "gemm: row gather needs a_group_stride >= a_rows_per_group";
  if (!p.A1 || !p.W) return "gemm: null operand";
  if ((p.lda1 % 8) || (p.K1 < p.K && (p.lda2 % 8))) return "gemm: lda must be a multiple of 8 (16-byte rows)";
  if (p.ldw && (p.ldw < p.K || p.ldw % 8)) return "gemm: ldw must be >= K and a multiple of 8";
  if (p.conv) {
    if (p.convC % BK || p.K != 9 * p.convC) return "gemm(conv): C_in must be a multiple of 64 and K = 9 * C_in";
    if (!p.zero || ((uintptr_t)p.zero & 15)) return "gemm(conv): zero page missing";
    if (p.A2 || p.a_rows_per_group) return "gemm(conv): no split-K / row gather in conv mode";
    if (p.conv_up && (p.convH % 2 || p.convW % 2)) return "gemm(conv): upsampled grid must be even";
  }
  if (((uintptr_t)p.A1 | (uintptr_t)p.W | (uintptr_t)(p.A2 ? p.A2 : p.A1)) & 15) return "gemm: operands must be 16-byte aligned";
  if (p.stats_out && ((epi != EPI_F32 && epi != EPI_RES) || p.stats_ld < (p.N + 255) / 256 || ((uintptr_t)p.stats_out & 7)))
    return "gemm: LayerNorm stats need the fp32 / residual epilogue and stats_ld >= ceil(N / 256)";
  if ((p.stats_out || p.ln_stats) && p.batch > 1) return "gemm: fused LayerNorm is not available for batched GEMMs";
  if ((p.out2 || p.stats_out2) && epi != EPI_RES) return "gemm: out2 / stats_out2 belong to the residual epilogue";
  if (p.out_fp8 && (p.N % 32 || p.ldo8 % 16 || !p.out_scale || p.out_scale_ld < p.M || p.batch > 1 ||
                    ((uintptr_t)p.out_fp8 & 15) || ((uintptr_t)p.out_scale & 3)))
    return "gemm: MXFP8 output needs N % 32 == 0, ldo8 % 16 == 0, a scale array with out_scale_ld >= M";
  if (p.fp8) {
    if (p.K % 128 || p.K1 != p.K || p.A2 || p.conv || p.a_rows_per_group || p.batch > 1)
      return "gemm(fp8): K must be a multiple of 128; no split-K, conv, row gather or batch";
    if (!p.a_scale || !p.w_scale || p.a_scale_ld < p.M || p.w_scale_ld < p.N || (p.lda1 % 16) || (p.ldw && p.ldw % 16))
      return "gemm(fp8): block scales missing or leading dimensions not multiples of 16 bytes";
    if (!fits_rsrc(p))
      return "gemm(fp8): an operand spans >= 2 GiB (32-bit buffer offsets); split M into smaller launches";
  }
  if (p.mx_center && (!p.out_fp8 || !p.stats_out || (epi != EPI_F32 && epi != EPI_RES)))
    return "gemm: mx_center needs the fp32 epilogue with both stats_out and the MXFP8 output";
  if (p.ln_gcol && (!p.fp8 || !p.ln_stats || p.ln_ld > 8 || ((uintptr_t)p.ln_gcol & 15)))
    return "gemm: ln_gcol (centred LayerNorm) needs an MXFP8 A operand, ln_stats with ln_D <= 2048 and 16-byte alignment";
  if (p.ln_stats) {
    if (!epi_rowout(epi)) return "gemm: the fused LayerNorm applies to the bf16 / GELU epilogues";
    if (!p.ln_colsum || ((uintptr_t)p.ln_colsum & 15) || p.ln_D <= 0 || p.ln_ld != (p.ln_D + 255) / 256)
      return "gemm: fused LayerNorm needs ln_colsum and ln_ld = ceil(ln_D / 256)";
  }
  if (epi == EPI_BF16 || epi == EPI_GELU) {
    // the MXFP8 copy alone is a valid output (fc1 -> fc2 operand of the fp8 forward)
    if ((!p.out_bf16 && !p.out_fp8 && !(g_gemm_dbg & 2)) || (p.out_bf16 && p.ldo % 4)) return "gemm: bf16 output missing or ldo not a multiple of 4";
  } else if (epi == EPI_RES) {
    if (!p.out_bf16 || p.ldo % 8 || ((uintptr_t)p.out_bf16 & 15)) return "gemm(residual): bf16 output with ldo % 8 == 0, 16-byte aligned";
    if (p.accumulate && (!p.res_in || p.ldri % 8 || ((uintptr_t)p.res_in & 15)))
      return "gemm(residual): accumulate needs res_in with ldri % 8 == 0, 16-byte aligned";
    if (p.N % 8 || p.batch > 1 || p.conv) return "gemm(residual): N % 8 == 0, no batch / conv";
    if (p.out2 && (p.out2_rpg <= 0 || p.out2_gs < p.out2_rpg || ((uintptr_t)p.out2 & 15) || p.out_fp8 ||
                   (p.stats_out2 && (!p.stats_out || ((uintptr_t)p.stats_out2 & 7)))))
      return "gemm(residual): out2 needs 0 < out2_rpg <= out2_gs, 16-byte alignment, no MXFP8 output; stats_out2 needs stats_out";
  } else if (epi == EPI_F32) {
    if (!p.out_f32 || (p.ldr % 4)) return "gemm: f32 output missing or ldr not a multiple of 4";
    if (p.res_f32 && (!p.accumulate || p.ldrf % 4 || ((uintptr_t)p.res_f32 & 15) || p.batch > 1))
      return "gemm: res_f32 needs accumulate, ldrf % 4 == 0, 16-byte alignment and no batch";
    if (p.out_bf16 && (p.ldo % 4)) return "gemm: ldo not a multiple of 4";
  } else {
    return "gemm: unknown epilogue";
  }
  return nullptr;
}

static int g_gemm_algo = 0;
// the MXFP8 residual GEMM (H/4 proj) on the persistent kernel under the automatic policy (an A/B build sets
// -DPDM_MX_RES_PERSIST=0 for gemm_mx_kernel<EPI_RES>)
#ifndef PDM_MX_RES_PERSIST
#define PDM_MX_RES_PERSIST 1
#endif
static bool g_mx_res_persist = PDM_MX_RES_PERSIST;
static int g_gemm_sk = 0;   // off by default: measured slower at every U-ViT shape (profiles/r05a, r05b)
static long long g_sk_launches = 0;   // stream-K launches so far (host count, tests)
void gemm_set_sk(int mode) { g_gemm_sk = mode; }
int gemm_get_sk() { return g_gemm_sk; }
long long gemm_sk_launches() { return g_sk_launches; }
int gemm_seg_stats(unsigned long long* out) {   // reads and clears the -DPDM_G8S_SEG counters (25; synchronises)
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_seg_stats), 25 * sizeof(unsigned long long)) != hipSuccess) return 1;
  unsigned long long z[25] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_seg_stats), z, sizeof(z)) != hipSuccess;
}
int gemm_sk_stats(unsigned long long* out) {   // reads and clears the device counters (synchronises the device)
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sk_stats), 3 * sizeof(unsigned long long)) != hipSuccess) return 1;
  const unsigned long long z[4] = {0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_sk_stats), z, sizeof(z)) != hipSuccess;
}
void gemm_set_tuning(int raster, int dbg_tile0) { g_gemm_raster = raster; g_gemm_dbg = dbg_tile0; }  // 0 auto, 1 = 128x128, 2 = 256x256 BK32 x4 ring, 3 = 256x256 BK64 x2, 4 = 256x256 8-phase
void gemm_set_algo(int algo) { g_gemm_algo = algo; }

template <int BK, int NS>
static hipError_t launch256(const GemmArgs& p, int epi, hipStream_t stream) {
  constexpr int SMEM = (BM2 + BN2) * BK * 2 * NS + EPI_LDS_EXTRA;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm256_kernel<EPI_BF16, BK, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    (void)hipFuncSetAttribute((const void*)gemm256_kernel<EPI_GELU, BK, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    (void)hipFuncSetAttribute((const void*)gemm256_kernel<EPI_F32, BK, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    attr_set = true;
  }
  const int tn = (p.N + BN2 - 1) / BN2, tm = (p.M + BM2 - 1) / BM2;
  const int nwg = tm * tn;
  dim3 grid(nwg, p.batch > 1 ? p.batch : 1), block(512);
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL((gemm256_kernel<EPI_BF16, BK, NS>), grid, block, SMEM, stream, p, tn, nwg); break;
    case EPI_GELU: hipLaunchKernelGGL((gemm256_kernel<EPI_GELU, BK, NS>), grid, block, SMEM, stream, p, tn, nwg); break;
    default: hipLaunchKernelGGL((gemm256_kernel<EPI_F32, BK, NS>), grid, block, SMEM, stream, p, tn, nwg); break;
  }
  return hipGetLastError();
}

template <int CONV>
static hipError_t launch8p(const GemmArgs& p, int epi, hipStream_t stream) {
  constexpr int SMEM = 2 * 4 * 128 * 128 + EPI_LDS_EXTRA;   // 128 KiB ring + LN row stats
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm8p_kernel<EPI_BF16, CONV>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    (void)hipFuncSetAttribute((const void*)gemm8p_kernel<EPI_GELU, CONV>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    (void)hipFuncSetAttribute((const void*)gemm8p_kernel<EPI_F32, CONV>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    attr_set = true;
  }
  const int tn = (p.N + BN2 - 1) / BN2, tm = (p.M + BM2 - 1) / BM2;
  const int nwg = tm * tn;
  dim3 grid(nwg, p.batch > 1 ? p.batch : 1), block(512);
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL((gemm8p_kernel<EPI_BF16, CONV>), grid, block, SMEM, stream, p, tn, nwg); break;
    case EPI_GELU: hipLaunchKernelGGL((gemm8p_kernel<EPI_GELU, CONV>), grid, block, SMEM, stream, p, tn, nwg); break;
    default: hipLaunchKernelGGL((gemm8p_kernel<EPI_F32, CONV>), grid, block, SMEM, stream, p, tn, nwg); break;
  }
  return hipGetLastError();
}

template <int CONV>
static hipError_t launch8t(const GemmArgs& p, int epi, hipStream_t stream) {
  constexpr int SMEM = 2 * 5 * 128 * 128;   // 160 KiB
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm8t_kernel<EPI_BF16, CONV>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    (void)hipFuncSetAttribute((const void*)gemm8t_kernel<EPI_F32, CONV>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    attr_set = true;
  }
  if (p.N > 128 || p.batch > 1 || (epi != EPI_BF16 && epi != EPI_F32)) return hipErrorInvalidValue;
  const int nwg = (p.M + 511) / 512;
  if (epi == EPI_BF16) hipLaunchKernelGGL((gemm8t_kernel<EPI_BF16, CONV>), dim3(nwg), dim3(512), SMEM, stream, p, nwg);
  else hipLaunchKernelGGL((gemm8t_kernel<EPI_F32, CONV>), dim3(nwg), dim3(512), SMEM, stream, p, nwg);
  return hipGetLastError();
}

template <int CONV>
static hipError_t launch8d_hn(const GemmArgs& p, int epi, hipStream_t stream) {
  constexpr int SMEM = 2 * 4 * 128 * 128 + EPI_LDS_EXTRA + COL_LDS_BYTES;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm8d_kernel<EPI_BF16, CONV, 2, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    (void)hipFuncSetAttribute((const void*)gemm8d_kernel<EPI_F32, CONV, 2, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    attr_set = true;
  }
  if (p.N > 128 || (epi != EPI_BF16 && epi != EPI_F32)) return hipErrorInvalidValue;
  const int nwg = (p.M + BM2 - 1) / BM2;
  dim3 grid(nwg, p.batch > 1 ? p.batch : 1), block(512);
  if (epi == EPI_BF16) hipLaunchKernelGGL((gemm8d_kernel<EPI_BF16, CONV, 2, 1>), grid, block, SMEM, stream, p, 1, nwg);
  else hipLaunchKernelGGL((gemm8d_kernel<EPI_F32, CONV, 2, 1>), grid, block, SMEM, stream, p, 1, nwg);
  return hipGetLastError();
}

template <int CONV, int SCHED>
static hipError_t launch8d(const GemmArgs& p, int epi, hipStream_t stream) {
  constexpr int SMEM = 2 * 4 * 128 * 128 + EPI_LDS_EXTRA + COL_LDS_BYTES;   // ring + LN rows + bias / colsum
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm8d_kernel<EPI_BF16, CONV, SCHED>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    (void)hipFuncSetAttribute((const void*)gemm8d_kernel<EPI_GELU, CONV, SCHED>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    (void)hipFuncSetAttribute((const void*)gemm8d_kernel<EPI_F32, CONV, SCHED>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    if constexpr (!CONV && SCHED == 2)
      (void)hipFuncSetAttribute((const void*)gemm8d_kernel<EPI_RES, 0, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    attr_set = true;
  }
  const int tn = (p.N + BN2 - 1) / BN2, tm = (p.M + BM2 - 1) / BM2;
  const int nwg = tm * tn;
  dim3 grid(nwg, p.batch > 1 ? p.batch : 1), block(512);
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL((gemm8d_kernel<EPI_BF16, CONV, SCHED>), grid, block, SMEM, stream, p, tn, nwg); break;
    case EPI_GELU: hipLaunchKernelGGL((gemm8d_kernel<EPI_GELU, CONV, SCHED>), grid, block, SMEM, stream, p, tn, nwg); break;
    case EPI_RES:
      if constexpr (!CONV && SCHED == 2) {
        hipLaunchKernelGGL((gemm8d_kernel<EPI_RES, 0, 2>), grid, block, SMEM, stream, p, tn, nwg);
        break;
      }
      return hipErrorInvalidValue;
    default: hipLaunchKernelGGL((gemm8d_kernel<EPI_F32, CONV, SCHED>), grid, block, SMEM, stream, p, tn, nwg); break;
  }
  return hipGetLastError();
}

static int g_num_cus = 0;
// q / nt0: the grouped launch's second problem and the first one's tile count (q = p, nt0 = all tiles: one problem)
static hipError_t launch8s(const GemmArgs& p, int epi, hipStream_t stream, const GemmArgs* p2 = nullptr) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm8s_kernel<EPI_BF16>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
    (void)hipFuncSetAttribute((const void*)gemm8s_kernel<EPI_GELU>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
    (void)hipFuncSetAttribute((const void*)gemm8s_kernel<EPI_RES>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
    (void)hipFuncSetAttribute((const void*)gemm8s_kernel<EPI_BF16, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
    (void)hipFuncSetAttribute((const void*)gemm8s_kernel<EPI_GELU, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
    (void)hipFuncSetAttribute((const void*)gemm8s_kernel<EPI_BF16, 0, 0, 0, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
    (void)hipFuncSetAttribute((const void*)gemm8s_kernel<EPI_GELU, 0, 0, 0, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
    (void)hipFuncSetAttribute((const void*)gemm8s_kernel<EPI_RES, 0, 0, 0, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
    (void)hipFuncSetAttribute((const void*)gemm8s_kernel<EPI_BF16, 1, 0, 0, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
    (void)hipFuncSetAttribute((const void*)gemm8s_kernel<EPI_GELU, 1, 0, 0, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      g_num_cus = n;
    else
      g_num_cus = 256;
    attr_set = true;
  }
  const int tn = (p.N + BN2 - 1) / BN2, tm = (p.M + BM2 - 1) / BM2;
  const int nt0 = tm * tn;
  const int ntiles = nt0 + (p2 ? (p2->M + BM2 - 1) / BM2 * tn : 0);
  const GemmArgs& q = p2 ? *p2 : p;
  const int grid = ntiles < g_num_cus ? ntiles : g_num_cus;
  // stream-K where the last wave of tiles leaves CUs idle and every workgroup's share is >= nk + 4 K-steps (so each
  // tile has at most two pieces and the consumer's tail normally finds its flag up, gemm8s_body)
  bool sk = false;
  if (!p2 && p.sk_flags && p.sk_slab && g_gemm_sk && ntiles > grid && grid <= SK_FLAG_WORDS && grid >= 8 &&
      ntiles % grid) {
    const int nk = p.K / 64, gx = (grid + 7) / 8, tmin = ntiles / 8;
    const int waves = (ntiles + grid - 1) / grid;
    const double fill = (double)ntiles / ((double)waves * grid);
    sk = (long long)tmin * nk >= (long long)gx * (nk + 4) && (g_gemm_sk == 2 || fill < 0.97);
  }
  if (sk) {
    ++g_sk_launches;
    static bool attr_sk = false;
    if (!attr_sk) {
      (void)hipFuncSetAttribute((const void*)gemm8s_kernel<EPI_BF16, 0, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
      (void)hipFuncSetAttribute((const void*)gemm8s_kernel<EPI_GELU, 0, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
      (void)hipFuncSetAttribute((const void*)gemm8s_kernel<EPI_RES, 0, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
      (void)hipFuncSetAttribute((const void*)gemm8s_kernel<EPI_BF16, 1, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
      (void)hipFuncSetAttribute((const void*)gemm8s_kernel<EPI_GELU, 1, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
      attr_sk = true;
    }
    if (p.out_fp8) {
      if (epi == EPI_BF16) hipLaunchKernelGGL((gemm8s_kernel<EPI_BF16, 1, 1>), dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles);
      else if (epi == EPI_GELU) hipLaunchKernelGGL((gemm8s_kernel<EPI_GELU, 1, 1>), dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles);
      else return hipErrorInvalidValue;
      return hipGetLastError();
    }
    switch (epi) {
      case EPI_BF16: hipLaunchKernelGGL((gemm8s_kernel<EPI_BF16, 0, 1>), dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles); break;
      case EPI_GELU: hipLaunchKernelGGL((gemm8s_kernel<EPI_GELU, 0, 1>), dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles); break;
      case EPI_RES: hipLaunchKernelGGL((gemm8s_kernel<EPI_RES, 0, 1>), dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  // the split-K second A operand (skip_linear's concat) needs the DUAL refill path; every other Linear takes DUAL = 0
  const bool dual = p.A2 && p.K1 < p.K;
  if (p.out_fp8) {   // fits_8s: bf16 / GELU with the MXFP8 copy as the only output
    if (epi == EPI_BF16 && dual) hipLaunchKernelGGL((gemm8s_kernel<EPI_BF16, 1>), dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles);
    else if (epi == EPI_BF16) hipLaunchKernelGGL((gemm8s_kernel<EPI_BF16, 1, 0, 0, 0>), dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles);
    else if (epi == EPI_GELU && dual) hipLaunchKernelGGL((gemm8s_kernel<EPI_GELU, 1>), dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles);
    else if (epi == EPI_GELU) hipLaunchKernelGGL((gemm8s_kernel<EPI_GELU, 1, 0, 0, 0>), dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (p2) {
    static bool attr_g = false;
    if (!attr_g) {
      (void)hipFuncSetAttribute((const void*)gemm8g_kernel<EPI_BF16>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
      (void)hipFuncSetAttribute((const void*)gemm8g_kernel<EPI_GELU>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
      (void)hipFuncSetAttribute((const void*)gemm8g_kernel<EPI_RES>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
      (void)hipFuncSetAttribute((const void*)gemm8g_kernel<EPI_BF16, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
      (void)hipFuncSetAttribute((const void*)gemm8g_kernel<EPI_GELU, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
      (void)hipFuncSetAttribute((const void*)gemm8g_kernel<EPI_RES, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, S_SMEM);
      attr_g = true;
    }
    // both problems share A2's presence and K1 (gemm_pair_groups)
    switch (epi) {
      case EPI_BF16:
        if (dual) hipLaunchKernelGGL(gemm8g_kernel<EPI_BF16>, dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles, view_of(q), nt0);
        else hipLaunchKernelGGL((gemm8g_kernel<EPI_BF16, 0>), dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles, view_of(q), nt0);
        break;
      case EPI_GELU:
        if (dual) hipLaunchKernelGGL(gemm8g_kernel<EPI_GELU>, dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles, view_of(q), nt0);
        else hipLaunchKernelGGL((gemm8g_kernel<EPI_GELU, 0>), dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles, view_of(q), nt0);
        break;
      case EPI_RES:
        if (dual) hipLaunchKernelGGL(gemm8g_kernel<EPI_RES>, dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles, view_of(q), nt0);
        else hipLaunchKernelGGL((gemm8g_kernel<EPI_RES, 0>), dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles, view_of(q), nt0);
        break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  switch (epi) {
    case EPI_BF16:
      if (dual) hipLaunchKernelGGL(gemm8s_kernel<EPI_BF16>, dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles);
      else hipLaunchKernelGGL((gemm8s_kernel<EPI_BF16, 0, 0, 0, 0>), dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles);
      break;
    case EPI_GELU:
      if (dual) hipLaunchKernelGGL(gemm8s_kernel<EPI_GELU>, dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles);
      else hipLaunchKernelGGL((gemm8s_kernel<EPI_GELU, 0, 0, 0, 0>), dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles);
      break;
    case EPI_RES:
      if (dual) hipLaunchKernelGGL(gemm8s_kernel<EPI_RES>, dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles);
      else hipLaunchKernelGGL((gemm8s_kernel<EPI_RES, 0, 0, 0, 0>), dim3(grid), dim3(512), S_SMEM, stream, p, tn, ntiles);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// the persistent kernel's preconditions (epilogues, no conv / batch / gather / MXFP8 operands, K >= 256, one A
// stride, buffer extents); an MXFP8 output only as the sole output of a bf16 / GELU epilogue (gemm_check has
// validated its shape: N % 32, ldo8 % 16, out_scale_ld >= M)
// The persistent kernel counts its VMEM ops by hand (the ring's vmcnt waits): a register spill would add scratch
// traffic it does not expect, so every instantiation is checked once for a private segment; with one, the
// persistent policy is off (whole-tile algo 7 instead) and the library says so on stderr.
static bool persist_kernels_ok() {
  static int ok = -1;
  if (ok < 0) {
    const void* fns[] = {(const void*)gemm8s_kernel<EPI_BF16>, (const void*)gemm8s_kernel<EPI_GELU>,
                         (const void*)gemm8s_kernel<EPI_RES>, (const void*)gemm8s_kernel<EPI_BF16, 1>,
                         (const void*)gemm8s_kernel<EPI_GELU, 1>, (const void*)gemm8s_kernel<EPI_BF16, 0, 1>,
                         (const void*)gemm8s_kernel<EPI_GELU, 0, 1>, (const void*)gemm8s_kernel<EPI_RES, 0, 1>,
                         (const void*)gemm8s_kernel<EPI_BF16, 1, 1>, (const void*)gemm8s_kernel<EPI_GELU, 1, 1>,
                         (const void*)gemm8g_kernel<EPI_BF16>, (const void*)gemm8g_kernel<EPI_GELU>,
                         (const void*)gemm8g_kernel<EPI_RES>, (const void*)gemm8s_kernel<EPI_BF16, 0, 0, 1, 0>,
                         (const void*)gemm8s_kernel<EPI_RES, 0, 0, 1, 0>, (const void*)gemm8s_kernel<EPI_BF16, 0, 0, 0, 0>,
                         (const void*)gemm8s_kernel<EPI_GELU, 0, 0, 0, 0>, (const void*)gemm8s_kernel<EPI_RES, 0, 0, 0, 0>,
                         (const void*)gemm8s_kernel<EPI_BF16, 1, 0, 0, 0>, (const void*)gemm8s_kernel<EPI_GELU, 1, 0, 0, 0>,
                         (const void*)gemm8g_kernel<EPI_BF16, 0>, (const void*)gemm8g_kernel<EPI_GELU, 0>,
                         (const void*)gemm8g_kernel<EPI_RES, 0>};
    ok = 1;
    for (const void* f : fns) {
      hipFuncAttributes at{};
      if (hipFuncGetAttributes(&at, f) != hipSuccess) continue;   // no device: the launch itself will fail
      if (at.localSizeBytes > 0) ok = 0;
    }
    if (!ok) fprintf(stderr, "libpdm: a persistent GEMM instantiation uses scratch (register spill); using algo 7\n");
  }
  return ok == 1;
}

static bool fits_8s(const GemmArgs& p, int epi) {
  const long long lim = 0x7fffffffLL;
  if (!persist_kernels_ok()) return false;
  if (epi != EPI_BF16 && epi != EPI_GELU && epi != EPI_RES) return false;
  if (p.conv || p.batch > 1 || p.a_rows_per_group > 0 || p.fp8 || p.mx_center || p.out2) return false;
  if (p.out_fp8) {
    if (epi == EPI_RES || p.out_bf16 || !p.out_scale || p.N % 32 || p.ldo8 % 16 || p.out_scale_ld < p.M) return false;
    if ((long long)p.M * p.ldo8 >= lim || (long long)((p.N + 127) >> 7) * p.out_scale_ld * 4 >= lim) return false;
    if (epi == EPI_GELU && p.act) return false;
    if (p.K < 256 || (p.A2 && p.K1 < p.K && p.lda2 != p.lda1) || (p.ln_stats && p.ln_ld > 8)) return false;
    if (p.dbg_tile0 & 15) return false;
    return fits_rsrc(p);
  }
  if (!p.out_bf16) return false;
  if (epi == EPI_GELU && p.act) return false;
  if (p.K < 256 || (p.A2 && p.K1 < p.K && p.lda2 != p.lda1) || p.N % 8 || p.ldo % 8 || ((uintptr_t)p.out_bf16 & 15) || (p.ln_stats && p.ln_ld > 8)) return false;
  if ((long long)p.M * p.ldo * 2 >= lim) return false;
  if (epi == EPI_RES && p.accumulate && (p.ldri % 8 || ((uintptr_t)p.res_in & 15) || (long long)p.M * p.ldri * 2 >= lim))
    return false;
  if (p.stats_out && (long long)p.M * p.stats_ld * 8 >= lim) return false;
  if (p.dbg_tile0 & 15) return false;   // gemm8d's timing modes
  return fits_rsrc(p);
}

// the persistent kernel's MXFP8-operand form (gemm8s_kernel<EPI, 0, 0, 1>): the bf16 epilogue with or without the
// (centred) LayerNorm consumer -- the U-ViT-H/4 qkv, algo 11 only -- and the bf16-residual epilogue without an MXFP8
// output copy -- the H/4 proj in 'fp8' mode (its x feeds the bf16 fc1), automatic where g_mx_res_persist allows
static bool fits_8s_mx(const GemmArgs& p, int epi) {
  const long long lim = 0x7fffffffLL;
  if (!persist_kernels_ok()) return false;
  if ((epi != EPI_BF16 && epi != EPI_RES) || !p.fp8 || p.out_fp8 || p.mx_center || p.A2 || p.K1 != p.K || p.conv ||
      p.batch > 1 || p.a_rows_per_group > 0 || p.out2)
    return false;
  if (!p.out_bf16 || p.N % 8 || p.ldo % 8 || ((uintptr_t)p.out_bf16 & 15) || p.K % 128 || p.K < 512) return false;
  if (p.ln_stats && p.ln_ld > 8) return false;
  if ((long long)p.M * p.ldo * 2 >= lim || (p.dbg_tile0 & 15)) return false;
  if (epi == EPI_RES && p.accumulate && (p.ldri % 8 || ((uintptr_t)p.res_in & 15) || (long long)p.M * p.ldri * 2 >= lim))
    return false;
  if (p.stats_out && (long long)p.M * p.stats_ld * 8 >= lim) return false;
  return fits_rsrc(p);
}

static hipError_t launch8s_mx(const GemmArgs& p, int epi, hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm8s_kernel<EPI_BF16, 0, 0, 1, 0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              S_SMEM_MX);
    (void)hipFuncSetAttribute((const void*)gemm8s_kernel<EPI_RES, 0, 0, 1, 0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              S_SMEM_MX);
    attr_set = true;
  }
  if (g_num_cus == 0) {   // as launch8s
    int dev = 0, n = 0;
    g_num_cus = (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0) ? n : 256;
  }
  const int tn = (p.N + BN2 - 1) / BN2, tm = (p.M + BM2 - 1) / BM2;
  const int ntiles = tm * tn;
  const int grid = ntiles < g_num_cus ? ntiles : g_num_cus;
  if (epi == EPI_RES)
    hipLaunchKernelGGL((gemm8s_kernel<EPI_RES, 0, 0, 1, 0>), dim3(grid), dim3(512), S_SMEM_MX, stream, p, tn, ntiles);
  else
    hipLaunchKernelGGL((gemm8s_kernel<EPI_BF16, 0, 0, 1, 0>), dim3(grid), dim3(512), S_SMEM_MX, stream, p, tn, ntiles);
  return hipGetLastError();
}

static hipError_t launch_mx(const GemmArgs& p, int epi, hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_mx_kernel<EPI_BF16>, hipFuncAttributeMaxDynamicSharedMemorySize, MX_SMEM);
    (void)hipFuncSetAttribute((const void*)gemm_mx_kernel<EPI_GELU>, hipFuncAttributeMaxDynamicSharedMemorySize, MX_SMEM);
    (void)hipFuncSetAttribute((const void*)gemm_mx_kernel<EPI_F32>, hipFuncAttributeMaxDynamicSharedMemorySize, MX_SMEM);
    (void)hipFuncSetAttribute((const void*)gemm_mx_kernel<EPI_RES>, hipFuncAttributeMaxDynamicSharedMemorySize, MX_SMEM);
    attr_set = true;
  }
  const int tn = (p.N + BN2 - 1) / BN2, tm = (p.M + BM2 - 1) / BM2;
  const int nwg = tm * tn;
  dim3 grid(nwg), block(512);
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL(gemm_mx_kernel<EPI_BF16>, grid, block, MX_SMEM, stream, p, tn, nwg); break;
    case EPI_GELU: hipLaunchKernelGGL(gemm_mx_kernel<EPI_GELU>, grid, block, MX_SMEM, stream, p, tn, nwg); break;
    case EPI_RES: hipLaunchKernelGGL(gemm_mx_kernel<EPI_RES>, grid, block, MX_SMEM, stream, p, tn, nwg); break;
    default: hipLaunchKernelGGL(gemm_mx_kernel<EPI_F32>, grid, block, MX_SMEM, stream, p, tn, nwg); break;
  }
  return hipGetLastError();
}

// The descriptor-addressed kernel needs every operand byte offset below 2^31 (32-bit per-lane offsets).
static bool fits_rsrc(const GemmArgs& p) {
  const long long lim = 0x7fffffffLL;
  const long long es = p.fp8 ? 1 : 2;   // operand bytes per element (MXFP8 rows are e4m3 bytes)
  long long a1;
  if (p.conv) a1 = (long long)(p.M / (p.convH * p.convW)) * (p.convH >> p.conv_up) * (p.convW >> p.conv_up) * p.convC * 2;
  else if (p.a_rows_per_group > 0)
    a1 = ((long long)((p.M - 1) / p.a_rows_per_group) * p.a_group_stride + p.a_rows_per_group) * p.lda1 * es;
  else a1 = (long long)p.M * p.lda1 * es;
  const long long a2 = p.A2 ? (long long)p.M * p.lda2 * 2 : 0;
  const long long w = (long long)p.N * (p.ldw > 0 ? p.ldw : p.K) * es;
  return a1 < lim && a2 < lim && w < lim &&
         (!p.conv || (p.convW <= 512 && p.convH <= 512 && p.M / (p.convH * p.convW) < 8192));   // conv_off's packing
}

// the second residual output of a launch whose kernel has no out2 store (the 128 tile, a split launch): the rows
// (and partials) copied from out_bf16 / stats_out after it, as 4-byte words
static hipError_t out2_copy(const GemmArgs& p, hipStream_t stream) {
  return rowcopy_launch(reinterpret_cast<float*>(p.out2), p.ldo / 2, reinterpret_cast<const float*>(p.out_bf16),
                        p.ldo / 2, p.M, p.N / 2, p.out2_rpg, p.out2_gs, p.out2_rpg, stream, p.stats_out2,
                        p.stats_ld * 2, p.stats_out, p.stats_ld * 2, p.stats_out2 ? p.stats_ld * 2 : 0);
}

bool gemm_pair_groups(const GemmArgs& p, const GemmArgs& q, int epi) {
  const bool algo_ok = g_gemm_algo == 0 || g_gemm_algo == 11;
  const bool same = p.N == q.N && p.K == q.K && p.K1 == q.K1 && p.lda1 == q.lda1 && p.ldw == q.ldw && p.ldo == q.ldo &&
                    p.ldri == q.ldri && p.accumulate == q.accumulate && p.stats_ld == q.stats_ld && p.ln_ld == q.ln_ld &&
                    p.ln_D == q.ln_D && p.ln_eps == q.ln_eps && !p.bias == !q.bias && !p.ln_stats == !q.ln_stats &&
                    !p.stats_out == !q.stats_out && !p.A2 == !q.A2 && (!p.A2 || p.lda2 == q.lda2) && !p.out_fp8 && !q.out_fp8;
  // grouped only where each GEMM alone would take the persistent kernel (gemm_launch's rule), so a problem's
  // arithmetic -- and the sampler's batch invariance -- does not depend on the other problem's rows
  return algo_ok && same && p.M >= 4096 && q.M >= 4096 && p.N >= 256 && fits_8s(p, epi) && fits_8s(q, epi);
}

hipError_t gemm_launch_pair(const GemmArgs& a, const GemmArgs& b, int epi, hipStream_t stream) {
  GemmArgs p = a, q = b;
  p.raster = q.raster = g_gemm_raster ? g_gemm_raster : (p.N >= 8 * BN2 ? 8 : 0);
  p.dbg_tile0 = q.dbg_tile0 = g_gemm_dbg;
  if (gemm_pair_groups(p, q, epi)) return launch8s(p, epi, stream, &q);
  GemmArgs a1 = a, b1 = b;   // one flag block serves one launch
  a1.sk_flags = b1.sk_flags = nullptr;
  a1.sk_slab = b1.sk_slab = nullptr;
  const hipError_t e = gemm_launch(a1, epi, stream);
  return e != hipSuccess ? e : gemm_launch(b1, epi, stream);
}

// GemmArgs::gn_part: only the gemm8d (algo 7) and gemm8t (algo 9) epilogues write GroupNorm partials, on whole
// 256-row tiles of whole images; mirrors gemm_launch's automatic choice for conv / fp32 launches
bool gemm_gn_fusable(const GemmArgs& p, int epi) {
  if (g_gemm_algo != 0 || (epi != EPI_F32 && epi != EPI_BF16) || !(p.conv || epi == EPI_F32)) return false;
  if (p.fp8 || p.out_fp8 || p.batch > 1 || p.a_rows_per_group > 0 || p.ln_stats || p.stats_out || p.A2) return false;
  if (p.gn_P <= 0 || p.gn_P % 256 || p.M % p.gn_P || p.N % 32 || p.gn_cpg * 32 != p.N) return false;
  if (p.gn_cpg != 4 && p.gn_cpg != 8 && p.gn_cpg != 16 && p.gn_cpg != 32) return false;
  const bool a7 = p.M >= 4096 && p.N >= 256, a9 = p.M >= 65536 && p.N > 96 && p.N <= 128;
  if (!a7 && !a9) return false;
  if (epi == EPI_BF16 && (p.N % 8 || p.ldo % 8 || ((uintptr_t)p.out_bf16 & 15) || !p.out_bf16)) return false;
  if (epi == EPI_F32 && (p.N % 8 || p.ldr % 4 || ((uintptr_t)p.out_f32 & 15) ||
                         (p.out_bf16 && (p.ldo % 8 || ((uintptr_t)p.out_bf16 & 15)))))
    return false;
  return fits_rsrc(p) || p.conv;   // conv: gemm_launch splits past 2 GiB by whole images
}

hipError_t gemm_launch(const GemmArgs& args, int epi, hipStream_t stream) {
  if (args.gn_part && !gemm_gn_fusable(args, epi)) return hipErrorInvalidValue;
  GemmArgs p = args;
  // tile order: groups of 8 row panels once there are >= 8 column tiles (an XCD's 32 resident tiles then share
  // 4 A and 8 W panels instead of 2 and 16); measured by tools/gemm_tune.py
  p.raster = g_gemm_raster ? g_gemm_raster : (p.N >= 8 * BN2 ? 8 : 0);
  p.dbg_tile0 = g_gemm_dbg;
  int algo = g_gemm_algo;
  const long long rows_all = (long long)p.M * (p.batch > 1 ? p.batch : 1);
  // batched GEMMs (decoder AttnBlock q k^T and p v, 1024 rows per image at 256^2) count all batches' rows
  // 96 < N <= 128 with many rows (the decoder's 128-channel 512^2 convs and nin_shortcut): the 512 x 128 tall
  // tile, algo 9 (conv 128 -> 128 at 512^2 x 8 images: 870 us vs 1059 us on the 128 tile; the 256 x 128 half-N
  // tile, algo 8, measured 1070 us and is kept as an option only: tools/conv_bench.py, profiles/r03q)
  if (algo == 0) {
    algo = (rows_all >= 4096 && p.N >= 256) ? 7 : (rows_all >= 65536 && p.N > 96 && p.N <= 128 && p.batch <= 1) ? 9 : 1;
    if (algo == 7 && fits_8s(p, epi)) algo = 11;   // the persistent kernel where its epilogues apply
  }
  if (algo == 11) {
    if (!p.fp8 && fits_8s(p, epi)) return launch8s(p, epi, stream);
    algo = 7;
  }
  if ((algo == 8 || algo == 9) && (p.N > 128 || (epi != EPI_BF16 && epi != EPI_F32) || p.ln_stats || p.stats_out ||
                                    p.out_fp8 || p.a_rows_per_group > 0 || (algo == 9 && p.batch > 1))) algo = 1;
  // the 256-tile bf16 epilogue stores 16-byte row chunks: needs N, ldo multiples of 8 and an aligned output
  if ((epi == EPI_BF16 || epi == EPI_GELU) && (p.N % 8 || p.ldo % 8 || ((uintptr_t)p.out_bf16 & 15))) algo = 1;
  if (epi == EPI_F32 && (p.N % 8 || p.ldr % 4 || ((uintptr_t)p.out_f32 & 15) ||
                         (p.out_bf16 && (p.ldo % 8 || ((uintptr_t)p.out_bf16 & 15))))) algo = 1;
  if (p.fp8) {
    if (!fits_rsrc(p)) return hipErrorInvalidValue;
    // the persistent form under the automatic policy from 16 sequences of 258 tokens up (round 6, after its
    // issue-path changes): the H/4 forward at the bench's 50-row lanes 13.12 -> 12.99 ms with it on every MXFP8
    // shape (qkv with the centred LayerNorm consumer, proj, fc2; tools/forward_algo_ab.py, profiles/r06al); the
    // residual form alone: 64.3 -> 57.2 us at 100 rows, parity at 25-50 (tools/mx_res_bench.py, profiles/r06v)
    if ((g_gemm_algo == 11 || (g_gemm_algo == 0 && g_mx_res_persist && p.M >= 4096)) && fits_8s_mx(p, epi))
      return launch8s_mx(p, epi, stream);
    return launch_mx(p, epi, stream);
  }
  if (p.out_fp8) algo = 7;   // MXFP8 output lives in the 256-tile epilogue
  // no-store timing mode (pdm_set_gemm_tuning bit 1, gemm_check): only the 256-tile epilogue skips a missing output
  if ((epi == EPI_BF16 || epi == EPI_GELU) && !p.out_bf16 && !p.out_fp8) {
    if (!fits_rsrc(p) || p.conv || p.batch > 1) return hipErrorInvalidValue;
    algo = 7;
  }
  // operands past the descriptor kernels' 2 GiB byte-offset range (e.g. a 32-image chunk of 512^2 x 256-channel
  // conv inputs): split the rows into parts that fit -- whole images for a conv -- instead of dropping to the
  // 128-tile kernel
  if (algo >= 5 && !fits_rsrc(p) && p.batch <= 1 && p.a_rows_per_group == 0 && !p.out_fp8) {
    const int hw = p.conv ? p.convH * p.convW : 1;
    const int m1 = p.conv ? (p.M / hw / 2) * hw : ((p.M / 2 + BM2 - 1) / BM2) * BM2;
    if (m1 > 0 && m1 < p.M) {
      GemmArgs a = args, b = args;
      a.sk_flags = b.sk_flags = nullptr;   // one flag block serves one launch
      a.sk_slab = b.sk_slab = nullptr;
      a.out2 = b.out2 = nullptr;           // the second output: one copy after both parts
      a.stats_out2 = b.stats_out2 = nullptr;
      a.M = m1;
      b.M = p.M - m1;
      if (p.conv) b.A1 += (size_t)(m1 / hw) * (p.convH >> p.conv_up) * (p.convW >> p.conv_up) * p.convC;
      else {
        b.A1 += (size_t)m1 * p.lda1;
        if (b.A2) b.A2 += (size_t)m1 * p.lda2;
      }
      if (b.out_bf16) b.out_bf16 += (size_t)m1 * p.ldo;
      if (b.out_f32) b.out_f32 += (size_t)m1 * p.ldr;
      if (b.res_in) b.res_in += (size_t)m1 * p.ldri;
      if (b.res_f32) b.res_f32 += (size_t)m1 * p.ldrf;
      if (b.stats_out) b.stats_out += (size_t)m1 * p.stats_ld * 2;
      if (b.ln_stats) b.ln_stats += (size_t)m1 * p.ln_ld * 2;
      if (b.gn_part) b.gn_part += (size_t)(m1 / p.gn_P) * (p.gn_P >> 8) * 64;   // whole images (conv split)
      hipError_t e = gemm_launch(a, epi, stream);
      if (e == hipSuccess) e = gemm_launch(b, epi, stream);
      if (e == hipSuccess && p.out2) e = out2_copy(p, stream);
      return e;
    }
  }
  if (algo == 8 && fits_rsrc(p)) return p.conv ? launch8d_hn<1>(p, epi, stream) : launch8d_hn<0>(p, epi, stream);
  if (algo == 9 && fits_rsrc(p)) return p.conv ? launch8t<1>(p, epi, stream) : launch8t<0>(p, epi, stream);
  if (algo == 8 || algo == 9) algo = 1;
  if (epi == EPI_RES) {      // the residual epilogue exists in the default 256-tile schedule and the 128 tile
    if (algo != 1 && fits_rsrc(p)) return launch8d<0, 2>(p, epi, stream);
    algo = 1;
  }
  if (algo >= 5 && fits_rsrc(p)) {
    if (algo == 5) return p.conv ? launch8d<1, 0>(p, epi, stream) : launch8d<0, 0>(p, epi, stream);
    if (algo == 6) return p.conv ? launch8d<1, 1>(p, epi, stream) : launch8d<0, 1>(p, epi, stream);
    return p.conv ? launch8d<1, 2>(p, epi, stream) : launch8d<0, 2>(p, epi, stream);
  }
  if (algo >= 5) algo = 3;
  if (algo == 2 && p.K % 32 == 0) return launch256<32, 4>(p, epi, stream);
  if (algo == 4 && p.K % 128 == 0) return p.conv ? launch8p<1>(p, epi, stream) : launch8p<0>(p, epi, stream);
  if ((algo == 3 || algo == 4) && p.K % 64 == 0) return launch256<64, 2>(p, epi, stream);
  const int tiles_n = (p.N + BN - 1) / BN;
  const int tiles_m = (p.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  dim3 grid(nwg, p.batch > 1 ? p.batch : 1), block(256);
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL(gemm_bf16_kernel<EPI_BF16>, grid, block, SMEM_BYTES, stream, p, tiles_n, nwg); break;
    case EPI_GELU: hipLaunchKernelGGL(gemm_bf16_kernel<EPI_GELU>, grid, block, SMEM_BYTES, stream, p, tiles_n, nwg); break;
    case EPI_RES: hipLaunchKernelGGL(gemm_bf16_kernel<EPI_RES>, grid, block, SMEM_BYTES, stream, p, tiles_n, nwg); break;
    default: hipLaunchKernelGGL(gemm_bf16_kernel<EPI_F32>, grid, block, SMEM_BYTES, stream, p, tiles_n, nwg); break;
  }
  hipError_t e = hipGetLastError();
  // the 128-tile epilogue spreads a row over two waves: its LayerNorm partials come from a row pass instead
  if (e == hipSuccess && p.stats_out && p.batch <= 1) {
    if (epi == EPI_RES) e = rowstats_bf16_launch(p.out_bf16, p.ldo, p.M, p.N, p.stats_out, p.stats_ld, stream);
    else e = rowstats_launch(p.out_f32, p.ldr, p.M, p.N, nullptr, 0, p.stats_out, p.stats_ld, stream);
  }
  if (e == hipSuccess && epi == EPI_RES && p.out2) e = out2_copy(p, stream);
  return e;
}

}  // namespace pdm

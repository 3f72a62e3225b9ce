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
#include "pdm_common.h"
#include "pdm_kernels.h"

namespace pdm {

namespace {
constexpr int BM = 128, BN = 128, BK = 64;
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
      if (p.a_rows_per_group > 0 && k0 < p.K1) gm = (gm / p.a_rows_per_group) * p.a_group_stride + gm % p.a_rows_per_group;
      glds16(Ab + (size_t)gm * lda + ka + c * 8, (PDM_LDS void*)(sa + rg * 1024));
      int gn = n0 + row;
      gn = gn < p.N ? gn : p.N - 1;
      glds16(p.W + (size_t)gn * p.K + k0 + c * 8, (PDM_LDS void*)(sw + rg * 1024));
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
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = n0 + wn * 64 + ni * 16 + (lane >> 4) * 4;
    if (n >= p.N) continue;  // N % 4 == 0: a lane's 4 columns are all in or all out
    f32x4 b = f32x4{0.f, 0.f, 0.f, 0.f};
    if (p.bias) b = *reinterpret_cast<const f32x4*>(p.bias + n);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int m = m0 + wm * 64 + mi * 16 + (lane & 15);
      if (m >= p.M) continue;
      f32x4 v = acc[ni][mi] + b;
      if constexpr (EPI == EPI_BF16) {
        *reinterpret_cast<bf16x4*>(p.out_bf16 + (size_t)m * p.ldo + n) = to_bf16x4(v[0], v[1], v[2], v[3]);
      } else if constexpr (EPI == EPI_GELU) {
        *reinterpret_cast<bf16x4*>(p.out_bf16 + (size_t)m * p.ldo + n) =
            to_bf16x4(gelu_erf(v[0]), gelu_erf(v[1]), gelu_erf(v[2]), gelu_erf(v[3]));
      } else {
        f32x4* r = reinterpret_cast<f32x4*>(p.out_f32 + (size_t)m * p.ldr + n);
        if (p.accumulate) v += *r;
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

  const int prow = lane / CPR;
  const int pch = lane % CPR;
  const bf16* asrc[PPW];
  const bf16* a2src[PPW];
  const bf16* wsrc[PPW];
  int soff[PPW];
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
    int gn = n0 + row;
    gn = gn < p.N ? gn : p.N - 1;
    wsrc[i] = p.W + (size_t)gn * p.K;
  }

  auto issue = [&](int j) {
    const int k0 = j * BK;
    char* slot = smem + (j % NS) * SLOT;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int piece = wave * PPW + i;
      const bf16* src = (k0 < p.K1) ? asrc[i] + k0 + soff[i] : a2src[i] + (k0 - p.K1) + soff[i];
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

  if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU) {
    // bf16 epilogue staged through LDS (the ring is free now): the 256x256 bf16 tile (128 KiB) is written
    // with a row-XOR chunk swizzle, then stored row-contiguously with 16-byte stores (full lines, half the
    // store instructions of the per-lane 8-byte scatter).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int nl = wn * 64 + ni * 16 + (lane >> 4) * 4;       // column within the tile
      const int n = n0 + nl;
      f32x4 b = f32x4{0.f, 0.f, 0.f, 0.f};
      if (p.bias && n < p.N) b = *reinterpret_cast<const f32x4*>(p.bias + n);
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        const int ml = wm * 128 + mi * 16 + (lane & 15);
        f32x4 v = acc[ni][mi] + b;
        if constexpr (EPI == EPI_GELU) {
          v[0] = gelu_erf(v[0]); v[1] = gelu_erf(v[1]); v[2] = gelu_erf(v[2]); v[3] = gelu_erf(v[3]);
        }
        const int off = ml * 512 + ((((nl >> 3) ^ (ml & 31)) << 4) | ((nl & 4) << 1));
        *reinterpret_cast<bf16x4*>(smem + off) = to_bf16x4(v[0], v[1], v[2], v[3]);
      }
    }
    __syncthreads();
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
      const int idx = it * 512 + tid;
      const int ml = idx >> 5, ch = idx & 31;
      const int m = m0 + ml, n = n0 + ch * 8;
      const i32x4 v = *reinterpret_cast<const i32x4*>(smem + ml * 512 + ((ch ^ (ml & 31)) << 4));
      if (m < p.M && n < p.N) *reinterpret_cast<i32x4*>(p.out_bf16 + (size_t)m * p.ldo + n) = v;
    }
    return;
  }
  // fp32 residual epilogue staged through LDS in two 128-row passes (128 KiB each): the accumulator tile
  // is written with a row-XOR chunk swizzle, then every thread owns 8 consecutive columns of a row:
  // 2 x 16-byte residual loads, 2 x 16-byte stores and one 16-byte bf16 copy store per row chunk.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (wm == pass) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int nl = wn * 64 + ni * 16 + (lane >> 4) * 4;
        const int n = n0 + nl;
        f32x4 b = f32x4{0.f, 0.f, 0.f, 0.f};
        if (p.bias && n < p.N) b = *reinterpret_cast<const f32x4*>(p.bias + n);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
          const int ml = mi * 16 + (lane & 15);
          *reinterpret_cast<f32x4*>(smem + ml * 1024 + (((nl >> 2) ^ (ml & 63)) << 4)) = acc[ni][mi] + b;
        }
      }
    }
    __syncthreads();
#pragma unroll 2
    for (int it = 0; it < 8; ++it) {
      const int idx = it * 512 + tid;
      const int ml = idx >> 5, c8 = idx & 31;
      const int m = m0 + pass * 128 + ml, n = n0 + c8 * 8;
      f32x4 v0 = *reinterpret_cast<const f32x4*>(smem + ml * 1024 + (((2 * c8) ^ (ml & 63)) << 4));
      f32x4 v1 = *reinterpret_cast<const f32x4*>(smem + ml * 1024 + (((2 * c8 + 1) ^ (ml & 63)) << 4));
      if (m < p.M && n < p.N) {
        f32x4* r = reinterpret_cast<f32x4*>(p.out_f32 + (size_t)m * p.ldr + n);
        if (p.accumulate) {
          v0 += r[0];
          v1 += r[1];
        }
        r[0] = v0;
        r[1] = v1;
        if (p.out_bf16) {
          bf16x8 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) { o[j] = (bf16)v0[j]; o[4 + j] = (bf16)v1[j]; }
          *reinterpret_cast<bf16x8*>(p.out_bf16 + (size_t)m * p.ldo + n) = o;
        }
      }
    }
    __syncthreads();
  }
}
}  // namespace

const char* gemm_check(const GemmArgs& p, int epi) {
  if (p.M <= 0 || p.N <= 0 || p.K <= 0) return "gemm: M, N, K must be positive";
  if (p.N % 4) return "gemm: N must be a multiple of 4";
  if (p.K % BK) return "gemm: K must be a multiple of 64";
  if (p.K1 % BK || p.K1 <= 0 || p.K1 > p.K) return "gemm: K1 must be a positive multiple of 64 and <= K";
  if (p.K1 < p.K && !p.A2) return "gemm: split-K operand A2 missing";
  if (!p.A1 || !p.W) return "gemm: null operand";
  if ((p.lda1 % 8) || (p.K1 < p.K && (p.lda2 % 8))) return "gemm: lda must be a multiple of 8 (16-byte rows)";
  if (((uintptr_t)p.A1 | (uintptr_t)p.W | (uintptr_t)(p.A2 ? p.A2 : p.A1)) & 15) return "gemm: operands must be 16-byte aligned";
  if (epi == EPI_BF16 || epi == EPI_GELU) {
    if (!p.out_bf16 || (p.ldo % 4)) return "gemm: bf16 output missing or ldo not a multiple of 4";
  } else if (epi == EPI_F32) {
    if (!p.out_f32 || (p.ldr % 4)) return "gemm: f32 output missing or ldr not a multiple of 4";
    if (p.out_bf16 && (p.ldo % 4)) return "gemm: ldo not a multiple of 4";
  } else {
    return "gemm: unknown epilogue";
  }
  return nullptr;
}

static int g_gemm_algo = 0;  // 0 auto, 1 = 128x128, 2 = 256x256 BK32 x4 ring, 3 = 256x256 BK64 x2
void gemm_set_algo(int algo) { g_gemm_algo = algo; }

template <int BK, int NS>
static hipError_t launch256(const GemmArgs& p, int epi, hipStream_t stream) {
  constexpr int SMEM = (BM2 + BN2) * BK * 2 * NS;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm256_kernel<EPI_BF16, BK, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    (void)hipFuncSetAttribute((const void*)gemm256_kernel<EPI_GELU, BK, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    (void)hipFuncSetAttribute((const void*)gemm256_kernel<EPI_F32, BK, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    attr_set = true;
  }
  const int tn = (p.N + BN2 - 1) / BN2, tm = (p.M + BM2 - 1) / BM2;
  const int nwg = tm * tn;
  dim3 grid(nwg), block(512);
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL((gemm256_kernel<EPI_BF16, BK, NS>), grid, block, SMEM, stream, p, tn, nwg); break;
    case EPI_GELU: hipLaunchKernelGGL((gemm256_kernel<EPI_GELU, BK, NS>), grid, block, SMEM, stream, p, tn, nwg); break;
    default: hipLaunchKernelGGL((gemm256_kernel<EPI_F32, BK, NS>), grid, block, SMEM, stream, p, tn, nwg); break;
  }
  return hipGetLastError();
}

hipError_t gemm_launch(const GemmArgs& p, int epi, hipStream_t stream) {
  int algo = g_gemm_algo;
  if (algo == 0) algo = (p.M >= 4096 && p.N >= 512) ? 3 : 1;
  // the 256-tile bf16 epilogue stores 16-byte row chunks: needs N, ldo multiples of 8 and an aligned output
  if ((epi == EPI_BF16 || epi == EPI_GELU) && (p.N % 8 || p.ldo % 8 || ((uintptr_t)p.out_bf16 & 15))) algo = 1;
  if (epi == EPI_F32 && (p.N % 8 || p.ldr % 4 || ((uintptr_t)p.out_f32 & 15) ||
                         (p.out_bf16 && (p.ldo % 8 || ((uintptr_t)p.out_bf16 & 15))))) algo = 1;
  if (algo == 2 && p.K % 32 == 0) return launch256<32, 4>(p, epi, stream);
  if (algo == 3 && p.K % 64 == 0) return launch256<64, 2>(p, epi, stream);
  const int tiles_n = (p.N + BN - 1) / BN;
  const int tiles_m = (p.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  dim3 grid(nwg), block(256);
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL(gemm_bf16_kernel<EPI_BF16>, grid, block, SMEM_BYTES, stream, p, tiles_n, nwg); break;
    case EPI_GELU: hipLaunchKernelGGL(gemm_bf16_kernel<EPI_GELU>, grid, block, SMEM_BYTES, stream, p, tiles_n, nwg); break;
    default: hipLaunchKernelGGL(gemm_bf16_kernel<EPI_F32>, grid, block, SMEM_BYTES, stream, p, tiles_n, nwg); break;
  }
  return hipGetLastError();
}

}  // namespace pdm

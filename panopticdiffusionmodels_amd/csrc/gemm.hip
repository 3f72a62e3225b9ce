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

hipError_t gemm_launch(const GemmArgs& p, int epi, hipStream_t stream) {
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

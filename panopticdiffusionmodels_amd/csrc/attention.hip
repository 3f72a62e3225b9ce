// Fused multi-head self-attention for U-ViT tokens (gfx950).
//
// Restates libs/uvit.py:66-92 (flash branch): per (b, h), softmax(Q K^T * Dh^-1/2) V with no mask, read
// straight out of the packed qkv GEMM output (token-major, (3, H, Dh) columns) and written token-major
// (H, Dh) for the proj GEMM -- no rearrange pass.  Awkward lengths (L = 257, 258, 334, 590) are handled by
// key masking and clamped loads; Dh = 72 (U-ViT-H) is padded to 96 for the QK^T k-steps.
//
// One wave owns 16 queries; a workgroup is 4 waves (64 consecutive queries of one (b, h)).  Keys stream
// through LDS in chunks of 64 with an online softmax.  S^T = K Q^T is computed (K as the MFMA A operand),
// so each lane holds 4 consecutive keys of one query: the softmax row statistics need only two xor-shuffles
// and P^T feeds the P V MFMA as its B operand with no lane movement (the k order inside a 32-key step is
// permuted consistently on both operands).  V^T fragments come from ds_read_b64_tr_b16 transposed reads of
// the row-major V chunk.
#include "pdm_common.h"
#include "pdm_kernels.h"

namespace pdm {

namespace {

__device__ __forceinline__ s16x4 lds_read_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((PDM_LDS s16x4*)(p));
}

template <int DH>
__global__ __launch_bounds__(256) void attention_kernel(AttentionArgs p, int nqt) {
  constexpr int KC = 64;
  constexpr int DHP = (DH + 31) / 32 * 32;
  constexpr int NKS = DHP / 32;
  constexpr int NDT = (DH + 15) / 16;
  constexpr int KSTR = DHP * 2 + 16;   // bytes; conflict-free ds_read_b128 column slices
  constexpr int VSTR = DHP * 2 + 32;   // bytes; conflict-free ds_read_b64_tr_b16
  constexpr int PIECES = KC * DH / 8;  // 16-byte pieces per K (or V) chunk
  constexpr int NP = (PIECES + 255) / 256;
  __shared__ __attribute__((aligned(16))) char Ks[KC * KSTR];
  __shared__ __attribute__((aligned(16))) char Vs[KC * VSTR];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // 1-D grid; blocks b and b+8 share an XCD (round-robin dispatch, placement affects speed only): give
  // every query block of one (b, h) the same bid % 8 so its K/V chunks are re-read from that XCD's L2.
  const int nqb = (nqt + 3) / 4;
  const int bid = blockIdx.x;
  const int grp = bid / (8 * nqb), rem = bid % (8 * nqb);
  const int bh = grp * 8 + (rem & 7);
  const int qb = rem >> 3;
  if (bh >= p.B * p.H) return;
  const int b = bh / p.H, h = bh % p.H;
  const int qt = qb * 4 + wave;
  const bool active = qt < nqt;
  const int L = p.L, D = p.H * DH;
  const bf16* base = p.qkv + (size_t)b * L * p.ldq;
  const int g = lane >> 4, col = lane & 15;

  // zero the padded head columns once (never overwritten by the chunk loads)
  if constexpr (DHP > DH) {
    for (int i = tid; i < KC * (DHP - DH) / 8; i += 256) {
      const int r = i / ((DHP - DH) / 8), j = i % ((DHP - DH) / 8);
      *reinterpret_cast<int4*>(Ks + r * KSTR + (DH + j * 8) * 2) = int4{0, 0, 0, 0};
      *reinterpret_cast<int4*>(Vs + r * VSTR + (DH + j * 8) * 2) = int4{0, 0, 0, 0};
    }
  }

  // Q^T fragments (B operand): lane holds Q[q = qt*16 + col][d = ks*32 + g*8 .. +8]
  bf16x8 qf[NKS];
  {
    int q = qt * 16 + col;
    q = q < L ? q : L - 1;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int d0 = ks * 32 + g * 8;
      if (d0 < DH) qf[ks] = *reinterpret_cast<const bf16x8*>(base + (size_t)q * p.ldq + h * DH + d0);
      else qf[ks] = bf16x8{};
    }
  }

  i32x4 kreg[NP], vreg[NP];
#define PDM_ATT_PREFETCH(cc)                                                            \
  _Pragma("unroll") for (int i = 0; i < NP; ++i) {                                     \
    const int pi = tid + i * 256;                                                      \
    if (pi < PIECES) {                                                                 \
      const int r = pi / (DH / 8), j = pi % (DH / 8);                                  \
      int key = (cc) * KC + r;                                                         \
      key = key < L ? key : L - 1;                                                     \
      const bf16* rowp = base + (size_t)key * p.ldq + h * DH + j * 8;                  \
      kreg[i] = *reinterpret_cast<const i32x4*>(rowp + D);                              \
      vreg[i] = *reinterpret_cast<const i32x4*>(rowp + 2 * D);                          \
    }                                                                                  \
  }
#define PDM_ATT_COMMIT()                                                                \
  _Pragma("unroll") for (int i = 0; i < NP; ++i) {                                     \
    const int pi = tid + i * 256;                                                      \
    if (pi < PIECES) {                                                                 \
      const int r = pi / (DH / 8), j = pi % (DH / 8);                                  \
      *reinterpret_cast<i32x4*>(Ks + r * KSTR + j * 16) = kreg[i];                      \
      *reinterpret_cast<i32x4*>(Vs + r * VSTR + j * 16) = vreg[i];                      \
    }                                                                                  \
  }

  const float sl2 = p.scale * 1.4426950408889634f;
  float m_run = -1e30f, l_run = 0.f;
  f32x4 acc[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nch = (L + KC - 1) / KC;
  PDM_ATT_PREFETCH(0)
  for (int c = 0; c < nch; ++c) {
    __syncthreads();
    PDM_ATT_COMMIT()
    __syncthreads();
    if (c + 1 < nch) { PDM_ATT_PREFETCH(c + 1) }
    if (active) {
      f32x4 s[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + (kt * 16 + col) * KSTR + (ks * 32 + g * 8) * 2);
          s[kt] = mfma16x16x32(kf, qf[ks], s[kt]);
        }
      }
      float cmax = -1e30f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int key = c * KC + kt * 16 + g * 4 + j;
          const float v = key < L ? s[kt][j] * sl2 : -1e30f;
          s[kt][j] = v;
          cmax = fmaxf(cmax, v);
        }
      cmax = fmaxf(cmax, __shfl_xor(cmax, 16, 64));
      cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
      const float m_new = fmaxf(m_run, cmax);
      const float alpha = exp2f(m_run - m_new);
      m_run = m_new;
      l_run *= alpha;
#pragma unroll
      for (int i = 0; i < NDT; ++i) acc[i] *= alpha;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float e = exp2f(s[kt][j] - m_new);
          s[kt][j] = e;
          l_run += e;
        }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 pf;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pf[j] = (bf16)s[2 * kk][j];
          pf[4 + j] = (bf16)s[2 * kk + 1][j];
        }
        const int qq = col >> 2, pp = col & 3;
        const char* r1 = Vs + (kk * 32 + 4 * g + qq) * VSTR + 8 * pp;
        const char* r2 = r1 + 16 * VSTR;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const s16x4 lo = lds_read_tr16(r1 + dt * 32);
          const s16x4 hi = lds_read_tr16(r2 + dt * 32);
          bf16x8 vf;
          const bf16x4 lob = __builtin_bit_cast(bf16x4, lo);
          const bf16x4 hib = __builtin_bit_cast(bf16x4, hi);
#pragma unroll
          for (int j = 0; j < 4; ++j) { vf[j] = lob[j]; vf[4 + j] = hib[j]; }
          acc[dt] = mfma16x16x32(vf, pf, acc[dt]);
        }
      }
    }
  }

#undef PDM_ATT_PREFETCH
#undef PDM_ATT_COMMIT
  if (!active) return;
  l_run += __shfl_xor(l_run, 16, 64);
  l_run += __shfl_xor(l_run, 32, 64);
  const float inv = 1.0f / l_run;
  const int q = qt * 16 + col;
  if (q < L) {
    bf16* orow = p.out + ((size_t)b * L + q) * p.ldo + h * DH;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      const int d = dt * 16 + g * 4;
      if (d < DH) {
        const f32x4 v = acc[dt] * inv;
        *reinterpret_cast<bf16x4*>(orow + d) = to_bf16x4(v[0], v[1], v[2], v[3]);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Head-resident variant for Dh = 64 and L <= 640 (every U-ViT-L/M/S, CIFAR and t2i shape): one workgroup
// per (b, h) stages the head's whole K and V (L x 128 B each, XOR-swizzled rows, no padding) into LDS with
// LDS-DMA once, then every wave runs T query tiles of 16 over all keys with no further barrier.  K/V are
// read from HBM once per head (not once per 64-query block), the 16-query tiles tile L with one ragged
// tile, and each K / V^T fragment read from LDS feeds T MFMAs.
//   K rows: 16-B chunk c stored at c ^ ((row >> 1) & 7)   (conflict-free ds_read_b128 fragment reads)
//   V rows: 32-B unit u stored at u ^ ((row >> 1) & 3)    (conflict-free ds_read_b64_tr_b16 reads)
// The softmax scale is folded into one FMA before exp2; key masking only runs in the last 64-key block.
template <int T>
__global__ __launch_bounds__(T == 2 ? 768 : 512) void attention_kv_kernel(AttentionArgs p, int nqt, int Lp) {
  constexpr int DH = 64;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* Ks = lds;
  char* Vs = lds + Lp * 128;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const int bh = blockIdx.x;
  const int b = bh / p.H, h = bh % p.H;
  const int L = p.L, D = p.H * DH;
  const bf16* base = p.qkv + (size_t)b * L * p.ldq + h * DH;

  // stage K and V: one wave-instruction = 8 rows x 128 B, lane -> (row = lane >> 3, physical chunk lane & 7)
  {
    const int r8 = lane >> 3, pc = lane & 7;
    for (int grp = wave; grp < Lp / 8; grp += nw) {
      const int row = grp * 8 + r8;
      const int key = row < L ? row : L - 1;
      const bf16* src = base + (size_t)key * p.ldq;
      const int kc = pc ^ ((row >> 1) & 7);
      const int vc = ((((pc >> 1) ^ ((row >> 1) & 3)) << 1) | (pc & 1));
      glds16(src + D + kc * 8, (PDM_LDS void*)(Ks + grp * 1024));
      glds16(src + 2 * D + vc * 8, (PDM_LDS void*)(Vs + grp * 1024));
    }
  }

  const int g = lane >> 4, col = lane & 15;
  // Q^T fragments of this wave's tiles (B operand): lane holds Q[q = tile*16 + col][d = ks*32 + g*8 .. +8]
  bf16x8 qf[T][2];
  bool tv[T];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int tile = wave + t * nw;
    tv[t] = tile < nqt;
    int q = tile * 16 + col;
    q = q < L ? q : L - 1;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) qf[t][ks] = *reinterpret_cast<const bf16x8*>(base + (size_t)q * p.ldq + ks * 32 + g * 8);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (!tv[0]) return;

  const float sl2 = p.scale * 1.4426950408889634f;
  float m_run[T], l_run[T];
  f32x4 acc[T][4];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    m_run[t] = -1e30f;
    l_run[t] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[t][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  const int nch = (L + 63) / 64;
  for (int c = 0; c < nch; ++c) {
    const int kvalid = L - c * 64;           // keys of this block (>= 64 except in the last block)
    f32x4 s[T][4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int t = 0; t < T; ++t) s[t][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (kt * 16 < kvalid) {
        const int row = c * 64 + kt * 16 + col;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + row * 128 + (((ks * 4 + g) ^ ((row >> 1) & 7)) << 4));
#pragma unroll
          for (int t = 0; t < T; ++t)
            if (t == 0 || tv[t]) s[t][kt] = mfma16x16x32(kf, qf[t][ks], s[t][kt]);
        }
      }
    }
    if (kvalid < 64) {   // ragged last block: mask keys >= L
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (kt * 16 + g * 4 + j >= kvalid)
#pragma unroll
            for (int t = 0; t < T; ++t) s[t][kt][j] = -INFINITY;
    }
#pragma unroll
    for (int t = 0; t < T; ++t) {
      float cmax = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
        cmax = fmaxf(cmax, fmaxf(fmaxf(s[t][kt][0], s[t][kt][1]), fmaxf(s[t][kt][2], s[t][kt][3])));
      cmax = fmaxf(cmax, __shfl_xor(cmax, 16, 64));
      cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
      const float m_new = fmaxf(m_run[t], cmax * sl2);
      const float alpha = exp2f(m_run[t] - m_new);
      m_run[t] = m_new;
      float ls = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float e = exp2f(fmaf(s[t][kt][j], sl2, -m_new));
          s[t][kt][j] = e;
          ls += e;
        }
      l_run[t] = l_run[t] * alpha + ls;
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[t][i] *= alpha;
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      if (kk * 32 >= kvalid) break;
      bf16x8 pf[T];
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pf[t][j] = (bf16)s[t][2 * kk][j];
          pf[t][4 + j] = (bf16)s[t][2 * kk + 1][j];
        }
      const int qq = col >> 2, pp = col & 3;
      const int r1 = c * 64 + kk * 32 + 4 * g + qq, r2 = r1 + 16;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const s16x4 lo = lds_read_tr16(Vs + r1 * 128 + ((dt ^ ((r1 >> 1) & 3)) << 5) + 8 * pp);
        const s16x4 hi = lds_read_tr16(Vs + r2 * 128 + ((dt ^ ((r2 >> 1) & 3)) << 5) + 8 * pp);
        const bf16x4 lob = __builtin_bit_cast(bf16x4, lo);
        const bf16x4 hib = __builtin_bit_cast(bf16x4, hi);
        bf16x8 vf;
#pragma unroll
        for (int j = 0; j < 4; ++j) { vf[j] = lob[j]; vf[4 + j] = hib[j]; }
#pragma unroll
        for (int t = 0; t < T; ++t)
          if (t == 0 || tv[t]) acc[t][dt] = mfma16x16x32(vf, pf[t], acc[t][dt]);
      }
    }
  }

#pragma unroll
  for (int t = 0; t < T; ++t) {
    if (!tv[t]) continue;
    float l = l_run[t];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = 1.0f / l;
    const int q = (wave + t * nw) * 16 + col;
    if (q < L) {
      bf16* orow = p.out + ((size_t)b * L + q) * p.ldo + h * DH;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const f32x4 v = acc[t][dt] * inv;
        *reinterpret_cast<bf16x4*>(orow + dt * 16 + g * 4) = to_bf16x4(v[0], v[1], v[2], v[3]);
      }
    }
  }
}
}  // namespace

const char* attention_check(const AttentionArgs& p) {
  if (p.B <= 0 || p.L <= 0 || p.H <= 0) return "attention: B, L, H must be positive";
  if (!(p.Dh == 32 || p.Dh == 64 || p.Dh == 72 || p.Dh == 96 || p.Dh == 128))
    return "attention: head dim must be one of 32, 64, 72, 96, 128";
  if (p.ldq % 8 || p.ldq < 3 * p.H * p.Dh) return "attention: ldq must be a multiple of 8 and >= 3*H*Dh";
  if (p.ldo % 4 || p.ldo < p.H * p.Dh) return "attention: ldo must be a multiple of 4 and >= H*Dh";
  if (((uintptr_t)p.qkv & 15) || ((uintptr_t)p.out & 7)) return "attention: misaligned qkv/out";
  return nullptr;
}

static int g_attention_algo = 0;   // 0 auto, 1 = 64-query blocks with streamed K/V, 2/3 = head-resident T = 2/3
void attention_set_algo(int algo) { g_attention_algo = algo; }

hipError_t attention_launch(const AttentionArgs& p, hipStream_t stream) {
  const int nqt = (p.L + 15) / 16;
  int algo = g_attention_algo;
  const int Lp = (p.L + 31) / 32 * 32;   // PV reads whole 32-key steps
  if (p.Dh != 64 || Lp * 256 > 160 * 1024) algo = 1;
  // automatic choice stays on the streamed structure until the head-resident one has been measured on the
  // device (tools/attn_bench.py); both are covered by tests/test_gpu_kernels.py::test_attention_algos
  if (algo == 0) algo = 1;
  if (algo == 2 || algo == 3) {
    const int T = algo;
    const int nw = (nqt + T - 1) / T;
    if (nw <= (T == 2 ? 12 : 8)) {
      const int smem = Lp * 256;
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute((const void*)attention_kv_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)attention_kv_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
      }
      if (T == 2) hipLaunchKernelGGL(attention_kv_kernel<2>, dim3(p.B * p.H), dim3(nw * 64), smem, stream, p, nqt, Lp);
      else hipLaunchKernelGGL(attention_kv_kernel<3>, dim3(p.B * p.H), dim3(nw * 64), smem, stream, p, nqt, Lp);
      return hipGetLastError();
    }
  }
  const int nqb = (nqt + 3) / 4;
  const int nbh = p.B * p.H;
  dim3 grid(((nbh + 7) / 8) * 8 * nqb), block(256);
  switch (p.Dh) {
    case 32: hipLaunchKernelGGL(attention_kernel<32>, grid, block, 0, stream, p, nqt); break;
    case 64: hipLaunchKernelGGL(attention_kernel<64>, grid, block, 0, stream, p, nqt); break;
    case 72: hipLaunchKernelGGL(attention_kernel<72>, grid, block, 0, stream, p, nqt); break;
    case 96: hipLaunchKernelGGL(attention_kernel<96>, grid, block, 0, stream, p, nqt); break;
    default: hipLaunchKernelGGL(attention_kernel<128>, grid, block, 0, stream, p, nqt); break;
  }
  return hipGetLastError();
}

}  // namespace pdm

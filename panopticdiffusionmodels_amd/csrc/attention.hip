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
#include <type_traits>

#include "pdm_common.h"
#include "pdm_kernels.h"

namespace pdm {

namespace {

__device__ __forceinline__ s16x4 lds_read_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((PDM_LDS s16x4*)(p));
}

// K / V staging of the head-resident kernels: 16-byte LDS-DMA through a buffer descriptor (the rows of one batch
// entry), not the global-address form -- after a global_load_lds hipcc drains vmcnt to 0 before the next LDS read
// (it cannot tell the DMA's destination from the block being read), which serialised every head's first pass behind
// its whole K/V transfer; the buffer form leaves the ordering to the kernels' own counted waits
__device__ __forceinline__ __amdgpu_buffer_rsrc_t att_rsrc(const void* base, long long bytes) {
  const unsigned n = bytes >= 0x7fffffffLL ? 0x7fffffffu : (unsigned)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)n, 0x00020000);
}
__device__ __forceinline__ void att_dma16(__amdgpu_buffer_rsrc_t r, unsigned voff, PDM_LDS void* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, lds, 16, (int)voff, 0, 0, 0);
}

// V^T fragment reads of one 32-key step as ONE asm statement with its lgkmcnt wait: hipcc treats the transposed-read
// builtin as aliasing any pending LDS-DMA and waits vmcnt(0) in front of it (draining the K/V transfer still in
// flight); the data read here were retired by the kernels' counted vmcnt waits + barriers.
__device__ __forceinline__ unsigned att_lds_addr(const void* p) { return (unsigned)(uintptr_t)(PDM_LDS const void*)p; }
__device__ __forceinline__ bf16x8 att_pair(s16x4 lo, s16x4 hi) {
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
// Dh 64: four fragments, fragment dt = rows at a[dt] and a[dt] + 2048
__device__ __forceinline__ void lds_vt4(const char* a0, const char* a1, const char* a2, const char* a3, bf16x8 (&vf)[4]) {
  s16x4 l0, h0, l1, h1, l2, h2, l3, h3;
  asm volatile(
      "ds_read_b64_tr_b16 %0, %8\n\tds_read_b64_tr_b16 %1, %8 offset:2048\n\t"
      "ds_read_b64_tr_b16 %2, %9\n\tds_read_b64_tr_b16 %3, %9 offset:2048\n\t"
      "ds_read_b64_tr_b16 %4, %10\n\tds_read_b64_tr_b16 %5, %10 offset:2048\n\t"
      "ds_read_b64_tr_b16 %6, %11\n\tds_read_b64_tr_b16 %7, %11 offset:2048\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(l0), "=&v"(h0), "=&v"(l1), "=&v"(h1), "=&v"(l2), "=&v"(h2), "=&v"(l3), "=&v"(h3)
      : "v"(att_lds_addr(a0)), "v"(att_lds_addr(a1)), "v"(att_lds_addr(a2)), "v"(att_lds_addr(a3))
      : "memory");
  vf[0] = att_pair(l0, h0);
  vf[1] = att_pair(l1, h1);
  vf[2] = att_pair(l2, h2);
  vf[3] = att_pair(l3, h3);
}
// Dh 72 (144-B rows): five fragments, fragment dt = rows at a + 32 dt and a + 2304 + 32 dt
__device__ __forceinline__ void lds_vt5(const char* a, bf16x8 (&vf)[5]) {
  s16x4 l[5], h[5];
  asm volatile(
      "ds_read_b64_tr_b16 %0, %10\n\tds_read_b64_tr_b16 %1, %10 offset:2304\n\t"
      "ds_read_b64_tr_b16 %2, %10 offset:32\n\tds_read_b64_tr_b16 %3, %10 offset:2336\n\t"
      "ds_read_b64_tr_b16 %4, %10 offset:64\n\tds_read_b64_tr_b16 %5, %10 offset:2368\n\t"
      "ds_read_b64_tr_b16 %6, %10 offset:96\n\tds_read_b64_tr_b16 %7, %10 offset:2400\n\t"
      "ds_read_b64_tr_b16 %8, %10 offset:128\n\tds_read_b64_tr_b16 %9, %10 offset:2432\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(l[0]), "=&v"(h[0]), "=&v"(l[1]), "=&v"(h[1]), "=&v"(l[2]), "=&v"(h[2]), "=&v"(l[3]), "=&v"(h[3]),
        "=&v"(l[4]), "=&v"(h[4])
      : "v"(att_lds_addr(a))
      : "memory");
#pragma unroll
  for (int dt = 0; dt < 5; ++dt) vf[dt] = att_pair(l[dt], h[dt]);
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

// ------------------------------------------------------------------------------------------------
// Head-resident v2 (Dh = 64): a 4-wave workgroup per (b, h), two workgroups per CU (LDS-bound), so one
// head's K/V DMA overlaps the other head's math.  K and V (L x 128 B each, layouts as above) are staged by
// LDS-DMA in 64-key blocks; the first pass waits per block (counted vmcnt + one barrier), so its math starts
// as soon as block 0 has landed.  Q fragments of a wave's first pass are loaded by inline-asm global loads
// issued ahead of the DMA and waited for explicitly (a compiler-visible load would drain the DMA queue).
// Wave w owns query tiles w, w + 4, w + 8, ... and runs them two at a time, so each K and V^T fragment read
// feeds two MFMAs.  DEBUG 1: loads only; DEBUG 2: math only (timing experiments, wrong results).
__device__ __forceinline__ void wait_vmcnt_dyn(int n) {
  switch (n) {
#define PDM_W(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    PDM_W(0) PDM_W(1) PDM_W(2) PDM_W(3) PDM_W(4) PDM_W(5) PDM_W(6) PDM_W(7) PDM_W(8) PDM_W(9) PDM_W(10)
    PDM_W(11) PDM_W(12) PDM_W(13) PDM_W(14) PDM_W(15) PDM_W(16) PDM_W(17) PDM_W(18) PDM_W(19) PDM_W(20)
    PDM_W(21) PDM_W(22) PDM_W(23) PDM_W(24) PDM_W(25) PDM_W(26) PDM_W(27) PDM_W(28) PDM_W(29) PDM_W(30)
#undef PDM_W
    default: asm volatile("s_waitcnt vmcnt(31)" ::: "memory"); break;
  }
}

// The explicit wait for the inline-asm Q loads, with the Q registers pinned by the wait itself: one asm statement
// holding a compare chain over n = 0 .. 30 (each arm one `s_waitcnt vmcnt(n)`, the fall-through vmcnt(31)), "+v" on
// every Q register.  hipcc sees the loads' destinations as live, unmoved values up to this statement and cannot place
// a copy of them between a case's wait and its use, and every path through the chain passes exactly one wait -- so
// tools/check_asm_loads.py, which walks every path of the shipped code object from each load to its first vmcnt
// wait, proves that nothing touches a Q register while the load may be in flight (run by
// tests/test_cpu_lib.py).  A C++ switch over separate asm waits lowered to a compare chain with merged case flags,
// whose skip-every-case paths a path-insensitive walk cannot rule out.
#define PDM_WQ_CASE(k) "s_cmp_eq_u32 %[n], " #k "\n\ts_cbranch_scc0 .Lpdm_wq_" #k "_%=\n\ts_waitcnt vmcnt(" #k ")\n\t" \
                       "s_branch .Lpdm_wq_end_%=\n.Lpdm_wq_" #k "_%=:\n\t"
#define PDM_WAIT_Q(NV, ...)                                                                                               \
  asm volatile(PDM_WQ_CASE(0) PDM_WQ_CASE(1) PDM_WQ_CASE(2) PDM_WQ_CASE(3) PDM_WQ_CASE(4) PDM_WQ_CASE(5)             \
               PDM_WQ_CASE(6) PDM_WQ_CASE(7) PDM_WQ_CASE(8) PDM_WQ_CASE(9) PDM_WQ_CASE(10) PDM_WQ_CASE(11)           \
               PDM_WQ_CASE(12) PDM_WQ_CASE(13) PDM_WQ_CASE(14) PDM_WQ_CASE(15) PDM_WQ_CASE(16) PDM_WQ_CASE(17)       \
               PDM_WQ_CASE(18) PDM_WQ_CASE(19) PDM_WQ_CASE(20) PDM_WQ_CASE(21) PDM_WQ_CASE(22) PDM_WQ_CASE(23)       \
               PDM_WQ_CASE(24) PDM_WQ_CASE(25) PDM_WQ_CASE(26) PDM_WQ_CASE(27) PDM_WQ_CASE(28) PDM_WQ_CASE(29)       \
               PDM_WQ_CASE(30) "s_waitcnt vmcnt(31)\n.Lpdm_wq_end_%=:"                                               \
               : __VA_ARGS__ : [n] "s"(NV) : "memory", "scc")

__device__ __forceinline__ i32x4 gload16_asm(const void* ptr) {
  i32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(ptr) : "memory");
  return v;
}

// q * (scale * log2 e) for kernels whose producer did not pre-scale q (AttentionArgs::q_log2 == 0)
__device__ __forceinline__ bf16x8 scale_bf16x8(bf16x8 v, float sc) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)v[j] * sc);
  return v;
}
// cross-lane max / sum over the four 16-lane rows holding one query's keys (lanes col, col+16, col+32,
// col+48): v_permlane16/32_swap half exchanges, no LDS round trip (ds_bpermute)
__device__ __forceinline__ float xrow_max(float v) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float xrow_sum(float v) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// NW = waves per workgroup: 4 when two heads fit per CU (L <= 320), else 8 so the single resident head still
// has two waves per SIMD (t2i image / mask streams, L = 334 / 590)
// ONES: the softmax row sums come from a fifth PV tile whose V^T operand is a constant ones row (one extra MFMA per
// 32 keys and tile) instead of VALU adds over the scores
template <int DEBUG, int NW, bool ONES = false>
__global__ __launch_bounds__(NW * 64, NW == 4 ? 2 : 1) void attention_v2_kernel(AttentionArgs p, int nqt, int Lp) {
  constexpr int DH = 64;
  constexpr float RESCALE_THR = 8.0f;   // deferred rescale (log2 units): P <= 2^8 in bf16, O / l stay fp32
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* Ks = lds;
  char* Vs = lds + Lp * 128;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar waits and branches
  const int bh = blockIdx.x;
  const int b = bh / p.H, h = bh % p.H;
  const int L = p.L, D = p.H * DH;
  const bf16* base = p.qkv + (size_t)b * L * p.ldq + h * DH;
  const int g = lane >> 4, col = lane & 15;

  // tiles of this wave: w, w+NW, ...; passes of two tiles (the last pass may hold one)
  const int my_tiles = nqt > wave ? (nqt - wave + NW - 1) / NW : 0;
  // passes of two tiles; an odd count folds its last tile into the final pass (three tiles) instead of a
  // one-tile pass of its own (L = 258: the ragged 17th tile of wave 0)
  const int npass = my_tiles == 1 ? 1 : my_tiles / 2;

  auto qptr = [&](int tile, int ks) {
    int q = tile * 16 + col;
    q = q < L ? q : L - 1;
    return base + (size_t)q * p.ldq + ks * 32 + g * 8;
  };
  // Q fragments of the first pass (B operand): lane holds Q[q = tile*16 + col][d = ks*32 + g*8 .. +8], loaded
  // by inline asm ahead of the K/V DMA (a compiler-visible load would make hipcc drain the DMA queue)
  i32x4 q0[3][2];
  if (npass > 0 && DEBUG != 2) {
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int tile = min(wave + NW * t, nqt - 1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) q0[t][ks] = gload16_asm(qptr(tile, ks));
    }
  }
  // K / V DMA in 64-key blocks: block c = row groups 8c .. 8c+7 (8 rows x 128 B each); wave w stages groups
  // 8c + w (+ 4 with 4 waves) of K and of V (the last block may have fewer)
  const int ngrp = Lp / 8;
  if (DEBUG != 2) {
    const int r8 = lane >> 3, pc = lane & 7;
    const __amdgpu_buffer_rsrc_t rq = att_rsrc(p.qkv + (size_t)b * L * p.ldq, (long long)L * p.ldq * 2);
    for (int grp0 = 0; grp0 < ngrp; grp0 += 8) {
#pragma unroll
      for (int i = 0; i < 8 / NW; ++i) {
        const int grp = grp0 + wave + NW * i;
        if (grp < ngrp) {
          const int row = grp * 8 + r8;
          const int key = row < L ? row : L - 1;
          const unsigned rowoff = (unsigned)(key * p.ldq + h * DH);
          const int kc = pc ^ ((row >> 1) & 7);
          const int vc = ((((pc >> 1) ^ ((row >> 1) & 3)) << 1) | (pc & 1));
          att_dma16(rq, (rowoff + D + kc * 8) * 2u, (PDM_LDS void*)(Ks + grp * 1024));
          att_dma16(rq, (rowoff + 2 * D + vc * 8) * 2u, (PDM_LDS void*)(Vs + grp * 1024));
        }
      }
    }
  }
  // LDS-DMA ops this wave issued for blocks > c (the vmcnt that retires Q and blocks 0..c)
  auto ops_after = [&](int c) {
    int n = 0;
    for (int grp0 = (c + 1) * 8; grp0 < ngrp; grp0 += 8)
      for (int i = 0; i < 8 / NW; ++i) n += (grp0 + wave + NW * i < ngrp) ? 2 : 0;
    return n;
  };
  auto block_ready = [&](int c) {   // pass 0: block c of K/V landed (all waves) before anyone reads it
    if (DEBUG == 0) wait_vmcnt_dyn(ops_after(c));
    else if (DEBUG == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  const float sl2 = p.scale * 1.4426950408889634f;
  const int nfull = L / 64, nch = (L + 63) / 64;

  // one pass over all keys for NT query tiles (qf), writing the normalised rows of tiles tl[0..NT)
  auto run_pass = [&](auto ntc, const bf16x8 (&qf)[3][2], const int (&tl)[3], bool first) {
    constexpr int NT = decltype(ntc)::value;
    constexpr int NA = ONES ? 5 : 4;
    float m_run[NT], l_run[NT];
    f32x4 acc[NT][NA];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      m_run[t] = -INFINITY;
      l_run[t] = 0.f;
#pragma unroll
      for (int i = 0; i < NA; ++i) acc[t][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const bf16x8 z8 = bf16x8{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const bf16x8 ones_row = col == 0 ? bf16x8{1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f} : z8;   // V^T row 0 of tile 4
    // LDS addresses: both swizzles are independent of the block c and of kt / kk (row = c*64 + kt*16 + col gives
    // (row >> 1) & 7 = (col >> 1) & 7; V row r = c*64 + kk*32 + 4g + qq gives (r >> 1) & 3 = (2g + (qq >> 1)) & 3),
    // so every fragment read is a per-lane base + c * 8 KiB + an immediate offset (no address VALU per read)
    const char* kbase[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) kbase[ks] = Ks + col * 128 + (((ks * 4 + g) ^ ((col >> 1) & 7)) << 4);
    const char* vbase[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
      vbase[dt] = Vs + (4 * g + (col >> 2)) * 128 + ((dt ^ ((2 * g + (col >> 3)) & 3)) << 5) + 8 * (col & 3);
    // Scores live in log2 units relative to the running max: Q carries scale * log2(e) (q_log2), and every block
    // after a pass's first starts its Q K^T accumulators at -m_run, so P = exp2(S) needs no per-score FMA.
    auto do_block = [&](int c, auto tailc, auto firstc) {
      constexpr int TAIL = decltype(tailc)::value, FIRST = decltype(firstc)::value;
      const int kvalid = L - c * 64;
      // TAIL 1: a ragged last block of <= 16 keys (L = 258, 334, 590): only its first 16-key sub-block is live,
      // the others are neither computed, maxed, shifted nor exponentiated (P = 0), all decided at compile time (a
      // runtime per-sub-block skip measured slower: the branches split the block's straight-line MFMA / VALU code).
      // TAIL 2: any other ragged block, masked over all four sub-blocks.
      constexpr int nkt = TAIL == 1 ? 1 : 4;
      f32x4 s[NT][4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
        for (int t = 0; t < NT; ++t) s[t][kt] = FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : f32x4(-m_run[t]);
        if (TAIL == 1 ? kt >= 1 : (TAIL && kt * 16 >= kvalid)) continue;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kbase[ks] + c * 8192 + kt * 2048);
#pragma unroll
          for (int t = 0; t < NT; ++t) s[t][kt] = mfma16x16x32(kf, qf[t][ks], s[t][kt]);
        }
      }
      if constexpr (TAIL) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (kt < nkt && kt * 16 + g * 4 + j >= kvalid)
#pragma unroll
              for (int t = 0; t < NT; ++t) s[t][kt][j] = -INFINITY;
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        f32x4 m4 = s[t][0];
#pragma unroll
        for (int kt = 1; kt < 4; ++kt) {
          if (TAIL && kt >= nkt) break;
#pragma unroll
          for (int j = 0; j < 4; ++j) m4[j] = fmaxf(m4[j], s[t][kt][j]);
        }
        const float cmax = xrow_max(fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3])));
        if constexpr (FIRST) {   // the running max starts at the first block's
          m_run[t] = cmax;
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
            if (!TAIL || kt < nkt) s[t][kt] -= cmax;
        } else if (__builtin_amdgcn_ballot_w64(cmax > RESCALE_THR)) {
          // deferred rescale: the running max moves only when a block exceeds it by RESCALE_THR (rare)
          const float d = cmax > RESCALE_THR ? cmax : 0.f;
          const float alpha = __builtin_amdgcn_exp2f(-d);
          m_run[t] += d;
          l_run[t] *= alpha;
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
            if (!TAIL || kt < nkt) s[t][kt] -= d;
#pragma unroll
          for (int i = 0; i < NA; ++i) acc[t][i] *= alpha;
        }
        f32x4 l4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
          if (TAIL && kt >= nkt) {
            s[t][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
            continue;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) s[t][kt][j] = __builtin_amdgcn_exp2f(s[t][kt][j]);
          if constexpr (!ONES) l4 += s[t][kt];
        }
        if constexpr (!ONES) l_run[t] += (l4[0] + l4[1]) + (l4[2] + l4[3]);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        if (TAIL == 1 ? kk >= 1 : (TAIL && kk * 32 >= kvalid)) break;
        bf16x8 pf[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            pf[t][j] = (bf16)s[t][2 * kk][j];
            pf[t][4 + j] = (bf16)s[t][2 * kk + 1][j];
          }
        bf16x8 vf[4];
        lds_vt4(vbase[0] + c * 8192 + kk * 4096, vbase[1] + c * 8192 + kk * 4096, vbase[2] + c * 8192 + kk * 4096,
                vbase[3] + c * 8192 + kk * 4096, vf);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[t][dt] = mfma16x16x32(vf[dt], pf[t], acc[t][dt]);
        if constexpr (ONES) {
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[t][4] = mfma16x16x32(ones_row, pf[t], acc[t][4]);
        }
      }
    };
    if (first) block_ready(0);
    if (DEBUG != 1) {
      if (nfull > 0) do_block(0, std::false_type{}, std::true_type{});
      else do_block(0, std::integral_constant<int, 2>{}, std::true_type{});
    }
    for (int c = 1; c < nfull; ++c) {
      if (first) block_ready(c);
      if (DEBUG != 1) do_block(c, std::false_type{}, std::false_type{});
    }
    if (nfull < nch && nfull > 0) {
      if (first) block_ready(nfull);
      if (DEBUG != 1) {
        do_block(nfull, std::integral_constant<int, 2>{}, std::false_type{});
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float lsum = l_run[t];
      if constexpr (ONES) lsum = g == 0 ? acc[t][NA - 1][0] : 0.f;   // V^T row 0 of tile 4: lanes of k-group 0
      const float inv = 1.0f / xrow_sum(lsum);
      const int q = tl[t] * 16 + col;
      if (q < L) {
        bf16* orow = p.out + ((size_t)b * L + q) * p.ldo + h * DH;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const f32x4 v = acc[t][dt] * inv;
          *reinterpret_cast<bf16x4*>(orow + dt * 16 + g * 4) = to_bf16x4(v[0], v[1], v[2], v[3]);
        }
      }
    }
  };

  if (npass == 0) {   // no tiles: still join pass 0's per-block barriers
    for (int c = 0; c < nch; ++c) block_ready(c);
    return;
  }
  bf16x8 qf[3][2];
  if (DEBUG != 2) {
    asm volatile("" : "+v"(q0[0][0]), "+v"(q0[0][1]), "+v"(q0[1][0]), "+v"(q0[1][1]), "+v"(q0[2][0]), "+v"(q0[2][1]));
  }
  for (int pass = 0; pass < npass; ++pass) {
    const int tl[3] = {wave + 2 * NW * pass, wave + 2 * NW * pass + NW, wave + 2 * NW * pass + 2 * NW};
    const int nt = my_tiles == 1 ? 1 : (pass == npass - 1 && (my_tiles & 1) ? 3 : 2);
    if (pass == 0) {
      if (DEBUG == 0) {
        // Q (the oldest loads) retired together with block 0; "+v" keeps every consumer below the wait
        PDM_WAIT_Q(ops_after(0), "+v"(q0[0][0]), "+v"(q0[0][1]), "+v"(q0[1][0]), "+v"(q0[1][1]), "+v"(q0[2][0]), "+v"(q0[2][1]));
      } else if (DEBUG == 1) {
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(q0[0][0]), "+v"(q0[0][1]), "+v"(q0[1][0]), "+v"(q0[1][1]), "+v"(q0[2][0]),
                     "+v"(q0[2][1]));
      }
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) qf[t][ks] = __builtin_bit_cast(bf16x8, q0[t][ks]);
    } else {
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) qf[t][ks] = *reinterpret_cast<const bf16x8*>(qptr(t < nt ? tl[t] : tl[0], ks));
      // consumed here, so hipcc's waits for these loads stay in this branch (its wait tracking merges the branches:
      // otherwise every MFMA / LDS read of the shared pass code waits vmcnt(0))
      asm volatile("" : "+v"(qf[0][0]), "+v"(qf[0][1]), "+v"(qf[1][0]), "+v"(qf[1][1]), "+v"(qf[2][0]), "+v"(qf[2][1]));
    }
    if (!p.q_log2) {   // q not pre-scaled by the producer: scale * log2(e) applied here (one extra bf16 rounding)
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) qf[t][ks] = scale_bf16x8(qf[t][ks], sl2);
    }
    if (nt == 3) run_pass(std::integral_constant<int, 3>{}, qf, tl, pass == 0);
    else if (nt == 2) run_pass(std::integral_constant<int, 2>{}, qf, tl, pass == 0);
    else run_pass(std::integral_constant<int, 1>{}, qf, tl, pass == 0);
  }
}

// ------------------------------------------------------------------------------------------------
// Persistent head-resident attention (Dh = 64, round 5): attention_v2_kernel's math, but each workgroup loops over
// heads bh = blockIdx, blockIdx + grid, ... and streams the NEXT head's K/V into LDS while its last pass over the
// current head runs: after every 64-key block of that pass a barrier releases the block's LDS rows and the waves
// issue the next head's rows for it.  v2 launches one workgroup per head, and every workgroup on the chip stages its
// head at the same moment and then computes with the memory system idle (the phases stay in lockstep across the
// chip); here K/V traffic runs beside the MFMA / exp work of the previous head.  Every wave runs the same number of
// passes (1-3 tiles each, balanced), so the per-block barriers of the first head's first pass and of each releasing
// last pass pair up across waves.  Needs nqt >= NW (every wave owns a tile).  DEBUG 1: loads only; 2: math only.
// TK 1: L % 64 in [1, 16] with L > 64 (the last key block's one live sub-block resolved at compile time, do_block)
template <int DEBUG, int NW, int TK = 2>
__global__ __launch_bounds__(NW * 64, NW == 4 ? 2 : 1) void attention_v3_kernel(AttentionArgs p, int nqt, int Lp) {
  constexpr int DH = 64;
  constexpr int NA = 5;                  // four PV output tiles + the ones-row tile carrying the softmax row sums
  constexpr float RESCALE_THR = 8.0f;    // deferred rescale (log2 units): P <= 2^8 in bf16, O / l stay fp32
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* Ks = lds;
  char* Vs = lds + Lp * 128;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nbh = p.B * p.H, L = p.L, D = p.H * DH;
  const int g = lane >> 4, col = lane & 15;
  const int my_tiles = (nqt - wave + NW - 1) / NW;      // >= 1
  const int npass = ((nqt + NW - 1) / NW + 2) / 3;      // uniform over the waves
  const int ngrp = Lp / 8, nfull = L / 64, nch = (L + 63) / 64;
  const int r8 = lane >> 3, pc = lane & 7;

  // K / V row groups [grp0, grp1) of head (b, h) (8 rows x 128 B per group; wave w takes grp0 + w, + NW, ...)
  auto stage = [&](int b_, int h_, int grp0, int grp1) {
    if (DEBUG == 2) return;
    const __amdgpu_buffer_rsrc_t rq = att_rsrc(p.qkv + (size_t)b_ * L * p.ldq, (long long)L * p.ldq * 2);
    for (int grp = grp0 + wave; grp < grp1; grp += NW) {
      const int row = grp * 8 + r8;
      const int key = row < L ? row : L - 1;
      const unsigned rowoff = (unsigned)(key * p.ldq + h_ * DH);
      const int kc = pc ^ ((row >> 1) & 7);
      const int vc = ((((pc >> 1) ^ ((row >> 1) & 3)) << 1) | (pc & 1));
      att_dma16(rq, (rowoff + D + kc * 8) * 2u, (PDM_LDS void*)(Ks + grp * 1024));
      att_dma16(rq, (rowoff + 2 * D + vc * 8) * 2u, (PDM_LDS void*)(Vs + grp * 1024));
    }
  };
  // this wave's DMA ops of the first head past block c (the vmcnt that retires Q and blocks 0..c)
  auto ops_after = [&](int c) {
    int n = 0;
    for (int grp = 8 * (c + 1) + ((wave - 8 * (c + 1)) % NW + NW) % NW; grp < ngrp; grp += NW) n += 2;
    return n;
  };
  auto bar = []() {
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  int bh = blockIdx.x;
  int b = bh / p.H, h = bh - (bh / p.H) * p.H;
  auto qptr = [&](int b_, int h_, int tile, int ks) {
    int q = tile * 16 + col;
    q = q < L ? q : L - 1;
    return p.qkv + ((size_t)b_ * L + q) * p.ldq + h_ * DH + ks * 32 + g * 8;
  };
  // first head: Q of the first pass by inline asm ahead of the K/V DMA, then the whole head staged
  const int nt0 = my_tiles / npass + (my_tiles % npass ? 1 : 0);
  i32x4 q0[3][2];
  if (DEBUG != 2) {
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) q0[t][ks] = gload16_asm(qptr(b, h, wave + NW * min(t, nt0 - 1), ks));
  }
  stage(b, h, 0, ngrp);

  const bf16x8 z8 = bf16x8{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bf16x8 ones_row = col == 0 ? bf16x8{1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f} : z8;   // V^T row 0 of tile 4
  const char* kbase[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) kbase[ks] = Ks + col * 128 + (((ks * 4 + g) ^ ((col >> 1) & 7)) << 4);
  const char* vbase[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
    vbase[dt] = Vs + (4 * g + (col >> 2)) * 128 + ((dt ^ ((2 * g + (col >> 3)) & 3)) << 5) + 8 * (col & 3);

  // one pass over all keys for NT query tiles; wait_blocks: the first head's first pass waits per block for its
  // DMA; release: after each block, barrier + stage that block of the next head (bn, hn)
  auto run_pass = [&](auto ntc, const bf16x8 (&qf)[3][2], const int (&tl)[3], bool wait_blocks, bool release, int bn,
                      int hn) {
    constexpr int NT = decltype(ntc)::value;
    float m_run[NT];
    f32x4 acc[NT][NA];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      m_run[t] = -INFINITY;
#pragma unroll
      for (int i = 0; i < NA; ++i) acc[t][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    auto do_block = [&](int c, auto tailc, auto firstc) {
      constexpr int TAIL = decltype(tailc)::value, FIRST = decltype(firstc)::value;
      const int kvalid = L - c * 64;
      // TAIL 1: a ragged last block of <= 16 keys (L = 258, 334, 590): only its first 16-key sub-block is live,
      // the others are neither computed, maxed, shifted nor exponentiated (P = 0), all decided at compile time (a
      // runtime per-sub-block skip measured slower: the branches split the block's straight-line MFMA / VALU code).
      // TAIL 2: any other ragged block, masked over all four sub-blocks.
      constexpr int nkt = TAIL == 1 ? 1 : 4;
      f32x4 s[NT][4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
        for (int t = 0; t < NT; ++t) s[t][kt] = FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : f32x4(-m_run[t]);
        if (TAIL == 1 ? kt >= 1 : (TAIL && kt * 16 >= kvalid)) continue;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kbase[ks] + c * 8192 + kt * 2048);
#pragma unroll
          for (int t = 0; t < NT; ++t) s[t][kt] = mfma16x16x32(kf, qf[t][ks], s[t][kt]);
        }
      }
      if constexpr (TAIL) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (kt < nkt && kt * 16 + g * 4 + j >= kvalid)
#pragma unroll
              for (int t = 0; t < NT; ++t) s[t][kt][j] = -INFINITY;
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        f32x4 m4 = s[t][0];
#pragma unroll
        for (int kt = 1; kt < 4; ++kt) {
          if (TAIL && kt >= nkt) break;
#pragma unroll
          for (int j = 0; j < 4; ++j) m4[j] = fmaxf(m4[j], s[t][kt][j]);
        }
        const float cmax = xrow_max(fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3])));
        if constexpr (FIRST) {
          m_run[t] = cmax;
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
            if (!TAIL || kt < nkt) s[t][kt] -= cmax;
        } else if (__builtin_amdgcn_ballot_w64(cmax > RESCALE_THR)) {
          const float d = cmax > RESCALE_THR ? cmax : 0.f;
          const float alpha = __builtin_amdgcn_exp2f(-d);
          m_run[t] += d;
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
            if (!TAIL || kt < nkt) s[t][kt] -= d;
#pragma unroll
          for (int i = 0; i < NA; ++i) acc[t][i] *= alpha;
        }
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
          if (TAIL && kt >= nkt) {
            s[t][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
            continue;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) s[t][kt][j] = __builtin_amdgcn_exp2f(s[t][kt][j]);
        }
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        if (TAIL == 1 ? kk >= 1 : (TAIL && kk * 32 >= kvalid)) break;
        bf16x8 pf[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            pf[t][j] = (bf16)s[t][2 * kk][j];
            pf[t][4 + j] = (bf16)s[t][2 * kk + 1][j];
          }
        bf16x8 vf[4];
        lds_vt4(vbase[0] + c * 8192 + kk * 4096, vbase[1] + c * 8192 + kk * 4096, vbase[2] + c * 8192 + kk * 4096,
                vbase[3] + c * 8192 + kk * 4096, vf);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[t][dt] = mfma16x16x32(vf[dt], pf[t], acc[t][dt]);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t][4] = mfma16x16x32(ones_row, pf[t], acc[t][4]);
      }
    };
    auto block = [&](int c, auto tailc, auto firstc) {
      if (wait_blocks) {
        if (DEBUG == 0) wait_vmcnt_dyn(ops_after(c));
        else if (DEBUG == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();
      }
      if (DEBUG != 1) do_block(c, tailc, firstc);
      if (release) {   // every wave is done with block c: its rows take the next head's
        bar();
        stage(bn, hn, 8 * c, min(8 * c + 8, ngrp));
      }
    };
    if (nfull > 0) block(0, std::false_type{}, std::true_type{});
    else block(0, std::integral_constant<int, 2>{}, std::true_type{});
    for (int c = 1; c < nfull; ++c) block(c, std::false_type{}, std::false_type{});
    if (nfull < nch && nfull > 0) {
      block(nfull, std::integral_constant<int, TK>{}, std::false_type{});
    }
    // (the next head's Q is not prefetched here by inline-asm loads: hipcc does not know such a load is in flight,
    // and across this epilogue it may hand the destination registers to other values, which the late data then
    // overwrites -- the likely cause of a GPU memory fault with that prefetch at 1600 heads, profiles/r05c)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const float lsum = g == 0 ? acc[t][NA - 1][0] : 0.f;   // V^T row 0 of tile 4: lanes of k-group 0
      const float inv = 1.0f / xrow_sum(lsum);
      const int q = tl[t] * 16 + col;
      if (q < L) {
        bf16* orow = p.out + ((size_t)b * L + q) * p.ldo + h * DH;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const f32x4 v = acc[t][dt] * inv;
          *reinterpret_cast<bf16x4*>(orow + dt * 16 + g * 4) = to_bf16x4(v[0], v[1], v[2], v[3]);
        }
      }
    }
  };

  const float sl2 = p.scale * 1.4426950408889634f;
  bool first_head = true;
  for (;;) {
    const int bhn = bh + gridDim.x;
    const bool has_next = bhn < nbh;
    const int bn = has_next ? bhn / p.H : 0, hn = has_next ? bhn - (bhn / p.H) * p.H : 0;
    int start = 0;
    for (int pass = 0; pass < npass; ++pass) {
      const int nt = my_tiles / npass + (pass < my_tiles % npass ? 1 : 0);
      const int tl[3] = {wave + NW * start, wave + NW * (start + (nt > 1 ? 1 : 0)), wave + NW * (start + (nt > 2 ? 2 : 0))};
      start += nt;
      bf16x8 qf[3][2];
      if (first_head && pass == 0) {   // Q from the prologue
        if (DEBUG == 0) {
          PDM_WAIT_Q(ops_after(0), "+v"(q0[0][0]), "+v"(q0[0][1]), "+v"(q0[1][0]), "+v"(q0[1][1]), "+v"(q0[2][0]), "+v"(q0[2][1]));   // Q (the oldest loads) retire with block 0
        } else if (DEBUG == 1) {
          asm volatile("s_waitcnt vmcnt(0)" : "+v"(q0[0][0]), "+v"(q0[0][1]), "+v"(q0[1][0]), "+v"(q0[1][1]),
                       "+v"(q0[2][0]), "+v"(q0[2][1]));
        }
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) qf[t][ks] = __builtin_bit_cast(bf16x8, q0[t][ks]);
      } else {
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            qf[t][ks] = DEBUG == 2 ? bf16x8{} : *reinterpret_cast<const bf16x8*>(qptr(b, h, tl[t], ks));
        // consumed in this branch: hipcc's waits for these loads stay here (see attention_v2_kernel)
        asm volatile("" : "+v"(qf[0][0]), "+v"(qf[0][1]), "+v"(qf[1][0]), "+v"(qf[1][1]), "+v"(qf[2][0]), "+v"(qf[2][1]));
      }
      if (!p.q_log2) {
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) qf[t][ks] = scale_bf16x8(qf[t][ks], sl2);
      }
      const bool wait_blocks = first_head && pass == 0;
      const bool release = has_next && pass == npass - 1;
      if (nt == 3) run_pass(std::integral_constant<int, 3>{}, qf, tl, wait_blocks, release, bn, hn);
      else if (nt == 2) run_pass(std::integral_constant<int, 2>{}, qf, tl, wait_blocks, release, bn, hn);
      else run_pass(std::integral_constant<int, 1>{}, qf, tl, wait_blocks, release, bn, hn);
    }
    if (!has_next) break;
    bh = bhn;
    b = bn;
    h = hn;
    first_head = false;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's share of the next head (and its stores)
    bar();                                             // everyone's
  }
}

// ------------------------------------------------------------------------------------------------
// Head-resident kernel for Dh = 72 (U-ViT-H/2 and H/4: libs/uvit.py:66-92 with embed_dim 1152, 16 heads), the
// v2 structure above with the head dim cut as 64 + 8 instead of padded to 96:
//   Q K^T: three v_mfma_f32_16x16x32_bf16 k-steps, the third over d 64..95 with d 64..71 in k-group 0 and the
//          running max folded into its padding slot d = 72 (K = 1, Q = -m_run): scores leave the MFMA chain as
//          q'k - m in log2 units (q carries Dh^-0.5 log2 e), ready for exp2;
//   P V:   five 16-column output tiles (d 64..79 for the last; rows 73..79 of it are never stored and row 72, with
//          V^T row 72 := ones, accumulates the softmax row sum).
// K and V rows stay unpadded (144 B) so a head's K + V fit twice per CU at L = 258:
//   LDS = [V rows 0 .. round8(L)) [K rows 0 .. round16(L)), 144 B each; staged by LDS-DMA as a flat array of
//   16-B chunks (chunk ci -> row ci / 9, column chunk ci % 9).  PV reads whole 32-key steps, so V rows past
//   round8(L) read the (finite) K rows behind them and are multiplied by P = 0; K rows past round8(L) are never
//   staged and their scores are masked.  The 144-B stride leaves 2-way bank conflicts on the fragment reads
//   (no 16-B chunk permutation of a 9-chunk row removes them; the MFMAs, not LDS, bound the loop).
// Measured against round 5's variants of this kernel (profiles/r05e/attn_h72_variants.log, same box): staging K / V
// by buffer LDS-DMA with per-block counted waits, K split into swizzled 128-B rows + a 16-B tail array and V^T read
// by one asm statement took 122-126 us at 100 rows (this kernel 104) and 74-76 us at 50 rows (60): the conflict-free
// K reads saved 2 % of the math, the 64 scattered 16-B tail reads per block cost more in the loads, so the global
// DMA form and the 144-B rows stay here (attention_h72p_kernel, algo 14, is the persistent variant of the new layout).
template <int DEBUG, int TK = 2>   // TK: as attention_v3_kernel
__global__ __launch_bounds__(256, 2) void attention_h72_kernel(AttentionArgs p, int nqt, int LV, int L16) {
  constexpr int DH = 72, ROWB = 144, NCH = 9;
  constexpr float RESCALE_THR = 8.0f;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* Vs = lds;
  char* Ks = lds + LV * ROWB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bh = blockIdx.x;
  const int b = bh / p.H, h = bh % p.H;
  const int L = p.L, D = p.H * DH;
  const bf16* base = p.qkv + (size_t)b * L * p.ldq + h * DH;
  const int g = lane >> 4, col = lane & 15;
  const bool glo = g < 2;   // output rows d 64..71 of the fifth PV tile (rows 72..79 are padding)

  const int my_tiles = nqt > wave ? (nqt - wave + 3) / 4 : 0;
  const int npass = (my_tiles + 1) / 2;

  auto qrow = [&](int tile) {
    int q = tile * 16 + col;
    q = q < L ? q : L - 1;
    return base + (size_t)q * p.ldq;
  };
  // Q fragments of the first pass: d = ks*32 + g*8 .. +7 (x32 steps) and d = 64 + 4g .. +3 (x16 step, g < 2)
  i32x4 q0[2][2];
  i32x4 q0r[2];   // Q[q][64 .. 71] (used by the lanes of k-group 0)
  if (npass > 0 && DEBUG != 2) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const bf16* qr = qrow(min(wave + 4 * t, nqt - 1));
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) q0[t][ks] = gload16_asm(qr + ks * 32 + g * 8);
      q0r[t] = gload16_asm(qr + 64);
    }
  }
  // K / V DMA: 64 chunks (1 KiB) per instruction, instruction i of each tensor issued by wave i % 4, V before K
  const int ndma = (LV * NCH + 63) / 64;
  if (DEBUG != 2) {
    for (int i = wave; i < ndma; i += 4) {
      const int ci = i * 64 + lane;
      if (ci < LV * NCH) {
        const int row = ci / NCH, ch = ci - row * NCH;
        const bf16* src = base + (size_t)(row < L ? row : L - 1) * p.ldq + ch * 8;
        glds16(src + 2 * D, (PDM_LDS void*)(Vs + i * 1024));
        glds16(src + D, (PDM_LDS void*)(Ks + i * 1024));
      }
    }
  }
  // DMA instructions (both tensors) this wave issued past block c: rows < 64 (c + 1) are chunks < 576 (c + 1)
  auto ops_after = [&](int c) {
    const int need = min(ndma, 9 * (c + 1));
    int n = 0;
    for (int i = wave; i < ndma; i += 4) n += i >= need ? 2 : 0;
    return n;
  };
  auto block_ready = [&](int c) {
    if (DEBUG == 0) wait_vmcnt_dyn(ops_after(c));
    else if (DEBUG == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  const float sl2 = p.scale * 1.4426950408889634f;
  const int nfull = L / 64, nch = (L + 63) / 64;
  const bf16x8 ones8 = bf16x8{1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
  const bf16x8 one8 = bf16x8{1.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bf16x8 zero8 = bf16x8{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

  auto run_pass = [&](auto ntc, const bf16x8 (&qf)[2][2], const bf16x8 (&qr)[2], const int (&tl)[2], bool first) {
    constexpr int NT = decltype(ntc)::value;
    float m_run[NT];
    f32x4 acc[NT][5];
    bf16x8 qm[NT];   // Q of the d 64..95 step: d 64..71 (k-group 0) and the slot d = 72 (k-group 1) = -m_run
    auto set_qm = [&](int t) {
      bf16x8 v = qr[t];
      if (g == 1) v[0] = (bf16)(-m_run[t]);
      qm[t] = v;
    };
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      qm[t] = qr[t];   // first block: slot 0 (no shift yet)
      m_run[t] = -INFINITY;
#pragma unroll
      for (int i = 0; i < 5; ++i) acc[t][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const char* kbase = Ks + col * ROWB;   // per-lane bases; block / kt / kk / dt offsets are immediates
    const char* vbase = Vs + (4 * g + (col >> 2)) * ROWB + 8 * (col & 3);
    // log2-domain scores relative to the running max, as attention_v2_kernel
    auto do_block = [&](int c, auto tailc, auto firstc) {
      constexpr int TAIL = decltype(tailc)::value, FIRST = decltype(firstc)::value;
      const int kvalid = L - c * 64;
      // TAIL 1: a ragged last block of <= 16 keys (L = 258, 334, 590): only its first 16-key sub-block is live,
      // the others are neither computed, maxed, shifted nor exponentiated (P = 0), all decided at compile time (a
      // runtime per-sub-block skip measured slower: the branches split the block's straight-line MFMA / VALU code).
      // TAIL 2: any other ragged block, masked over all four sub-blocks.
      constexpr int nkt = TAIL == 1 ? 1 : 4;
      f32x4 s[NT][4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        if (TAIL == 1 ? kt >= 1 : (TAIL && kt * 16 >= kvalid)) continue;
        const char* krow = kbase + c * (64 * ROWB) + kt * (16 * ROWB);
        // a third 16x16x32 step over d 64..95 carries d 64..71 (k-group 0) and, in the padding slot d = 72
        // (k-group 1), K = 1 against Q = -m_run, so the chain leaves q'k - m_run with no VALU pass over the scores
        // (one uniform MFMA chain: a 16x16x16 step chained with 16x16x32 ones got too few SrcC wait states
        // from hipcc on gfx950, measured wrong scores in both orders)
        bf16x8 kx = *reinterpret_cast<const bf16x8*>(krow + 128);
        kx = g == 0 ? kx : (g == 1 ? one8 : zero8);
#pragma unroll
        for (int t = 0; t < NT; ++t) s[t][kt] = mfma16x16x32(kx, qm[t], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(krow + (ks * 4 + g) * 16);
#pragma unroll
          for (int t = 0; t < NT; ++t) s[t][kt] = mfma16x16x32(kf, qf[t][ks], s[t][kt]);
        }
      }
      if constexpr (TAIL) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (kt < nkt && kt * 16 + g * 4 + j >= kvalid)
#pragma unroll
              for (int t = 0; t < NT; ++t) s[t][kt][j] = -INFINITY;
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        f32x4 m4 = s[t][0];
#pragma unroll
        for (int kt = 1; kt < 4; ++kt) {
          if (TAIL && kt >= nkt) break;
#pragma unroll
          for (int j = 0; j < 4; ++j) m4[j] = fmaxf(m4[j], s[t][kt][j]);
        }
        const float cmax = xrow_max(fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3])));
        // m_run stays bf16-representable (it enters the MFMA as a bf16 operand); the shift is exact in fp32
        if constexpr (FIRST) {
          m_run[t] = (float)(bf16)cmax;
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
            if (!TAIL || kt < nkt) s[t][kt] -= m_run[t];
          set_qm(t);
        } else if (__builtin_amdgcn_ballot_w64(cmax > RESCALE_THR)) {
          const float d = cmax > RESCALE_THR ? (float)(bf16)(m_run[t] + cmax) - m_run[t] : 0.f;
          const float alpha = __builtin_amdgcn_exp2f(-d);
          m_run[t] += d;
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
            if (!TAIL || kt < nkt) s[t][kt] -= d;
#pragma unroll
          for (int i = 0; i < 5; ++i) acc[t][i] *= alpha;
          set_qm(t);
        }
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
          if (TAIL && kt >= nkt) {
            s[t][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
            continue;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) s[t][kt][j] = __builtin_amdgcn_exp2f(s[t][kt][j]);
        }
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        if (TAIL == 1 ? kk >= 1 : (TAIL && kk * 32 >= kvalid)) break;
        bf16x8 pf[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            pf[t][j] = (bf16)s[t][2 * kk][j];
            pf[t][4 + j] = (bf16)s[t][2 * kk + 1][j];
          }
        const char* v1 = vbase + c * (64 * ROWB) + kk * (32 * ROWB);
        const char* v2 = v1 + 16 * ROWB;
#pragma unroll
        for (int dt = 0; dt < 5; ++dt) {
          const s16x4 lo = lds_read_tr16(v1 + dt * 32);
          const s16x4 hi = lds_read_tr16(v2 + dt * 32);
          bf16x8 vf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          // output row d = 72 (padding, never stored) becomes the softmax row sum: V^T row 72 := ones
          if (dt == 4) vf = (lane & 15) == 8 ? ones8 : vf;
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[t][dt] = mfma16x16x32(vf, pf[t], acc[t][dt]);
        }
      }
    };
    if (first) block_ready(0);
    if (DEBUG != 1) {
      if (nfull > 0) do_block(0, std::false_type{}, std::true_type{});
      else do_block(0, std::integral_constant<int, 2>{}, std::true_type{});
    }
    for (int c = 1; c < nfull; ++c) {
      if (first) block_ready(c);
      if (DEBUG != 1) do_block(c, std::false_type{}, std::false_type{});
    }
    if (nfull < nch && nfull > 0) {
      if (first) block_ready(nfull);
      if (DEBUG != 1) {
        do_block(nfull, std::integral_constant<int, TK>{}, std::false_type{});
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const float inv = 1.0f / xrow_sum(g == 2 ? acc[t][4][0] : 0.f);   // row d = 72: lanes of k-group 2, j = 0
      const int q = tl[t] * 16 + col;
      if (q < L) {
        bf16* orow = p.out + ((size_t)b * L + q) * p.ldo + h * DH;
#pragma unroll
        for (int dt = 0; dt < 5; ++dt) {
          if (dt == 4 && !glo) break;   // d 72..79 of the last tile are padding
          const f32x4 v = acc[t][dt] * inv;
          *reinterpret_cast<bf16x4*>(orow + dt * 16 + g * 4) = to_bf16x4(v[0], v[1], v[2], v[3]);
        }
      }
    }
  };

  if (npass == 0) {
    for (int c = 0; c < nch; ++c) block_ready(c);
    return;
  }
  bf16x8 qf[2][2];
  bf16x8 qr[2];
  if (DEBUG != 2) {
    asm volatile("" : "+v"(q0[0][0]), "+v"(q0[0][1]), "+v"(q0[1][0]), "+v"(q0[1][1]), "+v"(q0r[0]), "+v"(q0r[1]));
  }
  for (int pass = 0; pass < npass; ++pass) {
    const int tl[2] = {wave + 8 * pass, wave + 8 * pass + 4};
    const bool two = tl[1] < nqt;
    if (pass == 0) {
      if (DEBUG == 0) {
        PDM_WAIT_Q(ops_after(0), "+v"(q0[0][0]), "+v"(q0[0][1]), "+v"(q0[1][0]), "+v"(q0[1][1]), "+v"(q0r[0]), "+v"(q0r[1]));
      } else if (DEBUG == 1) {
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(q0[0][0]), "+v"(q0[0][1]), "+v"(q0[1][0]), "+v"(q0[1][1]), "+v"(q0r[0]),
                     "+v"(q0r[1]));
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) qf[t][ks] = __builtin_bit_cast(bf16x8, q0[t][ks]);
        qr[t] = g == 0 ? __builtin_bit_cast(bf16x8, q0r[t]) : zero8;
      }
    } else {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const bf16* r = qrow(t == 0 || two ? tl[t] : tl[0]);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) qf[t][ks] = *reinterpret_cast<const bf16x8*>(r + ks * 32 + g * 8);
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(r + 64);
        qr[t] = g == 0 ? v : zero8;
      }
      // consumed in this branch (see attention_v2_kernel)
      asm volatile("" : "+v"(qf[0][0]), "+v"(qf[0][1]), "+v"(qf[1][0]), "+v"(qf[1][1]), "+v"(qr[0]), "+v"(qr[1]));
    }
    if (!p.q_log2) {   // q not pre-scaled by the producer: scale * log2(e) applied here (one extra bf16 rounding)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) qf[t][ks] = scale_bf16x8(qf[t][ks], sl2);
        qr[t] = scale_bf16x8(qr[t], sl2);
      }
    }
    if (two) run_pass(std::integral_constant<int, 2>{}, qf, qr, tl, pass == 0);
    else run_pass(std::integral_constant<int, 1>{}, qf, qr, tl, pass == 0);
  }
}

// ------------------------------------------------------------------------------------------------
// Persistent Dh = 72 kernel (round 5): attention_h72_kernel's math and LDS layout, with attention_v3_kernel's head
// loop -- the next head's K / V block c is staged right after the last pass releases block c -- and balanced, uniform
// passes of 1-3 tiles.  DEBUG 1: loads only; 2: math only.
template <int DEBUG>
__global__ __launch_bounds__(256, 2) void attention_h72p_kernel(AttentionArgs p, int nqt, int LV, int L16) {
  constexpr int DH = 72, ROWB = 144, NCH = 9, NW = 4;
  constexpr float RESCALE_THR = 8.0f;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* Vs = lds;
  char* Km = lds + LV * ROWB;   // K d 0..63, swizzled 128-B rows
  char* Kt = Km + L16 * 128;     // K d 64..71, 16 B per row
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nbh = p.B * p.H, L = p.L, D = p.H * DH;
  const int g = lane >> 4, col = lane & 15;
  const bool glo = g < 2;   // output rows d 64..71 of the fifth PV tile (rows 72..79 are padding)
  const int my_tiles = (nqt - wave + NW - 1) / NW;      // >= 1 (launched with nqt >= 4)
  const int npass = ((nqt + NW - 1) / NW + 2) / 3;
  const int nfull = L / 64, nch = (L + 63) / 64;
  const int r8 = lane >> 3, pc = lane & 7;
  // K / V DMA items per 64-key block c: V 9c .. 9c+8, K d 0..63 8c .. 8c+7, K d 64..71 c (18 per block, the last
  // block possibly fewer), dealt round robin over the head's item list: item k of block c has k = 18c + local
  const int ndmaV = (LV * NCH + 63) / 64, ndmaK = L16 / 8, nblk = (L16 + 63) / 64;
  auto stage_block = [&](int b_, int h_, int c) {
    if (DEBUG == 2) return;
    const __amdgpu_buffer_rsrc_t rq = att_rsrc(p.qkv + (size_t)b_ * L * p.ldq, (long long)L * p.ldq * 2);
    int k = 18 * c;
    for (int i = 9 * c; i < min(9 * c + 9, ndmaV); ++i, ++k) {
      if ((k & 3) != wave) continue;
      const int ci = i * 64 + lane;
      if (ci < LV * NCH) {
        const int row = ci / NCH, ch = ci - row * NCH;
        att_dma16(rq, (unsigned)((row < L ? row : L - 1) * p.ldq + h_ * DH + 2 * D + ch * 8) * 2u,
                  (PDM_LDS void*)(Vs + i * 1024));
      }
    }
    for (int j = 8 * c; j < min(8 * c + 8, ndmaK); ++j, ++k) {
      if ((k & 3) != wave) continue;
      const int row = j * 8 + r8;
      const int kc = pc ^ ((row >> 1) & 7);
      att_dma16(rq, (unsigned)((row < L ? row : L - 1) * p.ldq + h_ * DH + D + kc * 8) * 2u,
                (PDM_LDS void*)(Km + j * 1024));
    }
    if ((k & 3) == wave) {
      const int row = c * 64 + lane;
      if (row < L16)
        att_dma16(rq, (unsigned)((row < L ? row : L - 1) * p.ldq + h_ * DH + D + 64) * 2u, (PDM_LDS void*)(Kt + c * 1024));
    }
  };
  auto items_in = [&](int c) {   // this wave's DMA items of block c
    int n = 0, k = 18 * c;
    for (int i = 9 * c; i < min(9 * c + 9, ndmaV); ++i, ++k) n += (k & 3) == wave;
    for (int j = 8 * c; j < min(8 * c + 8, ndmaK); ++j, ++k) n += (k & 3) == wave;
    return n + ((k & 3) == wave);
  };
  auto ops_after = [&](int c) {   // the first head: this wave's items of blocks past c
    int n = 0;
    for (int cc = c + 1; cc < nblk; ++cc) n += items_in(cc);
    return n;
  };
  auto bar = []() {
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  int bh = blockIdx.x;
  int b = bh / p.H, h = bh - (bh / p.H) * p.H;
  auto qrow = [&](int b_, int h_, int tile) {
    int q = tile * 16 + col;
    q = q < L ? q : L - 1;
    return p.qkv + ((size_t)b_ * L + q) * p.ldq + h_ * DH;
  };
  const int nt0 = my_tiles / npass + (my_tiles % npass ? 1 : 0);
  i32x4 q0[3][2], q0r[3];
  if (DEBUG != 2) {
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const bf16* qr_ = qrow(b, h, wave + NW * min(t, nt0 - 1));
#pragma unroll
      // compiler-visible loads: with inline-asm loads and PDM_WAIT_Q, hipcc split these nine live ranges and copied
      // a destination (v_mov_b64) ahead of the wait -- tools/check_asm_loads.py flagged it in the shipped code
      // object; this opt-in kernel (algo 14) takes hipcc's own wait (vmcnt(0) at first use) instead
      for (int ks = 0; ks < 2; ++ks) q0[t][ks] = *reinterpret_cast<const i32x4*>(qr_ + ks * 32 + g * 8);
      q0r[t] = *reinterpret_cast<const i32x4*>(qr_ + 64);
    }
  }
  for (int c = 0; c < nblk; ++c) stage_block(b, h, c);

  const float sl2 = p.scale * 1.4426950408889634f;
  const bf16x8 ones8 = bf16x8{1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
  const bf16x8 one8 = bf16x8{1.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bf16x8 zero8 = bf16x8{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const char* kbase[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) kbase[ks] = Km + col * 128 + (((ks * 4 + g) ^ ((col >> 1) & 7)) << 4);
  const char* ktail = Kt + col * 16;
  const char* vbase = Vs + (4 * g + (col >> 2)) * ROWB + 8 * (col & 3);

  auto run_pass = [&](auto ntc, const bf16x8 (&qf)[3][2], const bf16x8 (&qr)[3], const int (&tl)[3], bool wait_blocks,
                      bool release, int bn, int hn) {
    constexpr int NT = decltype(ntc)::value;
    float m_run[NT];
    f32x4 acc[NT][5];
    bf16x8 qm[NT];   // Q of the d 64..95 step: d 64..71 (k-group 0) and the slot d = 72 (k-group 1) = -m_run
    auto set_qm = [&](int t) {
      bf16x8 v = qr[t];
      if (g == 1) v[0] = (bf16)(-m_run[t]);
      qm[t] = v;
    };
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      qm[t] = qr[t];
      m_run[t] = -INFINITY;
#pragma unroll
      for (int i = 0; i < 5; ++i) acc[t][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    auto do_block = [&](int c, auto tailc, auto firstc) {
      constexpr int TAIL = decltype(tailc)::value, FIRST = decltype(firstc)::value;
      const int kvalid = L - c * 64;
      // TAIL 1: a ragged last block of <= 16 keys (L = 258, 334, 590): only its first 16-key sub-block is live,
      // the others are neither computed, maxed, shifted nor exponentiated (P = 0), all decided at compile time (a
      // runtime per-sub-block skip measured slower: the branches split the block's straight-line MFMA / VALU code).
      // TAIL 2: any other ragged block, masked over all four sub-blocks.
      constexpr int nkt = TAIL == 1 ? 1 : 4;
      f32x4 s[NT][4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        if (TAIL == 1 ? kt >= 1 : (TAIL && kt * 16 >= kvalid)) continue;
        bf16x8 kx = *reinterpret_cast<const bf16x8*>(ktail + c * 1024 + kt * 256);
        kx = g == 0 ? kx : (g == 1 ? one8 : zero8);
#pragma unroll
        for (int t = 0; t < NT; ++t) s[t][kt] = mfma16x16x32(kx, qm[t], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kbase[ks] + c * 8192 + kt * 2048);
#pragma unroll
          for (int t = 0; t < NT; ++t) s[t][kt] = mfma16x16x32(kf, qf[t][ks], s[t][kt]);
        }
      }
      if constexpr (TAIL) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (kt < nkt && kt * 16 + g * 4 + j >= kvalid)
#pragma unroll
              for (int t = 0; t < NT; ++t) s[t][kt][j] = -INFINITY;
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        f32x4 m4 = s[t][0];
#pragma unroll
        for (int kt = 1; kt < 4; ++kt) {
          if (TAIL && kt >= nkt) break;
#pragma unroll
          for (int j = 0; j < 4; ++j) m4[j] = fmaxf(m4[j], s[t][kt][j]);
        }
        const float cmax = xrow_max(fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3])));
        if constexpr (FIRST) {
          m_run[t] = (float)(bf16)cmax;
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
            if (!TAIL || kt < nkt) s[t][kt] -= m_run[t];
          set_qm(t);
        } else if (__builtin_amdgcn_ballot_w64(cmax > RESCALE_THR)) {
          const float d = cmax > RESCALE_THR ? (float)(bf16)(m_run[t] + cmax) - m_run[t] : 0.f;
          const float alpha = __builtin_amdgcn_exp2f(-d);
          m_run[t] += d;
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
            if (!TAIL || kt < nkt) s[t][kt] -= d;
#pragma unroll
          for (int i = 0; i < 5; ++i) acc[t][i] *= alpha;
          set_qm(t);
        }
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
          if (TAIL && kt >= nkt) {
            s[t][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
            continue;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) s[t][kt][j] = __builtin_amdgcn_exp2f(s[t][kt][j]);
        }
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        if (TAIL == 1 ? kk >= 1 : (TAIL && kk * 32 >= kvalid)) break;
        bf16x8 pf[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            pf[t][j] = (bf16)s[t][2 * kk][j];
            pf[t][4 + j] = (bf16)s[t][2 * kk + 1][j];
          }
        bf16x8 vf[5];
        lds_vt5(vbase + c * (64 * ROWB) + kk * (32 * ROWB), vf);
        vf[4] = (lane & 15) == 8 ? ones8 : vf[4];
#pragma unroll
        for (int dt = 0; dt < 5; ++dt)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[t][dt] = mfma16x16x32(vf[dt], pf[t], acc[t][dt]);
      }
    };
    auto block = [&](int c, auto tailc, auto firstc) {
      if (wait_blocks) {
        if (DEBUG == 0) wait_vmcnt_dyn(ops_after(c));
        else if (DEBUG == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();
      }
      if (DEBUG != 1) do_block(c, tailc, firstc);
      if (release) {   // every wave is done with block c: its rows take the next head's
        bar();
        stage_block(bn, hn, c);
      }
    };
    if (nfull > 0) block(0, std::false_type{}, std::true_type{});
    else block(0, std::integral_constant<int, 2>{}, std::true_type{});
    for (int c = 1; c < nfull; ++c) block(c, std::false_type{}, std::false_type{});
    if (nfull < nch && nfull > 0) {
      block(nfull, std::integral_constant<int, 2>{}, std::false_type{});
    }
    // (no prefetch of the next head's Q here as in attention_v3_kernel: held across the passes it spills at NT = 3)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const float inv = 1.0f / xrow_sum(g == 2 ? acc[t][4][0] : 0.f);   // row d = 72: lanes of k-group 2, j = 0
      const int q = tl[t] * 16 + col;
      if (q < L) {
        bf16* orow = p.out + ((size_t)b * L + q) * p.ldo + h * DH;
#pragma unroll
        for (int dt = 0; dt < 5; ++dt) {
          if (dt == 4 && !glo) break;
          const f32x4 v = acc[t][dt] * inv;
          *reinterpret_cast<bf16x4*>(orow + dt * 16 + g * 4) = to_bf16x4(v[0], v[1], v[2], v[3]);
        }
      }
    }
  };

  bool first_head = true;
  for (;;) {
    const int bhn = bh + gridDim.x;
    const bool has_next = bhn < nbh;
    const int bn = has_next ? bhn / p.H : 0, hn = has_next ? bhn - (bhn / p.H) * p.H : 0;
    int start = 0;
    for (int pass = 0; pass < npass; ++pass) {
      const int nt = my_tiles / npass + (pass < my_tiles % npass ? 1 : 0);
      const int tl[3] = {wave + NW * start, wave + NW * (start + (nt > 1 ? 1 : 0)), wave + NW * (start + (nt > 2 ? 2 : 0))};
      start += nt;
      bf16x8 qf[3][2], qr[3];
      if (first_head && pass == 0) {
        if (DEBUG == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int t = 0; t < 3; ++t) {
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) qf[t][ks] = __builtin_bit_cast(bf16x8, q0[t][ks]);
          qr[t] = g == 0 ? __builtin_bit_cast(bf16x8, q0r[t]) : zero8;
        }
      } else {
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          const bf16* r = qrow(b, h, tl[t]);
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) qf[t][ks] = DEBUG == 2 ? zero8 : *reinterpret_cast<const bf16x8*>(r + ks * 32 + g * 8);
          const bf16x8 v = DEBUG == 2 ? zero8 : *reinterpret_cast<const bf16x8*>(r + 64);
          qr[t] = g == 0 ? v : zero8;
        }
        asm volatile("" : "+v"(qf[0][0]), "+v"(qf[0][1]), "+v"(qf[1][0]), "+v"(qf[1][1]), "+v"(qf[2][0]), "+v"(qf[2][1]),
                     "+v"(qr[0]), "+v"(qr[1]), "+v"(qr[2]));
      }
      if (!p.q_log2) {
#pragma unroll
        for (int t = 0; t < 3; ++t) {
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) qf[t][ks] = scale_bf16x8(qf[t][ks], sl2);
          qr[t] = scale_bf16x8(qr[t], sl2);
        }
      }
      const bool wait_blocks = first_head && pass == 0;
      const bool release = has_next && pass == npass - 1;
      if (nt == 3) run_pass(std::integral_constant<int, 3>{}, qf, qr, tl, wait_blocks, release, bn, hn);
      else if (nt == 2) run_pass(std::integral_constant<int, 2>{}, qf, qr, tl, wait_blocks, release, bn, hn);
      else run_pass(std::integral_constant<int, 1>{}, qf, qr, tl, wait_blocks, release, bn, hn);
    }
    if (!has_next) break;
    bh = bhn;
    b = bn;
    h = hn;
    first_head = false;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
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

// the last key block holds 1..16 keys behind >= 1 full block (L = 258, 334, 590): the kernels' TK = 1 tail
static bool tail1(int L) { return L > 64 && L % 64 != 0 && L % 64 <= 16; }
static int g_attention_algo = 0;   // 0 auto, 1 streamed K/V, 2/3 head-resident T = 2/3, 4 head-resident v2 (5/6 timing)
void attention_set_algo(int algo) { g_attention_algo = algo; }

hipError_t attention_launch(const AttentionArgs& args, hipStream_t stream) {
  AttentionArgs p = args;
  const int nqt = (p.L + 15) / 16;
  int algo = g_attention_algo;
  const int Lp = (p.L + 31) / 32 * 32;   // PV reads whole 32-key steps
  // Dh = 72 (U-ViT-H): head-resident 64 + 8 kernel when two heads' K + V fit per CU (L <= 280); 7/8/9 = timing
  // variants (normal / loads only / math only); measured tools/attn_bench.py
  const int LV = (p.L + 7) / 8 * 8, L16 = (p.L + 15) / 16 * 16;
  const int smem72 = (LV + L16) * 144;   // V rows read past LV (up to round32(L)) alias staged K rows below LV
  // persistent Dh = 72 (14; 15 / 16 = loads-only / math-only timing): every wave owns a tile (nqt >= 4)
  if (p.Dh == 72 && smem72 <= 80 * 1024 && (p.L + 31) / 32 * 32 <= 2 * LV && algo >= 14 && algo <= 16 && nqt >= 4) {
    static bool attr72p = false;
    static int ncu = 256;
    if (!attr72p) {
      (void)hipFuncSetAttribute((const void*)attention_h72p_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
      (void)hipFuncSetAttribute((const void*)attention_h72p_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
      (void)hipFuncSetAttribute((const void*)attention_h72p_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
        ncu = n;
      attr72p = true;
    }
    const int nbh = p.B * p.H, slots = 2 * ncu;
    const dim3 grid(nbh < slots ? nbh : slots), block(256);
    if (algo == 15) hipLaunchKernelGGL(attention_h72p_kernel<1>, grid, block, smem72, stream, p, nqt, LV, L16);
    else if (algo == 16) hipLaunchKernelGGL(attention_h72p_kernel<2>, grid, block, smem72, stream, p, nqt, LV, L16);
    else hipLaunchKernelGGL(attention_h72p_kernel<0>, grid, block, smem72, stream, p, nqt, LV, L16);
    return hipGetLastError();
  }
  if (algo >= 14 && algo <= 16) algo = p.Dh == 72 ? 7 : 0;
  if (p.Dh == 72 && smem72 <= 80 * 1024 && (p.L + 31) / 32 * 32 <= 2 * LV && (algo == 0 || (algo >= 7 && algo <= 9))) {
    static bool attr72 = false;
    if (!attr72) {
      (void)hipFuncSetAttribute((const void*)attention_h72_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
      (void)hipFuncSetAttribute((const void*)attention_h72_kernel<0, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
      (void)hipFuncSetAttribute((const void*)attention_h72_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
      (void)hipFuncSetAttribute((const void*)attention_h72_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
      attr72 = true;
    }
    const dim3 grid(p.B * p.H), block(256);
    if (algo == 8) hipLaunchKernelGGL(attention_h72_kernel<1>, grid, block, smem72, stream, p, nqt, LV, L16);
    else if (algo == 9) hipLaunchKernelGGL(attention_h72_kernel<2>, grid, block, smem72, stream, p, nqt, LV, L16);
    else if (tail1(p.L)) hipLaunchKernelGGL((attention_h72_kernel<0, 1>), grid, block, smem72, stream, p, nqt, LV, L16);
    else hipLaunchKernelGGL(attention_h72_kernel<0>, grid, block, smem72, stream, p, nqt, LV, L16);
    return hipGetLastError();
  }
  // persistent v3 (11; 12 / 13 = loads-only / math-only timing): Dh = 64, every wave owns a tile (nqt >= NW).  The
  // automatic choice wherever it applies: L/2 at 100 rows 76.4 -> 66.6 us, 190 rows 143.5 -> 136.5, 50 rows 44.8 ->
  // 44.0, t2i 334 / 590 unchanged (tools/attn_bench.py, profiles/r05d/attn.log)
  if (algo == 0 && p.Dh == 64 && Lp * 256 <= 160 * 1024) algo = 11;
  if (algo >= 11 && algo <= 13 && p.Dh == 64 && Lp * 256 <= 160 * 1024) {
    const int smem = Lp * 256;
    const int nw = smem <= 80 * 1024 ? 4 : 8;
    if (nqt >= nw) {
      static bool attr3 = false;
      static int ncu = 256;
      if (!attr3) {
        (void)hipFuncSetAttribute((const void*)attention_v3_kernel<0, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)attention_v3_kernel<0, 4, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)attention_v3_kernel<1, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)attention_v3_kernel<2, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)attention_v3_kernel<0, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)attention_v3_kernel<0, 8, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)attention_v3_kernel<1, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)attention_v3_kernel<2, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
          ncu = n;
        attr3 = true;
      }
      const int nbh = p.B * p.H, slots = ncu * (nw == 4 ? 2 : 1);
      const dim3 grid(nbh < slots ? nbh : slots);
      if (nw == 4) {
        if (algo == 11 && tail1(p.L)) hipLaunchKernelGGL((attention_v3_kernel<0, 4, 1>), grid, dim3(256), smem, stream, p, nqt, Lp);
        else if (algo == 11) hipLaunchKernelGGL((attention_v3_kernel<0, 4>), grid, dim3(256), smem, stream, p, nqt, Lp);
        else if (algo == 12) hipLaunchKernelGGL((attention_v3_kernel<1, 4>), grid, dim3(256), smem, stream, p, nqt, Lp);
        else hipLaunchKernelGGL((attention_v3_kernel<2, 4>), grid, dim3(256), smem, stream, p, nqt, Lp);
      } else {
        if (algo == 11 && tail1(p.L)) hipLaunchKernelGGL((attention_v3_kernel<0, 8, 1>), grid, dim3(512), smem, stream, p, nqt, Lp);
        else if (algo == 11) hipLaunchKernelGGL((attention_v3_kernel<0, 8>), grid, dim3(512), smem, stream, p, nqt, Lp);
        else if (algo == 12) hipLaunchKernelGGL((attention_v3_kernel<1, 8>), grid, dim3(512), smem, stream, p, nqt, Lp);
        else hipLaunchKernelGGL((attention_v3_kernel<2, 8>), grid, dim3(512), smem, stream, p, nqt, Lp);
      }
      return hipGetLastError();
    }
    algo = 4;
  }
  if (p.Dh != 64 || Lp * 256 > 160 * 1024) algo = 1;
  // automatic: the head-resident v2 structure wherever the head's K/V fit in LDS (Dh = 64: every U-ViT-S/M/L
  // shape); measured 152 vs 213 us (streamed) on L/2 at 190 rows (tools/attn_bench.py)
  if (algo == 0 && p.Dh == 64 && Lp * 256 <= 160 * 1024) algo = 4;
  if (algo == 10 && p.Dh == 64 && Lp * 256 <= 160 * 1024) {   // v2 with VALU row sums (A/B: 145.7 vs 140.1 us, L/2)
    const int smem = Lp * 256;
    static bool attr10 = false;
    if (!attr10) {
      (void)hipFuncSetAttribute((const void*)attention_v2_kernel<0, 4, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)attention_v2_kernel<0, 8, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr10 = true;
    }
    if (smem <= 80 * 1024) hipLaunchKernelGGL((attention_v2_kernel<0, 4, false>), dim3(p.B * p.H), dim3(256), smem, stream, p, nqt, Lp);
    else hipLaunchKernelGGL((attention_v2_kernel<0, 8, false>), dim3(p.B * p.H), dim3(512), smem, stream, p, nqt, Lp);
    return hipGetLastError();
  }
  if (algo >= 4 && algo <= 6 && p.Dh == 64 && Lp * 256 <= 160 * 1024) {
    const int smem = Lp * 256;
    static bool attr2 = false;
    if (!attr2) {
      (void)hipFuncSetAttribute((const void*)attention_v2_kernel<0, 4, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)attention_v2_kernel<1, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)attention_v2_kernel<2, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)attention_v2_kernel<0, 8, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)attention_v2_kernel<1, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)attention_v2_kernel<2, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr2 = true;
    }
    const dim3 grid(p.B * p.H);
    if (smem <= 80 * 1024) {   // two heads per CU: 4 waves each
      if (algo == 4) hipLaunchKernelGGL((attention_v2_kernel<0, 4, true>), grid, dim3(256), smem, stream, p, nqt, Lp);
      else if (algo == 5) hipLaunchKernelGGL((attention_v2_kernel<1, 4>), grid, dim3(256), smem, stream, p, nqt, Lp);
      else hipLaunchKernelGGL((attention_v2_kernel<2, 4>), grid, dim3(256), smem, stream, p, nqt, Lp);
    } else {                   // one head per CU: 8 waves (two per SIMD)
      if (algo == 4) hipLaunchKernelGGL((attention_v2_kernel<0, 8, true>), grid, dim3(512), smem, stream, p, nqt, Lp);
      else if (algo == 5) hipLaunchKernelGGL((attention_v2_kernel<1, 8>), grid, dim3(512), smem, stream, p, nqt, Lp);
      else hipLaunchKernelGGL((attention_v2_kernel<2, 8>), grid, dim3(512), smem, stream, p, nqt, Lp);
    }
    return hipGetLastError();
  }
  // the kernels below compute exp2(S * scale * log2 e): with q pre-scaled by scale * log2(e) (q_log2) they take
  // scale = ln 2 (the head-resident kernels above read q_log2 themselves and work in log2 units either way)
  if (p.q_log2) p.scale = 0.69314718055994531f;
  if (algo == 0 || algo >= 4) algo = 1;
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

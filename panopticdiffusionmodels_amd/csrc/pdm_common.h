// Shared device helpers for the gfx950 (CDNA4) kernels of libpdm.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pdm {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));

#define PDM_LDS __attribute__((address_space(3)))

__device__ __forceinline__ f32x4 mfma16x16x32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// 16-byte async copy global -> LDS.  `lds_wave_base` must be wave-uniform; lane l lands at base + 16*l.
__device__ __forceinline__ void glds16(const void* gptr, PDM_LDS void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(gptr, lds_wave_base, 16, 0, 0);
}

// nn.GELU() default, exact erf form (libs/uvit.py:98 / libs/timm.py:102):  GELU(x) = x Phi(x) = x (1/2 + x P(x^2)).
// Phi - 1/2 is odd, so it is fitted as  s Q(s^2 - 1/2),  s = clamp(x / 4.5, -1, 1),  Q of degree 9: a minimax fit
// (linear programme over [0, 4.5]) constrained to Phi(4.5) := 1 exactly, so GELU(x) is exactly 0 for x <= -4.5
// and exactly x for x >= 4.5 (the true tails differ by < 1.6e-5).  The centred variable s^2 - 1/2 keeps the
// coefficients O(1) (no fp32 cancellation in Horner); the constant term is nudged so that fp32 Q(1/2) = 1/2.
// Error over the real line: |abs| <= 1.8e-5, relative <= 9.5e-4 wherever |GELU| > 1e-2 -- under half a bf16 ulp of
// the GEMM outputs it feeds.  No transcendental: 13 FMA/multiplies and 2 clamps, all packable two-wide.
#define PDM_GELU_COEFFS                                                                                        \
  7.060773373e-01f, -6.946521401e-01f, 9.834588766e-01f, -1.449834466e+00f, 2.078067064e+00f,                  \
      -2.640194416e+00f, 2.778215170e+00f, -3.625102520e+00f, 5.720444202e+00f, -4.195198536e+00f
__device__ __forceinline__ float gelu_erf(float x) {
  constexpr float c[10] = {PDM_GELU_COEFFS};
  const float s = __builtin_amdgcn_fmed3f(x * (1.0f / 4.5f), -1.0f, 1.0f);
  const float v = fmaf(s, s, -0.5f);
  float p = c[9];
#pragma unroll
  for (int k = 8; k >= 0; --k) p = fmaf(p, v, c[k]);
  return x * fmaf(s, p, 0.5f);
}

// The same GELU on two values at once, written on 2-wide vectors so the scaling, the polynomial and the final
// multiply issue as packed fp32 (v_pk_fma_f32 / v_pk_mul_f32: two lanes' work per VALU cycle); only the two
// clamps stay scalar.  Bit-identical to gelu_erf.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) {
  constexpr float c[10] = {PDM_GELU_COEFFS};
  f32x2 s = x * (1.0f / 4.5f);
  s[0] = __builtin_amdgcn_fmed3f(s[0], -1.0f, 1.0f);
  s[1] = __builtin_amdgcn_fmed3f(s[1], -1.0f, 1.0f);
  const f32x2 v = __builtin_elementwise_fma(s, s, f32x2(-0.5f));
  f32x2 p = f32x2(c[9]);
#pragma unroll
  for (int k = 8; k >= 0; --k) p = __builtin_elementwise_fma(p, v, f32x2(c[k]));
  return x * __builtin_elementwise_fma(s, p, f32x2(0.5f));
}
// gelu_erf2 on four independent pairs with each Horner step issued for all four before the next: hipcc otherwise
// emits one pair's 13 dependent packed ops back to back (an s_nop between each), so a GELU epilogue runs at the
// VALU latency, not its issue rate.  Bit-identical to gelu_erf (the same operations per element).
__device__ __forceinline__ void gelu_erf2x4(f32x2 (&x)[4]) {
  constexpr float c[10] = {PDM_GELU_COEFFS};
  f32x2 s[4], v[4], p[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    s[j] = x[j] * (1.0f / 4.5f);
    s[j][0] = __builtin_amdgcn_fmed3f(s[j][0], -1.0f, 1.0f);
    s[j][1] = __builtin_amdgcn_fmed3f(s[j][1], -1.0f, 1.0f);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = __builtin_elementwise_fma(s[j], s[j], f32x2(-0.5f));
#pragma unroll
  for (int j = 0; j < 4; ++j) p[j] = __builtin_elementwise_fma(f32x2(c[9]), v[j], f32x2(c[8]));
#pragma unroll
  for (int k = 7; k >= 0; --k)
#pragma unroll
    for (int j = 0; j < 4; ++j) p[j] = __builtin_elementwise_fma(p[j], v[j], f32x2(c[k]));
#pragma unroll
  for (int j = 0; j < 4; ++j) x[j] = x[j] * __builtin_elementwise_fma(s[j], p[j], f32x2(0.5f));
}
#undef PDM_GELU_COEFFS

// quick GELU (transformers QuickGELUActivation, CLIP text encoder): x * sigmoid(1.702 x)
// (hardware reciprocal instead of the IEEE divide: 1 ulp, and exp overflow for x << 0 still gives -0)
__device__ __forceinline__ float gelu_quick(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * x)); }
__device__ __forceinline__ float gelu_act(int act, float x) { return act ? gelu_quick(x) : gelu_erf(x); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Fused LayerNorm: merge one row's ceil(D/256) partials (sum, M2 about the group mean; groups of 256 columns,
// the last one D - 256 t wide) with Chan's update -> (mean, 1/sqrt(var + eps)), biased variance like torch.
__device__ __forceinline__ float2 ln_merge(const float* st, int T, int D, float eps) {
  float sum = 0.f;
  for (int t = 0; t < T; ++t) sum += st[2 * t];
  const float mean = sum / (float)D;
  float m2 = 0.f;
  for (int t = 0; t < T; ++t) {
    const float n = (float)min(256, D - 256 * t);
    const float d = st[2 * t] / n - mean;
    m2 += st[2 * t + 1] + n * d * d;
  }
  return make_float2(mean, 1.0f / sqrtf(m2 / (float)D + eps));
}

// MXFP8 quantisation of one 32-element block spread over 4 consecutive lanes (8 values each, lane & 3 =
// position in the block): E8M0 exponent e = ceil(log2(amax / 448)) + 127 (so |v| 2^-(e-127) <= 448, no
// saturation), e4m3 data with round-to-nearest-even (v_cvt_pk_fp8_f32, OCP e4m3 on gfx950).  Returns the 8
// packed bytes; *e8 receives the block's biased exponent.
__device__ __forceinline__ uint2 mx_quant8(const float (&v)[8], unsigned* e8) {
  float am = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) am = fmaxf(am, fabsf(v[j]));
  am = fmaxf(am, __shfl_xor(am, 1, 64));
  am = fmaxf(am, __shfl_xor(am, 2, 64));
  const unsigned bits = __float_as_uint(am * (1.0f / 448.0f));
  unsigned e = (bits >> 23) & 0xffu;
  e += (bits & 0x7fffffu) ? 1u : 0u;
  e = e > 254u ? 254u : e;
  const float inv = __uint_as_float((254u - e) << 23);   // 2^(127 - e)
  int w0 = 0, w1 = 0;
  w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, w0, false);
  w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, w0, true);
  w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, w1, false);
  w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, w1, true);
  *e8 = e;
  return make_uint2((unsigned)w0, (unsigned)w1);
}

// the same for a block spread over 8 consecutive lanes with 4 values each (row kernels, float4 per lane)
__device__ __forceinline__ unsigned mx_quant4(const f32x4& v, unsigned* e8) {
  float am = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
  am = fmaxf(am, __shfl_xor(am, 1, 64));
  am = fmaxf(am, __shfl_xor(am, 2, 64));
  am = fmaxf(am, __shfl_xor(am, 4, 64));
  const unsigned bits = __float_as_uint(am * (1.0f / 448.0f));
  unsigned e = (bits >> 23) & 0xffu;
  e += (bits & 0x7fffffu) ? 1u : 0u;
  e = e > 254u ? 254u : e;
  const float inv = __uint_as_float((254u - e) << 23);
  int w = 0;
  w = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, w, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, w, true);
  *e8 = e;
  return (unsigned)w;
}

// store of one quantised 8-column piece (row m, columns n .. n+7) of an MXFP8 output, and of its block scale
// by the block's first lane
__device__ __forceinline__ void mx_store8(unsigned char* out, int ldo8, unsigned* scale, int scale_ld, int m, int n,
                                          uint2 q, unsigned e8, bool first) {
  *reinterpret_cast<uint2*>(out + (size_t)m * ldo8 + n) = q;
  if (first)
    reinterpret_cast<unsigned char*>(scale)[((size_t)(n >> 7) * scale_ld + m) * 4 + ((n >> 5) & 3)] = (unsigned char)e8;
}

__device__ __forceinline__ bf16x4 to_bf16x4(float a, float b, float c, float d) {
  bf16x4 r;
  r[0] = (bf16)a; r[1] = (bf16)b; r[2] = (bf16)c; r[3] = (bf16)d;
  return r;
}

}  // namespace pdm

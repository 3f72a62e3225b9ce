// VALU issue-rate probe (dev tool): cycles per wave64 instruction for v_exp_f32, v_fma_f32, v_pk_fma_f32,
// v_cvt_pk_bf16_f32-style packing and v_lshl_add_u32, each in 8 independent chains, one wave per SIMD and four
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int N = 4096;
template <int OP>
__global__ void k(float* out, float seed, long long* cyc) {
  float a[8];
  f32x2 p[8];
  unsigned u[8];
  for (int i = 0; i < 8; ++i) { a[i] = seed + threadIdx.x * 1e-3f + i; p[i] = f32x2{a[i], a[i] * 0.5f}; u[i] = threadIdx.x + i; }
  const long long t0 = clock64();
  for (int it = 0; it < N; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (OP == 0) a[i] = __builtin_amdgcn_exp2f(a[i]);
      else if constexpr (OP == 1) a[i] = fmaf(a[i], 0.999f, 0.001f);
      else if constexpr (OP == 2) p[i] = __builtin_elementwise_fma(p[i], f32x2{0.999f, 0.999f}, f32x2{0.001f, 0.001f});
      else u[i] = (u[i] << 3) + u[(i + 1) & 7];
    }
  }
  const long long t1 = clock64();
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += a[i] + p[i][0] + p[i][1] + (float)u[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
int main() {
  float* o; long long* c;
  (void)hipMalloc(&o, 1 << 20); (void)hipMalloc(&c, 8);
  const char* nm[4] = {"v_exp_f32", "v_fma_f32", "v_pk_fma_f32", "lshl_add_u32"};
  for (int waves = 1; waves <= 4; waves *= 4)
    for (int op = 0; op < 4; ++op) {
      for (int r = 0; r < 2; ++r) {
        dim3 g(1), b(64 * 4 * waves);
        if (op == 0) hipLaunchKernelGGL(k<0>, g, b, 0, 0, o, 0.f, c);
        if (op == 1) hipLaunchKernelGGL(k<1>, g, b, 0, 0, o, 0.f, c);
        if (op == 2) hipLaunchKernelGGL(k<2>, g, b, 0, 0, o, 0.f, c);
        if (op == 3) hipLaunchKernelGGL(k<3>, g, b, 0, 0, o, 0.f, c);
        (void)hipDeviceSynchronize();
      }
      long long h; (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
      printf("%-14s waves/SIMD %d: %.2f clk per instruction per wave\n", nm[op], waves, (double)h / (N * 8.0));
    }
  return 0;
}

// lane-exchange probe (dev tool): each DPP / permlane step on lane ids, printed per lane, and gemm.hip's sum32
// (the 32-lane row-statistics reduction) on lane ids (expected 496 in lanes 0-31, 1520 in lanes 32-63)
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int CTRL>
__device__ float dpp_mov(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ float dpp_add(float x) { return x + dpp_mov<CTRL>(x); }
__device__ __forceinline__ float sum32(float x) {
  x = dpp_add<0xb1>(x);
  x = dpp_add<0x4e>(x);
  x = dpp_add<0x141>(x);
  x = dpp_add<0x140>(x);
  return x + __shfl_xor(x, 16, 64);
}
__global__ void k(float* out) {
  const int l = threadIdx.x;
  const float x = (float)l;
  out[0 * 64 + l] = dpp_mov<0xb1>(x);
  out[1 * 64 + l] = dpp_mov<0x4e>(x);
  out[2 * 64 + l] = dpp_mov<0x141>(x);
  out[3 * 64 + l] = dpp_mov<0x140>(x);
  const unsigned u = __builtin_bit_cast(unsigned, x);
  unsigned u2;
  asm volatile("v_mov_b32 %0, %1" : "=v"(u2) : "v"(u));
  const auto r = __builtin_amdgcn_permlane16_swap(u, u2, false, false);
  out[4 * 64 + l] = __builtin_bit_cast(float, r[0]);
  out[5 * 64 + l] = __builtin_bit_cast(float, r[1]);
  out[6 * 64 + l] = sum32(x);
}
int main() {
  float* d;
  (void)hipMalloc(&d, 7 * 64 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  float h[7 * 64];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[7] = {"qp1032", "qp2301", "halfmirror", "mirror", "pl16[0]", "pl16[1]", "sum32"};
  for (int s = 0; s < 7; ++s) {
    printf("%-10s", nm[s]);
    for (int l = 0; l < 64; ++l) printf(" %d", (int)h[s * 64 + l]);
    printf("\n");
  }
  int bad = 0;
  for (int l = 0; l < 64; ++l) bad += h[6 * 64 + l] != (l < 32 ? 496.f : 1520.f);
  printf("sum32 %s\n", bad ? "WRONG" : "ok");
  return bad != 0;
}

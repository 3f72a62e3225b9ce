// Probe: operand / scale lane layout of v_mfma_scale_f32_16x16x128_f8f6f4 (fp8 e4m3 x fp8 e4m3, E8M0 block
// scales) on gfx950, checked against a host reference on exact small-integer data.
// Result on MI355X (ROCm 7.2): lane l = 16 g + r holds row r, bytes 0-15 = k 16g .. 16g+15 and bytes 16-31 =
// k 64+16g .. 64+16g+15 (any consistent permutation multiplies correctly; this one is what the block scales
// see); the scale operand of lane 16 g + r (byte 0, opsel 0) scales row r's k-block g = k 32g .. 32g+31.  Each hypothesis maps the
// logical A[16][128] / B^T[16][128] into per-lane 32-byte fragments on the host; the kernel loads lane l's
// 32 bytes verbatim.  Build + run:  hipcc --offload-arch=gfx950 -O2 mx_layout.hip -o mx_layout && ./mx_layout
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void probe(const unsigned char* A, const unsigned char* B, const int* sa, const int* sb, float* C) {
  int l = threadIdx.x;
  v8i a, b;
  for (int i = 0; i < 8; ++i) { a[i] = ((const int*)(A + l * 32))[i]; b[i] = ((const int*)(B + l * 32))[i]; }
  v4f c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa[l], 0, sb[l]);
  for (int j = 0; j < 4; ++j) C[((l >> 4) * 4 + j) * 16 + (l & 15)] = c[j];
}

static float e4m3(unsigned char v) {
  int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float f = e ? ldexpf(1.f + m / 8.f, e - 7) : ldexpf(m / 8.f, -6);
  return s ? -f : f;
}

// k index of byte j (0..31) of lane l under hypothesis h
static int kmap(int h, int l, int j) {
  const int g = l >> 4;
  switch (h) {
    case 0: return 32 * g + j;                                  // contiguous 32 per lane group
    case 1: return (j < 16) ? 16 * g + j : 64 + 16 * g + (j - 16); // two K=64 halves
    case 2: return 8 * g + (j & 7) + 32 * (j >> 3);             // 8-byte groups interleaved
    default: return (j < 8) ? 8 * g + j : 32 + ((j - 8) % 24) + 0;
  }
}

int main() {
  unsigned char hA[16 * 128], hB[16 * 128];
  srand(1);
  const unsigned char code[5] = {0xB8, 0x00, 0x38, 0x40, 0x44};   // -1, 0, 1, 2, 3
  for (int i = 0; i < 16 * 128; ++i) { hA[i] = code[rand() % 5]; hB[i] = code[rand() % 5]; }
  unsigned char *dA, *dB;
  int *dsa, *dsb;
  float* dC;
  (void)hipMalloc(&dA, 2048); (void)hipMalloc(&dB, 2048); (void)hipMalloc(&dsa, 256); (void)hipMalloc(&dsb, 256);
  (void)hipMalloc(&dC, 1024);
  int best = -1;
  for (int h = 0; h < 3; ++h) {
    unsigned char la[2048], lb[2048];
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 32; ++j) {
        la[l * 32 + j] = hA[(l & 15) * 128 + kmap(h, l, j)];
        lb[l * 32 + j] = hB[(l & 15) * 128 + kmap(h, l, j)];
      }
    int ones[64];
    for (int i = 0; i < 64; ++i) ones[i] = 127;
    (void)hipMemcpy(dA, la, 2048, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, lb, 2048, hipMemcpyHostToDevice);
    (void)hipMemcpy(dsa, ones, 256, hipMemcpyHostToDevice);
    (void)hipMemcpy(dsb, ones, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC);
    float hC[256];
    (void)hipMemcpy(hC, dC, 1024, hipMemcpyDeviceToHost);
    double maxerr = 0;
    for (int r = 0; r < 16; ++r)
      for (int c = 0; c < 16; ++c) {
        double ref = 0;
        for (int k = 0; k < 128; ++k) ref += (double)e4m3(hA[r * 128 + k]) * e4m3(hB[c * 128 + k]);
        maxerr = fmax(maxerr, fabs(ref - hC[r * 16 + c]));
      }
    printf("hypothesis %d (unit scales): max |C - ref| = %g\n", h, maxerr);
    if (maxerr < 1e-3 && best < 0) best = h;
  }
  if (best < 0) return 1;
  // scale semantics: A one-hot (1.0 at lane L, byte j; row L & 15), B all 1.0 with unit scales, A scales of
  // lane group g = 2^(g+1): C[row][0] = 2^(g'+1) names the lane group g' whose scale covers that byte
  {
    unsigned char lb1[2048];
    for (int i = 0; i < 2048; ++i) lb1[i] = 0x38;   // 1.0
    (void)hipMemcpy(dB, lb1, 2048, hipMemcpyHostToDevice);
    int ones[64], s[64];
    for (int i = 0; i < 64; ++i) { ones[i] = 127; s[i] = 127 + (i >> 4) + 1; }
    (void)hipMemcpy(dsb, ones, 256, hipMemcpyHostToDevice);
    (void)hipMemcpy(dsa, s, 256, hipMemcpyHostToDevice);
    for (int L = 0; L < 64; L += 16) {
      printf("lane %2d bytes 0..31 -> scale group:", L);
      for (int j = 0; j < 32; ++j) {
        unsigned char la1[2048];
        memset(la1, 0, 2048);
        la1[L * 32 + j] = 0x38;
        (void)hipMemcpy(dA, la1, 2048, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC);
        float hC[256];
        (void)hipMemcpy(hC, dC, 1024, hipMemcpyDeviceToHost);
        const float v = hC[(L & 15) * 16 + 0];
        printf(" %d", v > 0 ? (int)lrintf(log2f(v)) - 1 : -9);
      }
      printf("\n");
    }
  }
  return 0;
}

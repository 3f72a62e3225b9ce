// Output stage of the sampling path: decoded images -> 8-bit PNG pixels, analog-bit
// panoptic masks -> ids -> colour-mapped pixels.  Restates, bit for bit:
//   datasets.py:104-108 unpreprocess: v = clamp(0.5 * (v + 1), 0, 1)
//   torchvision save_image (utils.py:629/633): u8 = (uint8) clamp(v * 255 + 0.5, 0, 255), HWC
//   utils.py:490-518 bits2int(pred_mask > 0) + utils.py:532-543 color_map: id = sum_i (b_i > 0) 2^(n-1-i),
//   rgb = colormap[id]
// Each float op is rounded separately (no contraction), as the reference's separate tensor ops are.
// Non-finite input: fmaxf/fminf map NaN to 0, so a NaN pixel is written as 0.  torch's clamp_ keeps the NaN and
// its float -> uint8 cast of NaN is undefined (0 on the x86 host path), so this is the one case where the output
// is defined here and not in the reference; ±inf saturate exactly as the torch ops do.  A diverged sample is still
// visible upstream: output.py images_to_u8 counts non-finite values and warns before quantising.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/pdm.h"
#include "pdm_kernels.h"

namespace pdm {
namespace {

__global__ __launch_bounds__(256) void images_to_u8_kernel(const float* img, uint8_t* out, int C, int HW, long long npix) {
  const long long i = blockIdx.x * 256ll + threadIdx.x;   // pixel (b, y, x)
  if (i >= npix) return;
  const long long b = i / HW;
  const int p = (int)(i - b * HW);
  const float* src = img + b * C * HW + p;
  uint8_t* dst = out + i * C;
  for (int c = 0; c < C; ++c) {
    float v = __fmul_rn(0.5f, __fadd_rn(src[(size_t)c * HW], 1.0f));
    v = fminf(fmaxf(v, 0.0f), 1.0f);
    float u = __fadd_rn(__fmul_rn(v, 255.0f), 0.5f);
    u = fminf(fmaxf(u, 0.0f), 255.0f);
    dst[c] = (uint8_t)u;   // truncation, as Tensor.to(torch.uint8)
  }
}

__global__ __launch_bounds__(256) void mask_bits_to_rgb_kernel(const float* bits, int nbits, const int32_t* cmap,
                                                               int32_t* ids, uint8_t* rgb, int HW, long long npix) {
  const long long i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= npix) return;
  const long long b = i / HW;
  const int p = (int)(i - b * HW);
  const float* src = bits + b * nbits * HW + p;
  int id = 0;
  for (int k = 0; k < nbits; ++k) id = (id << 1) | (src[(size_t)k * HW] > 0.0f ? 1 : 0);
  if (ids) ids[i] = id;
  if (rgb) {
    const int row = id & 255;
    rgb[i * 3 + 0] = (uint8_t)cmap[row * 3 + 0];
    rgb[i * 3 + 1] = (uint8_t)cmap[row * 3 + 1];
    rgb[i * 3 + 2] = (uint8_t)cmap[row * 3 + 2];
  }
}

}  // namespace
}  // namespace pdm

extern "C" {

int pdm_images_to_u8(const float* img, uint8_t* out, int B, int C, int H, int W, void* stream) {
  if (!img || !out || B <= 0 || C <= 0 || H <= 0 || W <= 0)
    return pdm::set_error(PDM_ERR_ARG, "pdm_images_to_u8: bad argument");
  const long long npix = (long long)B * H * W;
  hipLaunchKernelGGL(pdm::images_to_u8_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, img, out, C, H * W, npix);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? PDM_OK : pdm::set_error(PDM_ERR_HIP, hipGetErrorString(e));
}

int pdm_mask_bits_to_rgb(const float* bits, int nbits, const int32_t* colormap, int32_t* ids, uint8_t* rgb, int B,
                         int H, int W, void* stream) {
  if (!bits || nbits <= 0 || nbits > 8 || B <= 0 || H <= 0 || W <= 0 || (!ids && !rgb) || (rgb && !colormap))
    return pdm::set_error(PDM_ERR_ARG, "pdm_mask_bits_to_rgb: bad argument");
  const long long npix = (long long)B * H * W;
  hipLaunchKernelGGL(pdm::mask_bits_to_rgb_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, bits, nbits, colormap, ids, rgb, H * W, npix);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? PDM_OK : pdm::set_error(PDM_ERR_HIP, hipGetErrorString(e));
}

}  // extern "C"

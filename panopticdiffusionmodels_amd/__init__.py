"""MI355X-native Panoptic-Diffusion sampling hot path: U-ViT / U-ViT-t2i forward, DPM-Solver(++) loops with
classifier-free guidance and the KL-f8 decode, as hand-written gfx950 HIP kernels behind a C ABI
(include/pdm.h, libpdm.so).  The Python modules keep the reference's API surface."""
__version__ = "0.1.0"

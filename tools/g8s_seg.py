"""Shader cycles per main-loop segment of the persistent GEMM (dev tool; needs a -DPDM_G8S_SEG build,
tools/build_variant.sh): for wave 0 (first half) and wave 4 (second half, one barrier behind), the average cycles per
K-tile in each of the 12 segments (per phase: fragment reads, refill issue, vmcnt wait, barrier, MFMAs, barrier).
  PDM_LIB_PATH=ab/libpdm_seg.so python tools/g8s_seg.py [rows]"""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

lib = _lib.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100
D, L = 1024, 258
M = rows * L
g = torch.Generator(device="cuda").manual_seed(0)
A = torch.randn(M, 4 * D, device="cuda", generator=g).bfloat16()
X = torch.randn(M, D, device="cuda", generator=g)
Xb = X.bfloat16()
outb = torch.empty(M, 4 * D, device="cuda", dtype=torch.bfloat16)
st_out = torch.empty(M, (D + 255) // 256, 2, device="cuda")
_, ln_st = _lib.rowstats(X)
buf = (ctypes.c_ulonglong * 25)()
_w = (torch.randn(3 * D, D, device="cuda", generator=g) * D ** -0.5).bfloat16()
for _ in range(200):
    _lib.gemm_ex(_lib.EPI_BF16, A[:, :D], _w, None, out=outb[:, :3 * D])
torch.cuda.synchronize()
NAMES = ["rdA", "dmaA", "waitA", "barA", "mmaA", "barA2", "rdB", "dmaB", "waitB", "barB", "mmaB", "barB2"]
for name, N, K, kind in [("qkv", 3 * D, D, "ln"), ("proj", D, D, "res"), ("fc2", D, 4 * D, "res")]:
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    colsum = torch.randn(N, device="cuda", generator=g)
    a, o = A[:, :K], outb[:, :N]
    if kind == "ln":
        fn = lambda: _lib.gemm_ex(_lib.EPI_BF16, a, W, bias, out=o, ln_stats=ln_st, ln_colsum=colsum)
    else:
        fn = lambda: _lib.gemm_ex(_lib.EPI_RES, a, W, bias, out=Xb, res_in=Xb, accumulate=True, stats_out=st_out)
    ntiles = ((M + 255) // 256) * ((N + 255) // 256)
    for vn, bit in (("fwd", 0), ("noepi", 16)):
        lib.pdm_set_gemm_tuning(0, bit)
        for _ in range(10):
            fn()
        assert lib.pdm_gemm_seg_stats(buf) == 0
        n = 20
        for _ in range(n):
            fn()
        assert lib.pdm_gemm_seg_stats(buf) == 0
        lib.pdm_set_gemm_tuning(0, 0)
        nwg = buf[24]
        kt = ntiles * (K // 64) * n   # K-tiles over all workgroups
        w0 = [buf[i] / kt for i in range(12)]
        w4 = [buf[12 + i] / kt for i in range(12)]
        print(f"{name:5s} {vn:6s} M={M} N={N} K={K} ({nwg // n} wg): cycles per K-tile  wave0 " +
              " ".join(f"{k}={v:.0f}" for k, v in zip(NAMES, w0)) + f" sum={sum(w0):.0f} | wave4 " +
              " ".join(f"{k}={v:.0f}" for k, v in zip(NAMES, w4)) + f" sum={sum(w4):.0f}", flush=True)

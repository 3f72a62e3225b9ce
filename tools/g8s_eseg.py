"""Shader cycles per tile in each part of the persistent GEMM's epilogue (dev tool; needs a -DPDM_G8S_ESEG build,
tools/build_variant.sh): wave 0 (first half) and wave 4 (second half).  Parts: 0 rejoin barrier, 1 column tables +
LN row statistics + LDS sync, 2 barrier + next tile's tables + row reads, 3 residual loads + per-row compute + stores
(EPI_RES), 4 LayerNorm partials (EPI_RES), 5 LDS sync + barrier (EPI_RES), 6 combine + partial store (EPI_RES) /
output loop (bf16 / GELU).
  PDM_LIB_PATH=ab/libpdm_eseg.so python tools/g8s_eseg.py [rows]"""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

lib = _lib.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 50
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
NAMES = ["rejoin", "tables+lnstats", "bar+next+rows", "res+compute+st", "partials", "sync+bar", "combine/out"]
for name, N, K, kind in [("qkv", 3 * D, D, "ln"), ("fc1", 4 * D, D, "ln_gelu"), ("proj", D, D, "res"),
                         ("fc2", D, 4 * D, "res")]:
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    colsum = torch.randn(N, device="cuda", generator=g)
    a, o = A[:, :K], outb[:, :N]
    if kind == "ln":
        fn = lambda: _lib.gemm_ex(_lib.EPI_BF16, a, W, bias, out=o, ln_stats=ln_st, ln_colsum=colsum)
    elif kind == "ln_gelu":
        fn = lambda: _lib.gemm_ex(_lib.EPI_GELU, a, W, bias, out=o, ln_stats=ln_st, ln_colsum=colsum)
    else:
        fn = lambda: _lib.gemm_ex(_lib.EPI_RES, a, W, bias, out=Xb, res_in=Xb, accumulate=True, stats_out=st_out)
    ntiles = ((M + 255) // 256) * ((N + 255) // 256)
    for _ in range(10):
        fn()
    assert lib.pdm_gemm_seg_stats(buf) == 0
    n = 20
    for _ in range(n):
        fn()
    assert lib.pdm_gemm_seg_stats(buf) == 0
    w0 = [buf[i] / (ntiles * n) for i in range(7)]
    w4 = [buf[12 + i] / (ntiles * n) for i in range(7)]
    print(f"{name:5s} M={M} N={N} K={K}: cycles per tile  wave0 " + " ".join(f"{k}={v:.0f}" for k, v in zip(NAMES, w0)) +
          f" sum={sum(w0):.0f} | wave4 " + " ".join(f"{k}={v:.0f}" for k, v in zip(NAMES, w4)) + f" sum={sum(w4):.0f}",
          flush=True)

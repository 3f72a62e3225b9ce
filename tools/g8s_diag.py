"""What bounds the persistent GEMM's main loop (dev tool): each U-ViT block GEMM at the bench's rows with its forward
epilogue and with no epilogue (dbg bit 16).  Run it on builds with -DPDM_G8S_DIAG=bits (tools/build_variant.sh), whose
main loop drops its LDS-DMA refills (1) / fragment reads (2) / MFMAs (4) -- wrong results, timing only.
  PDM_LIB_PATH=ab/libpdm_diag1.so python tools/g8s_diag.py [rows] [D]"""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

lib = _lib.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100
D = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
L = 258
M = rows * L
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
A = torch.randn(M, 4 * D, device=dev, generator=g).bfloat16()
X = torch.randn(M, D, device=dev, generator=g)
Xb = X.bfloat16()
outb = torch.empty(M, 4 * D, device=dev, dtype=torch.bfloat16)
st_out = torch.empty(M, (D + 255) // 256, 2, device=dev)
_, ln_st = _lib.rowstats(X)


def timeit(fn, n=10, rounds=5):
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / n)
    return sorted(ts)[rounds // 2] * 1e3


_w = torch.randn(3 * D, D, device=dev, generator=g).bfloat16()
for _ in range(300):
    _lib.gemm_ex(_lib.EPI_BF16, A[:, :D], _w, None, out=outb[:, :3 * D])
torch.cuda.synchronize()

VARIANTS = [("fwd", 0), ("noepi", 16), ("nostore", 32)]
for name, N, K, kind in [("qkv", 3 * D, D, "ln"), ("proj", D, D, "res"), ("fc1", 4 * D, D, "ln_gelu"),
                         ("fc2", D, 4 * D, "res"), ("skip", D, 2 * D, "res")]:
    W = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device=dev, generator=g)
    colsum = torch.randn(N, device=dev, generator=g)
    a, o = A[:, :K], outb[:, :N]
    if kind == "ln":
        fn = lambda: _lib.gemm_ex(_lib.EPI_BF16, a, W, bias, out=o, ln_stats=ln_st, ln_colsum=colsum)
    elif kind == "ln_gelu":
        fn = lambda: _lib.gemm_ex(_lib.EPI_GELU, a, W, bias, out=o, ln_stats=ln_st, ln_colsum=colsum)
    else:
        fn = lambda: _lib.gemm_ex(_lib.EPI_RES, a, W, bias, out=Xb, res_in=Xb, accumulate=True, stats_out=st_out)
    f = 2.0 * M * N * K
    line = f"{name:5s} M={M} N={N} K={K}"
    for vn, bit in VARIANTS:
        lib.pdm_set_gemm_tuning(0, bit)
        try:
            fn()
            t = timeit(fn)
        finally:
            lib.pdm_set_gemm_tuning(0, 0)
        line += f" | {vn} {t:6.1f}us {f / t / 1e6:5.0f}TF"
    print(line, flush=True)

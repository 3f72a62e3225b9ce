"""Phase-stagger probe (dev tool): time the block GEMMs in their forward epilogue form with half of the first
wave's workgroups delayed by k x s_sleep(127) (GemmArgs::dbg_tile0 bit 4), k = 0..8."""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

lib = _lib.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 190
D, L = 1024, 258
M = rows * L
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
A = torch.randn(M, 4 * D, device=dev, generator=g).bfloat16()
X = torch.randn(M, D, device=dev, generator=g)
Xb = X.bfloat16()
outb = torch.empty(M, 4 * D, device=dev, dtype=torch.bfloat16)
st_out = torch.empty(M, (D + 255) // 256, 2, device=dev)
xb0, ln_st = _lib.rowstats(X)


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


for name, N, K, kind in [("qkv", 3 * D, D, "ln"), ("proj", D, D, "res"), ("fc1", 4 * D, D, "ln_gelu"),
                         ("fc2", D, 4 * D, "res")]:
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
    line = f"{name:5s} M={M} N={N} K={K}"
    for k in [0, 1, 2, 3, 4, 6, 8]:
        lib.pdm_set_gemm_tuning(0, (16 | (k << 8)) if k else 0)
        try:
            fn()
            t = timeit(fn)
        finally:
            lib.pdm_set_gemm_tuning(0, 0)
        line += f" | k={k} {t:6.1f}us"
    print(line, flush=True)

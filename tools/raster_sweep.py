"""Tile-order sweep of the persistent GEMM at the U-ViT block shapes with the forward's own epilogues (dev tool):
raster = row panels per tile group inside an XCD's range (0 = auto: 8 for N >= 2048, else row-major; 1 = row-major), median us of interleaved rounds.
Usage: python3 tools/raster_sweep.py [rows] [rasters]"""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 50
rasters = [int(r) for r in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1, 2, 4, 8, 16]
lib = _lib.load()
D, L = 1024, 258
M = rows * L
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
A = torch.randn(M, 4 * D, device=dev, generator=g).bfloat16()
Xb = torch.randn(M, D, device=dev, generator=g).bfloat16()
outb = torch.empty(M, 4 * D, device=dev, dtype=torch.bfloat16)
st_out = torch.empty(M, (D + 255) // 256, 2, device=dev)
_, ln_st = _lib.rowstats(torch.randn(M, D, device=dev, generator=g))


def timeit(fn, n=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for _ in range(200):   # clocks settle
    _lib.gemm_ex(_lib.EPI_BF16, A[:, :D], A[:3 * D, :D], None, out=outb[:, :3 * D])
torch.cuda.synchronize()
print(f"rows={rows} M={M}: us per GEMM by raster (0 = auto: 8 for N >= 2048, else row-major; 1 = row-major)")
for nm, N, K, kind in [("qkv", 3 * D, D, "ln"), ("proj", D, D, "res"), ("fc1", 4 * D, D, "ln_gelu"),
                       ("fc2", D, 4 * D, "res"), ("skip", D, 2 * D, "skip")]:
    W = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device=dev, generator=g)
    colsum = W.float().sum(1)
    if kind == "ln":
        fn = lambda: _lib.gemm_ex(_lib.EPI_BF16, A[:, :K], W, bias, out=outb[:, :N], ln_stats=ln_st, ln_colsum=colsum)
    elif kind == "ln_gelu":
        fn = lambda: _lib.gemm_ex(_lib.EPI_GELU, A[:, :K], W, bias, out=outb[:, :N], ln_stats=ln_st, ln_colsum=colsum)
    elif kind == "res":
        fn = lambda: _lib.gemm_ex(_lib.EPI_RES, A[:, :K], W, bias, out=Xb, res_in=Xb, accumulate=True, stats_out=st_out)
    else:
        fn = lambda: _lib.gemm_ex(_lib.EPI_RES, A[:, :D], W, bias, out=Xb, stats_out=st_out, a2=A[:, D:2 * D])
    t = {r: [] for r in rasters}
    for _ in range(7):
        for r in rasters:
            lib.pdm_set_gemm_tuning(r, 0)
            fn()
            torch.cuda.synchronize()
            t[r].append(timeit(fn))
    lib.pdm_set_gemm_tuning(0, 0)
    print(f"  {nm:5s} N={N:5d} K={K:5d}: " + "  ".join(f"r{r} {sorted(v)[3]:7.1f}" for r, v in t.items()), flush=True)

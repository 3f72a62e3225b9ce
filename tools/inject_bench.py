"""t2i injection GEMM shapes (dev tool): x_out = x + zeroconv(m) -- EPI_RES, N = K = 512, stats_out -- per GEMM
algorithm at the bench lane rows (32 x 334) and at 100 x 334, median us of interleaved rounds.
Usage: python3 tools/inject_bench.py"""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

lib = _lib.load()
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
D = 512


def timeit(fn, n=50):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


algos = [int(a) for a in (sys.argv[1].split(",") if len(sys.argv) > 1 else "0,1,3,5,6,7".split(","))]
for rows in (16, 32, 64, 100):
    M = rows * 334
    A = torch.randn(M, D, device=dev, generator=g).bfloat16()
    Xb = torch.randn(M, D, device=dev, generator=g).bfloat16()
    out = torch.empty_like(Xb)
    st = torch.empty(M, 2, 2, device=dev)
    W = (torch.randn(D, D, device=dev, generator=g) * D ** -0.5).bfloat16()
    bias = torch.randn(D, device=dev, generator=g)
    fn = lambda: _lib.gemm_ex(_lib.EPI_RES, A, W, bias, out=out, res_in=Xb, accumulate=True, stats_out=st)
    for _ in range(100):
        fn()
    torch.cuda.synchronize()
    t = {a: [] for a in algos}
    for _ in range(7):
        for a in algos:
            lib.pdm_set_gemm_algo(a)
            fn()
            torch.cuda.synchronize()
            t[a].append(timeit(fn))
    lib.pdm_set_gemm_algo(0)
    f = 2.0 * M * D * D
    byt = 3 * M * D * 2
    print(f"rows {rows:3d} M={M:6d}: " + "  ".join(
        f"algo {a}: {sorted(v)[3]:6.1f} us ({byt / sorted(v)[3] / 1e3:5.0f} GB/s)" for a, v in t.items()), flush=True)

# where the fixed cost of a one-tile-per-workgroup launch goes: epilogue variants and K at the bench lane rows
print("persistent kernel (algo 11), M = 32 x 334, N = 512:")
lib.pdm_set_gemm_algo(11)
M = 32 * 334
for K in (256, 512, 1024, 2048):
    A = torch.randn(M, K, device=dev, generator=g).bfloat16()
    Xb = torch.randn(M, D, device=dev, generator=g).bfloat16()
    out = torch.empty_like(Xb)
    st = torch.empty(M, 2, 2, device=dev)
    W = (torch.randn(D, K, device=dev, generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(D, device=dev, generator=g)
    variants = {"bf16": lambda: _lib.gemm_ex(_lib.EPI_BF16, A, W, bias, out=out),
                "res": lambda: _lib.gemm_ex(_lib.EPI_RES, A, W, bias, out=out, res_in=Xb, accumulate=True),
                "res+stats": lambda: _lib.gemm_ex(_lib.EPI_RES, A, W, bias, out=out, res_in=Xb, accumulate=True,
                                                  stats_out=st)}
    res = []
    for nm, fn in variants.items():
        for _ in range(50):
            fn()
        torch.cuda.synchronize()
        res.append(f"{nm}: {sorted(timeit(fn) for _ in range(5))[2]:6.1f} us")
    print(f"  K={K:5d}: " + "  ".join(res), flush=True)
lib.pdm_set_gemm_algo(0)

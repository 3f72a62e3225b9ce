"""Mainloop vs fixed-cost decomposition of the MXFP8 GEMM (gemm_mx_kernel) beside the bf16 one (gemm8d) on the
U-ViT-H/4 block shapes (dev tool): time(K) = fixed + K * slope over K in {1152 .. 4608} at fixed M x N; `slope`
gives the main-loop rate, `fixed` the per-launch prologue + epilogue + tail.
usage: python tools/gemm_mx_slope.py [rows]"""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100
M, D = rows * 258, 1152
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
KS = [1152, 2304, 3456, 4608]
A = torch.randn(M, max(KS), device=dev, generator=g)
Ab = A.bfloat16()
Aq, As = _lib.mx_quantize_gpu(A)


def timeit(fn, n=10, rounds=5):
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / n * 1e3)
    return sorted(ts)[len(ts) // 2]


def fit(ks, ts):
    n = len(ks)
    mk, mt = sum(ks) / n, sum(ts) / n
    slope = sum((k - mk) * (t - mt) for k, t in zip(ks, ts)) / sum((k - mk) ** 2 for k in ks)
    return mt - slope * mk, slope


for name, N in (("qkv", 3 * D), ("proj/fc2", D), ("fc1", 4 * D)):
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    bias = torch.randn(N, device=dev, generator=g)
    res = {"bf16": [], "mxfp8": []}
    for K in KS:
        W = torch.randn(N, K, device=dev, generator=g) * K ** -0.5
        Wb = W.bfloat16()
        Wq, Ws = _lib.mx_quantize_gpu(W)
        a_b = Ab[:, :K].contiguous()
        a_q = Aq[:, :K].contiguous()
        a_s = As[: K // 128].contiguous()
        res["bf16"].append(timeit(lambda: _lib.gemm_ex(_lib.EPI_BF16, a_b, Wb, bias, out=out)))
        res["mxfp8"].append(timeit(lambda: _lib.gemm_ex(_lib.EPI_BF16, a_q, Wq, bias, a_scale=a_s, w_scale=Ws,
                                                         out=out)))
    for kind, ts in res.items():
        fixed, slope = fit(KS, ts)
        main_pf = 2.0 * M * N / (slope * 1e-6) / 1e15
        print(f"{name:9s} N={N:5d} {kind:6s} t(K)={', '.join(f'{t:.1f}' for t in ts)} us  "
              f"main loop {main_pf:.2f} PF/s  fixed {fixed:.1f} us", flush=True)

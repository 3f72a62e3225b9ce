"""Mainloop vs fixed-cost decomposition of the default GEMM policy (dev tool): time the GEMM at fixed M x N
over several K.  time(K) = fixed + K * slope: `slope` is the mainloop cost per K (its TF/s is the mainloop
rate), `fixed` is the per-launch prologue + epilogue + tail cost.  Variants: bf16 / GELU epilogues, the
no-store timing mode (pdm_set_gemm_tuning dbg bit 1), with L2-resident operands (dbg bit 0) and the other
256-tile schedules (algos 5, 6) when a third argument is given, hipBLASLt (torch linear).
usage: python tools/gemm_slope.py [rows] [unused] [x]"""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

lib = _lib.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 190
EXTRA = len(sys.argv) > 3
M = rows * 258
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
A = torch.randn(M, 4096, device=dev, generator=g).bfloat16()
outb = torch.empty(M, 4096, device=dev, dtype=torch.bfloat16)


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
    return sorted(ts)[rounds // 2] * 1e3   # us


Ks = [512, 1024, 2048, 4096]
for N in (1024, 3072, 4096):
    res = {}
    for K in Ks:
        W = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
        bias = torch.randn(N, device=dev, generator=g)
        a = A[:, :K]
        o = outb[:, :N]
        bf = lambda: _lib.gemm_ex(_lib.EPI_BF16, a, W, bias, out=o)   # noqa: E731
        ge = lambda: _lib.gemm_ex(_lib.EPI_GELU, a, W, bias, out=o)   # noqa: E731
        r = {"bf16": timeit(bf), "gelu": timeit(ge)}
        ns = lambda: _lib.gemm_ex(_lib.EPI_BF16, a, W, bias)   # noqa: E731
        lib.pdm_set_gemm_tuning(0, 2)   # no global stores: mainloop + LDS staging only
        r["nostore"] = timeit(ns)
        if EXTRA:
            lib.pdm_set_gemm_tuning(0, 3)   # + every tile's operands from tile (0, 0): L2-resident operands
            r["nostore_l2"] = timeit(ns)
            lib.pdm_set_gemm_tuning(0, 2)
            for algo in (5, 6):
                lib.pdm_set_gemm_algo(algo)
                r[f"nostore_a{algo}"] = timeit(ns)
            lib.pdm_set_gemm_algo(0)
        lib.pdm_set_gemm_tuning(0, 0)
        ac = a.contiguous()
        r["hipblaslt"] = timeit(lambda: torch.nn.functional.linear(ac, W))
        res[K] = r
        f = 2.0 * M * N * K
        print(f"M={M} N={N} K={K}: " + " | ".join(f"{k} {v:7.1f}us {f / v / 1e6:5.0f}TF" for k, v in r.items()),
              flush=True)
    k0, k1 = Ks[1], Ks[-1]
    for nm in res[k0]:
        slope = (res[k1][nm] - res[k0][nm]) / (k1 - k0)
        fixed = res[k0][nm] - slope * k0
        print(f"  N={N} {nm:12s}: mainloop {2.0 * M * N / slope / 1e6:6.0f} TF/s, fixed {fixed:7.1f} us per launch",
              flush=True)

"""N = 128 GEMM vs conv under each tile policy (dev tool): separates the conv tap-addressing cost from the tile
shape.  python tools/tall_probe.py"""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

lib = _lib.load()
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)


def timeit(fn, n=5, rounds=3):
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


M, K = 8 * 512 * 512, 1152
a = torch.randn(M, K, device=dev, generator=g).bfloat16()
x = torch.randn(8, 512, 512, 128, device=dev, generator=g).bfloat16()
for N in (128, 256):
    w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
    wc = w.view(N, 3, 3, 128).permute(0, 3, 1, 2).contiguous()
    bias = torch.randn(N, device=dev, generator=g)
    ob = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    flops = 2.0 * M * N * K
    for name, fn in (("gemm", lambda: _lib.gemm(a, w, bias, _lib.EPI_BF16, out=ob)),
                     ("conv", lambda: _lib.gemm_conv3x3(x, wc, bias, _lib.EPI_BF16, out=ob))):
        line = f"N={N} {name}"
        for algo in (1, 7, 9):
            lib.pdm_set_gemm_algo(algo)
            try:
                fn()
                t = timeit(fn)
            finally:
                lib.pdm_set_gemm_algo(0)
            line += f" | a{algo} {t:7.1f}us {flops / t / 1e6:5.0f}TF"
        print(line, flush=True)

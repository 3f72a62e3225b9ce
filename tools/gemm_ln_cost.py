"""Cost of the fused-LayerNorm consumer and of the bias in the 256-tile GEMM epilogue (dev tool): the qkv and
fc1 shapes of the L/2 bench (rows 190) timed plain, with bias, and with bias + LN operands, interleaved rounds.
usage: python tools/gemm_ln_cost.py [rows]"""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 190
M, D = rows * 258, 1024
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
A = torch.randn(M, D, device=dev, generator=g).bfloat16()
st = torch.rand(M, D // 256, 2, device=dev, generator=g) + 1.0
for name, N, epi in (("qkv", 3 * D, _lib.EPI_BF16), ("fc1", 4 * D, _lib.EPI_GELU)):
    W = (torch.randn(N, D, device=dev, generator=g) * D ** -0.5).bfloat16()
    bias = torch.randn(N, device=dev, generator=g)
    colsum = torch.randn(N, device=dev, generator=g)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    variants = {
        "plain": lambda: _lib.gemm(A, W, None, epi, out=out),
        "bias": lambda: _lib.gemm(A, W, bias, epi, out=out),
        "bias+ln": lambda: _lib.gemm_ln(A, W, bias, epi, ln_stats=st, ln_colsum=colsum, out=out),
    }
    times = {k: [] for k in variants}
    for rnd in range(5):
        for k, f in variants.items():
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / 10 * 1e3)
    fl = 2.0 * M * N * D
    print(name, " | ".join(f"{k} {sorted(v)[2]:7.1f} us ({fl / sorted(v)[2] / 1e6:6.1f} TF/s)" for k, v in times.items()))

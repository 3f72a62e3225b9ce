"""Tile-order / memory-bound experiments on the 256-tile GEMM (dev tool, one process, interleaved rounds).
python tools/gemm_tune.py ALGO [raster list] -- prints TF/s per (shape, raster, dbg_tile0)."""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

lib = _lib.load()
algo = int(sys.argv[1]) if len(sys.argv) > 1 else 7
rasters = [int(r) for r in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 2, 4, 8]
assert lib.pdm_set_gemm_algo(algo) == 0, lib.pdm_last_error()
M = 49020
shapes = [("qkv", 3072, 1024, _lib.EPI_BF16), ("fc1", 4096, 1024, _lib.EPI_GELU), ("fc2", 1024, 4096, _lib.EPI_F32),
          ("big", 4096, 4096, _lib.EPI_BF16)]
g = torch.Generator(device="cuda").manual_seed(0)
A = torch.randn(M, 4096, device="cuda", generator=g).bfloat16()
res = torch.zeros(M, 1024, device="cuda")
outb = torch.empty(M, 4096, device="cuda", dtype=torch.bfloat16)
variants = [(r, 0) for r in rasters] + [(0, 1), (4, 1)]
for name, N, K, epi in shapes:
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    a = A[:, :K]
    times = {v: [] for v in variants}
    for rnd in range(5):
        for v in variants:
            assert lib.pdm_set_gemm_tuning(*v) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                if epi == _lib.EPI_F32:
                    _lib.gemm(a, W, bias, epi, out_f32=res, accumulate=False)
                else:
                    _lib.gemm(a, W, bias, epi, out=outb[:, :N])
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / 10)
    f = 2.0 * M * N * K
    line = f"{name:4s} N={N} K={K}"
    for v in variants:
        t = sorted(times[v])[2]
        line += f" | r{v[0]}{'D' if v[1] else ''} {f / t / 1e9:7.1f}"
    print(line, flush=True)
lib.pdm_set_gemm_tuning(0, 0)

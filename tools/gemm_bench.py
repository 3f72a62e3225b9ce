"""A/B timing of the GEMM tile policies on the U-ViT shapes (dev tool, one process, interleaved rounds)."""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

lib = _lib.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 128
D = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
ALGOS = [int(a) for a in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 2]
L = 258
M = rows * L
shapes = [("qkv", 3 * D, D, _lib.EPI_BF16), ("proj", D, D, _lib.EPI_F32), ("fc1", 4 * D, D, _lib.EPI_GELU),
          ("fc2", D, 4 * D, _lib.EPI_F32), ("skip", D, 2 * D, _lib.EPI_F32)]
g = torch.Generator(device="cuda").manual_seed(0)
A = torch.randn(M, 4 * D, device="cuda", generator=g).bfloat16()
res = torch.zeros(M, D, device="cuda")
outb = torch.empty(M, 4 * D, device="cuda", dtype=torch.bfloat16)
tot = {a: 0.0 for a in ALGOS}
flops = 0
for name, N, K, epi in shapes:
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    a = A[:, :K].contiguous()
    outs = {}
    for algo in ALGOS:
        assert lib.pdm_set_gemm_algo(algo) == 0, lib.pdm_last_error()
        o = _lib.gemm(a, W, bias, epi, out=None if epi != _lib.EPI_F32 else None)
        outs[algo] = o.float()
    err = max(float((outs[ALGOS[0]] - outs[x]).norm() / outs[ALGOS[0]].norm()) for x in ALGOS)
    times = {a: [] for a in ALGOS}
    for rnd in range(5):
        for algo in ALGOS:
            assert lib.pdm_set_gemm_algo(algo) == 0, lib.pdm_last_error()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                if epi == _lib.EPI_F32:
                    _lib.gemm(a, W, bias, epi, out_f32=res[:, :N] if N == D else None, accumulate=False)
                else:
                    _lib.gemm(a, W, bias, epi, out=outb[:, :N] if N == 4 * D else None)
            e1.record()
            torch.cuda.synchronize()
            times[algo].append(e0.elapsed_time(e1) / 10)
    # vendor reference point: hipBLASLt via torch (bf16 out, bias, no fused epilogue)
    bl = []
    for rnd in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        bb = bias.bfloat16()
        e0.record()
        for _ in range(10):
            torch.nn.functional.linear(a, W, bb)
        e1.record()
        torch.cuda.synchronize()
        bl.append(e0.elapsed_time(e1) / 10)
    f = 2.0 * M * N * K
    flops += f
    tbl = sorted(bl)[2]
    tot["blas"] = tot.get("blas", 0.0) + tbl
    line = f"{name:5s} M={M} N={N} K={K} maxrelerr={err:.1e}"
    for algo in ALGOS:
        t = sorted(times[algo])[len(times[algo]) // 2]
        tot[algo] += t
        line += f" | algo{algo} {t*1e3:8.1f} us {f/t/1e9:7.1f} TF/s"
    line += f" | hipblaslt {tbl*1e3:8.1f} us {f/tbl/1e9:7.1f} TF/s"
    print(line)
print(f"hipblaslt: block GEMMs {tot['blas']:.3f} ms -> {flops/tot['blas']/1e9:.1f} TF/s")
for algo in ALGOS:
    print(f"algo{algo}: block GEMMs {tot[algo]:.3f} ms -> {flops/tot[algo]/1e9:.1f} TF/s")
lib.pdm_set_gemm_algo(0)

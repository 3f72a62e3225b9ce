"""bf16 vs MXFP8 GEMM timing on the U-ViT-H block shapes (dev tool, one process, interleaved rounds).
python tools/gemm_fp8_bench.py [rows]"""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

lib = _lib.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100
M, D = rows * 258, 1152
g = torch.Generator(device="cuda").manual_seed(0)
shapes = [("qkv", 3 * D, D, _lib.EPI_BF16), ("fc1", 4 * D, D, _lib.EPI_GELU), ("fc2", D, 4 * D, _lib.EPI_F32)]
tot = {"bf16": 0.0, "fp8": 0.0}
flops = 0.0
for name, N, K, epi in shapes:
    a = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) * K ** -0.5
    bias = torch.randn(N, device="cuda", generator=g)
    ab, wb = a.bfloat16(), w.bfloat16()
    qa, sa = _lib.mx_quantize(a)
    qw, sw = _lib.mx_quantize(w)
    outb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    outf = torch.zeros(M, N, device="cuda")

    def run(kind):
        if kind == "bf16":
            if epi == _lib.EPI_F32:
                _lib.gemm_ex(epi, ab, wb, bias, out_f32=outf)
            else:
                _lib.gemm_ex(epi, ab, wb, bias, out=outb)
        else:
            if epi == _lib.EPI_F32:
                _lib.gemm_ex(epi, qa, qw, bias, sa, sw, out_f32=outf)
            else:
                _lib.gemm_ex(epi, qa, qw, bias, sa, sw, out=outb)
    times = {"bf16": [], "fp8": []}
    for rnd in range(5):
        for kind in ("bf16", "fp8"):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run(kind)
            e1.record()
            torch.cuda.synchronize()
            times[kind].append(e0.elapsed_time(e1) / 10)
    f = 2.0 * M * N * K
    flops += f
    line = f"{name:4s} M={M} N={N} K={K}"
    for kind in ("bf16", "fp8"):
        t = sorted(times[kind])[2]
        tot[kind] += t
        line += f" | {kind} {t * 1e3:8.1f} us {f / t / 1e9:7.1f} TF/s"
    print(line, flush=True)
for kind in ("bf16", "fp8"):
    print(f"{kind}: {tot[kind]:.3f} ms -> {flops / tot[kind] / 1e9:.1f} TF/s")

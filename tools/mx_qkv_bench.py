"""The U-ViT-H/4 fp8 qkv GEMM (centred-LN MXFP8 operand, N = 3456, K = 1152, bf16 out) per GEMM kernel: algo 7
(gemm_mx_kernel, one tile per workgroup) vs algo 11 (persistent gemm8s_kernel FP8), GPU time of graph replays,
interleaved rounds (dev tool).  Usage: python3 tools/mx_qkv_bench.py [rows,...]"""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402
from panopticdiffusionmodels_amd.native import gcol_table  # noqa: E402

lib = _lib.load()
N, K = 3456, 1152
for rows in [int(r) for r in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["50", "100"])]:
    M = rows * 258
    g = torch.Generator(device="cuda").manual_seed(rows)
    x = torch.randn(M, K, device="cuda", generator=g) * 1.5 + 3.0
    w = torch.randn(N, K, device="cuda", generator=g) * K ** -0.5
    bias = torch.randn(N, device="cuda", generator=g)
    qw, sw = _lib.mx_quantize(w)
    dw = _lib.mx_dequantize(qw, sw)
    _, st = _lib.rowstats(x, want_bf16=False)
    qx, sx = _lib.mx_quantize_centred(x, st)
    kw = dict(ln_stats=st, ln_colsum=dw.double().sum(1).float(), ln_gcol=gcol_table(dw))
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    graphs = {}
    for algo in (7, 11):
        lib.pdm_set_gemm_algo(algo)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            _lib.gemm_ex(_lib.EPI_BF16, qx, qw, bias, sx, sw, out=out, **kw)
        torch.cuda.current_stream().wait_stream(s)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(10):
                _lib.gemm_ex(_lib.EPI_BF16, qx, qw, bias, sx, sw, out=out, **kw)
        graphs[algo] = gr
    lib.pdm_set_gemm_algo(0)
    t = {a: [] for a in graphs}
    for _ in range(9):
        for a, gr in graphs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            gr.replay()
            e1.record()
            torch.cuda.synchronize()
            t[a].append(e0.elapsed_time(e1) / 10 * 1e3)
    fl = 2.0 * M * N * K
    print(f"rows {rows} M={M}: " + "  ".join(f"algo {a}: {sorted(v)[4]:6.1f} us ({fl / sorted(v)[4] / 1e6:5.0f} TF/s)"
                                             for a, v in t.items()), flush=True)

"""The U-ViT-H/4 fp8 proj GEMM (MXFP8 attention-output operand, N = K = 1152, bf16 residual in place + LayerNorm
partials) per GEMM kernel: algo 7 (gemm_mx_kernel<EPI_RES>, one tile per workgroup) vs algo 0 (automatic: the
persistent gemm8s_kernel<EPI_RES, 0, 0, 1>), GPU time of graph replays, interleaved rounds, plus the bit-identity of
the two outputs (dev tool).  Usage: python3 tools/mx_res_bench.py [rows,...] [N,K]"""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

lib = _lib.load()
N, K = (int(v) for v in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["1152", "1152"]))
for rows in [int(r) for r in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["50", "100"])]:
    M = rows * 258
    g = torch.Generator(device="cuda").manual_seed(rows)
    a = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) * K ** -0.5
    bias = torch.randn(N, device="cuda", generator=g)
    res0 = (torch.randn(M, N, device="cuda", generator=g) * 3 + 2).bfloat16()
    qa, sa = _lib.mx_quantize(a)
    qw, sw = _lib.mx_quantize(w)
    outs, graphs = {}, {}
    for algo in (7, 0):
        lib.pdm_set_gemm_algo(algo)
        out = res0.clone()
        st = torch.empty(M, (N + 255) // 256, 2, device="cuda")
        _lib.gemm_ex(_lib.EPI_RES, qa, qw, bias, sa, sw, out=out, res_in=out, accumulate=True, stats_out=st)
        torch.cuda.synchronize()
        outs[algo] = (out.clone(), st.clone())
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            _lib.gemm_ex(_lib.EPI_RES, qa, qw, bias, sa, sw, out=out, res_in=out, accumulate=True, stats_out=st)
        torch.cuda.current_stream().wait_stream(s)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(10):
                _lib.gemm_ex(_lib.EPI_RES, qa, qw, bias, sa, sw, out=out, res_in=out, accumulate=True, stats_out=st)
        graphs[algo] = gr
    lib.pdm_set_gemm_algo(0)
    same = torch.equal(outs[7][0], outs[0][0])
    dst = float((outs[7][1] - outs[0][1]).norm() / outs[7][1].norm())
    t = {a_: [] for a_ in graphs}
    for _ in range(9):
        for a_, gr in graphs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            gr.replay()
            e1.record()
            torch.cuda.synchronize()
            t[a_].append(e0.elapsed_time(e1) / 10 * 1e3)
    fl = 2.0 * M * N * K
    print(f"rows {rows} M={M} N={N} K={K}: output bit-identical {same}, partials rel {dst:.1e} | " +
          "  ".join(f"algo {a_}: {sorted(v)[4]:6.1f} us ({fl / sorted(v)[4] / 1e6:5.0f} TF/s)" for a_, v in t.items()),
          flush=True)

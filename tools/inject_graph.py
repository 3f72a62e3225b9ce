"""t2i injection GEMM (x_out = x + zeroconv(m[:, :Lx]), EPI_RES, N = K = 512, row gather, partials, second output)
timed as GPU time: 20 launches captured in a HIP graph and replayed (the Python launch cost of tools/inject_bench.py
dominates its numbers).  Variants: GEMM algo, with / without the gather and the second output.  Dev tool.
Usage: python3 tools/inject_graph.py [rows,...] [algos]"""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

lib = _lib.load()
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
D, Lx, Lm = 512, 334, 590
rows_list = [int(r) for r in sys.argv[1].split(",")] if len(sys.argv) > 1 else [32, 64]
algos = [int(a) for a in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1, 7]


def graph_time(fn, n=20, reps=7):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(n):
            fn()
    gr.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gr.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / n * 1e3)
    return sorted(ts)[reps // 2]


for rows in rows_list:
    M = rows * Lx
    mout = torch.randn(rows * Lm, D, device=dev, generator=g).bfloat16()
    A = mout.view(rows, Lm, D)[:, :Lx].contiguous().view(M, D)
    Xb = torch.randn(M, D, device=dev, generator=g).bfloat16()
    out = torch.empty_like(Xb)
    st = torch.empty(M, 2, 2, device=dev)
    MB = torch.empty(rows * Lm, D, device=dev, dtype=torch.bfloat16)
    STM = torch.empty(rows * Lm, 2, 2, device=dev)
    W = (torch.randn(D, D, device=dev, generator=g) * D ** -0.5).bfloat16()
    bias = torch.randn(D, device=dev, generator=g)
    variants = {
        "full": lambda: _lib.gemm_ex(_lib.EPI_RES, mout, W, bias, out=out, res_in=Xb, accumulate=True, stats_out=st,
                                     a_gather=(M, Lx, Lm), out2=MB, out2_gather=(Lx, Lm), stats_out2=STM),
        "no-out2": lambda: _lib.gemm_ex(_lib.EPI_RES, mout, W, bias, out=out, res_in=Xb, accumulate=True, stats_out=st,
                                        a_gather=(M, Lx, Lm)),
        "plain-res": lambda: _lib.gemm_ex(_lib.EPI_RES, A, W, bias, out=out, res_in=Xb, accumulate=True, stats_out=st),
        "bf16": lambda: _lib.gemm_ex(_lib.EPI_BF16, A, W, bias, out=out),
    }
    for a in algos:
        lib.pdm_set_gemm_algo(a)
        res = []
        for nm, fn in variants.items():
            try:
                res.append(f"{nm} {graph_time(fn):6.1f}")
            except RuntimeError as e:
                res.append(f"{nm} n/a")
        print(f"rows {rows:3d} M={M:6d} algo {a:2d}: " + "  ".join(res) + "  (us per launch)", flush=True)
    lib.pdm_set_gemm_algo(0)
    byt = 4 * M * D * 2
    print(f"  HBM floor (A, residual, out, out2 = {byt / 1e6:.1f} MB at 5 TB/s): {byt / 5e12 * 1e6:.1f} us", flush=True)

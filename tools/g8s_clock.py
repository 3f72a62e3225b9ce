"""In-kernel clock of the persistent GEMM (dev tool; needs a -DPDM_G8S_CLK build, tools/build_variant.sh): per shape
and variant, the wall time per launch and the shader clock the workgroups ran at (summed s_memtime / s_memrealtime
deltas x 100 MHz), so a slowdown splits into cycles and clock.
  PDM_LIB_PATH=ab/libpdm_clk.so python tools/g8s_clock.py [rows]"""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

lib = _lib.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100
D, L = 1024, 258
M = rows * L
g = torch.Generator(device="cuda").manual_seed(0)
A = torch.randn(M, 4 * D, device="cuda", generator=g).bfloat16()
X = torch.randn(M, D, device="cuda", generator=g)
Xb = X.bfloat16()
outb = torch.empty(M, 4 * D, device="cuda", dtype=torch.bfloat16)
st_out = torch.empty(M, (D + 255) // 256, 2, device="cuda")
_, ln_st = _lib.rowstats(X)
buf = (ctypes.c_ulonglong * 3)()


def stats():
    assert lib.pdm_gemm_sk_stats(buf) == 0
    return buf[0], buf[1], buf[2]


_w = (torch.randn(3 * D, D, device="cuda", generator=g) * D ** -0.5).bfloat16()
for _ in range(200):   # clocks / caches settle
    _lib.gemm_ex(_lib.EPI_BF16, A[:, :D], _w, None, out=outb[:, :3 * D])
torch.cuda.synchronize()
for name, N, K, kind in [("qkv", 3 * D, D, "ln"), ("proj", D, D, "res"), ("fc2", D, 4 * D, "res")]:
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    colsum = torch.randn(N, device="cuda", generator=g)
    a, o = A[:, :K], outb[:, :N]
    if kind == "ln":
        fn = lambda: _lib.gemm_ex(_lib.EPI_BF16, a, W, bias, out=o, ln_stats=ln_st, ln_colsum=colsum)
    else:
        fn = lambda: _lib.gemm_ex(_lib.EPI_RES, a, W, bias, out=Xb, res_in=Xb, accumulate=True, stats_out=st_out)
    line = f"{name:5s} M={M} N={N} K={K}"
    for vn, bit in (("fwd", 0), ("noepi", 16)) + ((("dropst", 32), ("dropres", 64), ("dropboth", 96)) if kind == "res"
                                                  else (("dropst", 32),)):
        lib.pdm_set_gemm_tuning(0, bit)
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        stats()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        lib.pdm_set_gemm_tuning(0, 0)
        t = e0.elapsed_time(e1) / n * 1e3
        tk, rt, nwg = stats()
        clk = tk / rt * 0.1 if rt else float("nan")   # GHz
        line += f" | {vn} {t:6.1f}us clk {clk:4.2f}GHz ({nwg // n} wg) {t * clk:7.0f}kcyc"
    print(line, flush=True)

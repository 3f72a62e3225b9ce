"""Stream-K diagnostics (dev tool): per L/2 block GEMM at a row count, whole tiles vs stream-K vs stream-K with the
slab traffic dropped (pdm_set_gemm_tuning bit 9, timing only), plus the hand-off statistics of one stream-K launch
(bit 8: tails, hand-offs not taken, mean poll time)."""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100
D = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
L = 258
lib = _lib.load()
M = rows * L
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
A = torch.randn(M, 4 * D, device=dev, generator=g).bfloat16()
Xb = torch.randn(M, D, device=dev, generator=g).bfloat16()
outb = torch.empty(M, 4 * D, device=dev, dtype=torch.bfloat16)
st_out = torch.empty(M, (D + 255) // 256, 2, device=dev)
_, ln_st = _lib.rowstats(torch.randn(M, D, device=dev, generator=g))


def timeit(fn, n=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def setm(sk, dbg):
    lib.pdm_set_gemm_sk(sk)
    lib.pdm_set_gemm_tuning(0, dbg)


for _ in range(200):
    _lib.gemm_ex(_lib.EPI_BF16, A[:, :D], A[:3 * D, :D], None, out=outb[:, :3 * D])
torch.cuda.synchronize()
variants = [("whole", 0, 0), ("sk", 6, 0), ("sk_noslab", 6, 512), ("sk_recompute", 6, 128)]
for nm, N, K, kind in [("qkv", 3 * D, D, "ln"), ("proj", D, D, "res"), ("fc1", 4 * D, D, "gelu"),
                       ("fc2", D, 4 * D, "res"), ("skip", D, 2 * D, "skip")]:
    W = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device=dev, generator=g)
    colsum = W.float().sum(1)
    if kind == "ln":
        fn = lambda: _lib.gemm_ex(_lib.EPI_BF16, A[:, :K], W, bias, out=outb[:, :N], ln_stats=ln_st, ln_colsum=colsum)
    elif kind == "gelu":
        fn = lambda: _lib.gemm_ex(_lib.EPI_GELU, A[:, :K], W, bias, out=outb[:, :N], ln_stats=ln_st, ln_colsum=colsum)
    elif kind == "res":
        fn = lambda: _lib.gemm_ex(_lib.EPI_RES, A[:, :K], W, bias, out=Xb, res_in=Xb, accumulate=True, stats_out=st_out)
    else:
        fn = lambda: _lib.gemm_ex(_lib.EPI_RES, A[:, :D], W, bias, out=Xb, stats_out=st_out, a2=A[:, D:2 * D])
    t = {v[0]: [] for v in variants}
    for _ in range(5):
        for vn, sk, dbg in variants:
            setm(sk, dbg)
            fn()
            t[vn].append(timeit(fn))
    setm(6, 256)
    st = (ctypes.c_ulonglong * 3)()
    lib.pdm_gemm_sk_stats(st)   # clear
    fn()
    lib.pdm_gemm_sk_stats(st)
    setm(0, 0)
    med = {k: sorted(v)[2] for k, v in t.items()}
    tails, miss, ticks = st[0], st[1], st[2]
    print(f"{nm:5s} N={N} K={K}: " + "  ".join(f"{k} {v:7.1f}" for k, v in med.items()) +
          f"  | tails {tails} not-taken {miss} mean poll {ticks * 10 / max(tails, 1):.0f} ns", flush=True)

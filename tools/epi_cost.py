"""Epilogue cost decomposition of the U-ViT block GEMMs (dev tool): for each shape, time the mainloop alone
(bf16 epilogue with no output pointer: accumulators staged, nothing stored), the plain bf16 / fp32 stores, and
the exact in-forward epilogue (fused LN operands, GELU, fp32 residual accumulate + bf16 copy + LN partials)."""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

lib = _lib.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 190
D = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
ALGO = int(sys.argv[3]) if len(sys.argv) > 3 else 0   # GEMM tile policy (pdm_set_gemm_algo; 0 = automatic)
lib.pdm_set_gemm_algo(ALGO)
L = 258
M = rows * L
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
A = torch.randn(M, 4 * D, device=dev, generator=g).bfloat16()
X = torch.randn(M, D, device=dev, generator=g)
Xb = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
outb = torch.empty(M, 4 * D, device=dev, dtype=torch.bfloat16)
st_out = torch.empty(M, (D + 255) // 256, 2, device=dev)
xb0, ln_st = _lib.rowstats(X)


def timeit(fn, n=10, rounds=5):
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / n)
    return sorted(ts)[rounds // 2] * 1e3   # us


# clocks / caches settle before the first measured shape (the first variants otherwise read 5-20 % slow)
_w = torch.randn(3 * D, D, device=dev, generator=g).bfloat16()
for _ in range(400):
    _lib.gemm_ex(_lib.EPI_BF16, A[:, :D], _w, None, out=outb[:, :3 * D])
torch.cuda.synchronize()

shapes = [("qkv", 3 * D, D, "ln"), ("proj", D, D, "res"), ("fc1", 4 * D, D, "ln_gelu"), ("fc2", D, 4 * D, "res"),
          ("skip", D, 2 * D, "res")]
for name, N, K, kind in shapes:
    W = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device=dev, generator=g)
    colsum = torch.randn(N, device=dev, generator=g)
    a = A[:, :K]
    o = outb[:, :N]
    f = 2.0 * M * N * K
    variants = {
        "bf16": lambda: _lib.gemm_ex(_lib.EPI_BF16, a, W, bias, out=o),
        "gelu": lambda: _lib.gemm_ex(_lib.EPI_GELU, a, W, bias, out=o),
    }
    if kind.startswith("ln"):
        variants["ln_bf16"] = lambda: _lib.gemm_ex(_lib.EPI_BF16, a, W, bias, out=o, ln_stats=ln_st, ln_colsum=colsum)
    if kind == "ln_gelu":
        variants["ln_gelu"] = lambda: _lib.gemm_ex(_lib.EPI_GELU, a, W, bias, out=o, ln_stats=ln_st, ln_colsum=colsum)
    if kind == "res":
        variants["f32"] = lambda: _lib.gemm_ex(_lib.EPI_F32, a, W, bias, out_f32=X)
        variants["f32_acc"] = lambda: _lib.gemm_ex(_lib.EPI_F32, a, W, bias, out_f32=X, accumulate=True)
        variants["f32_acc_b_st"] = lambda: _lib.gemm_ex(_lib.EPI_F32, a, W, bias, out_f32=X, accumulate=True, out=Xb,
                                                        stats_out=st_out)
        # the bf16 residual stream (EPI_RES): write only / read + write / + LayerNorm partials (the forward's form)
        variants["res"] = lambda: _lib.gemm_ex(_lib.EPI_RES, a, W, bias, out=Xb)
        variants["res_acc"] = lambda: _lib.gemm_ex(_lib.EPI_RES, a, W, bias, out=Xb, res_in=Xb, accumulate=True)
        variants["res_acc_st"] = lambda: _lib.gemm_ex(_lib.EPI_RES, a, W, bias, out=Xb, res_in=Xb, accumulate=True,
                                                      stats_out=st_out)
    def tuned(dbg, fn):
        def run():
            lib.pdm_set_gemm_tuning(0, dbg)
            try:
                fn()
            finally:
                lib.pdm_set_gemm_tuning(0, 0)
        return run
    if ALGO == 11:   # the persistent kernel's timing bits: 16 no epilogue, 32 stores dropped, 64 residual loads dropped
        fwd = {"qkv": "ln_bf16", "proj": "res_acc_st", "fc1": "ln_gelu", "fc2": "res_acc_st", "skip": "res_acc_st"}[name]
        for nm, bit in (("noepi", 16), ("dropst", 32), ("dropres", 64), ("dropboth", 96)):
            variants[fwd + "_" + nm] = tuned(bit, variants[fwd])
    variants["nostore"] = tuned(2, lambda: _lib.gemm_ex(_lib.EPI_BF16, a, W, bias))
    variants["halfstore"] = tuned(4, lambda: _lib.gemm_ex(_lib.EPI_BF16, a, W, bias, out=o))
    # every row tile stores onto rows 0..255 (an L2-resident 256 x N output): the store cost without HBM write-back
    variants["l2store"] = tuned(8, lambda: _lib.gemm_ex(_lib.EPI_BF16, a, W, bias, out=o))
    variants["hipblaslt"] = lambda: torch.nn.functional.linear(a, W)
    line = f"{name:5s} M={M} N={N} K={K}"
    for k, fn in variants.items():
        fn()
        t = timeit(fn)
        line += f" | {k} {t:7.1f}us {f / t / 1e6:6.0f}TF"
    print(line, flush=True)

"""Stream-K A/B (dev tool): every U-ViT block GEMM of a config at a row count, whole tiles (pdm_set_gemm_sk 0) vs
stream-K (auto policy, standalone state), interleaved rounds, median us; then the whole forward both ways.
Usage: python3 tools/sk_bench.py [config] [rows] [mode_on]"""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib, configs, weights  # noqa: E402
from panopticdiffusionmodels_amd.utils import get_nnet  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "imagenet256_uvit_large"
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 100
mode_on = int(sys.argv[3]) if len(sys.argv) > 3 else 1
lib = _lib.load()
cfg = configs.nnet_kwargs(name)
D = cfg["embed_dim"]
L = (cfg["img_size"] // cfg["patch_size"]) ** 2 + (2 if cfg.get("num_classes", -1) > 0 else 1)
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


def ab(fn, rounds=7):
    t = {0: [], 1: []}
    for _ in range(rounds):
        for m in (0, 1):
            lib.pdm_set_gemm_sk(mode_on | 4 if m else 0)
            fn()
            torch.cuda.synchronize()
            t[m].append(timeit(fn))
    lib.pdm_set_gemm_sk(0)
    return [sorted(v)[rounds // 2] for v in (t[0], t[1])]


for _ in range(200):   # clocks settle
    _lib.gemm_ex(_lib.EPI_BF16, A[:, :D], A[:3 * D, :D], None, out=outb[:, :3 * D])
torch.cuda.synchronize()
shapes = [("qkv", 3 * D, D, "ln"), ("proj", D, D, "res"), ("fc1", 4 * D, D, "ln_gelu"), ("fc2", D, 4 * D, "res"),
          ("skip", D, 2 * D, "skip")]
print(f"{name} rows={rows} M={M}: whole-tile vs stream-K (mode {mode_on}) us, median of interleaved rounds")
for nm, N, K, kind in shapes:
    W = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device=dev, generator=g)
    colsum = W.float().sum(1)
    if kind == "ln":
        fn = lambda: _lib.gemm_ex(_lib.EPI_BF16, A[:, :K], W, bias, out=outb[:, :N], ln_stats=ln_st, ln_colsum=colsum)
    elif kind == "ln_gelu":
        fn = lambda: _lib.gemm_ex(_lib.EPI_GELU, A[:, :K], W, bias, out=outb[:, :N], ln_stats=ln_st, ln_colsum=colsum)
    elif kind == "res":
        fn = lambda: _lib.gemm_ex(_lib.EPI_RES, A[:, :K], W, bias, out=Xb, res_in=Xb, accumulate=True, stats_out=st_out)
    else:
        fn = lambda: _lib.gemm_ex(_lib.EPI_RES, A[:, :D], W, bias, out=Xb, stats_out=st_out, a2=A[:, D:2 * D])
    t0, t1 = ab(fn)
    f = 2.0 * M * N * K
    print(f"  {nm:5s} N={N:5d} K={K:5d}: {t0:8.1f} -> {t1:8.1f} us  ({f / t0 / 1e6:7.0f} -> {f / t1 / 1e6:7.0f} TF/s)")

net = get_nnet(**cfg).to(dev)
net.load_state_dict(weights.nnet_state_dict(cfg, seed=0, device=dev))
zs = configs.get_config(name)["z_shape"]
x = torch.randn(rows, *zs, device=dev)
t = torch.rand(rows, device=dev) * 999
extra = (torch.randint(0, 1000, (rows,), device=dev) if cfg.get("num_classes", -1) > 0 else None,)
with torch.no_grad():
    tt = {0: [], 1: []}
    for _ in range(5):
        for m in (0, 1):
            lib.pdm_set_gemm_sk(mode_on if m else 0)
            net.forward_pre(x, t, *extra)
            tt[m].append(timeit(lambda: net.forward_pre(x, t, *extra), n=5))
    lib.pdm_set_gemm_sk(0)
print(f"  forward: {sorted(tt[0])[2] / 1e3:.2f} -> {sorted(tt[1])[2] / 1e3:.2f} ms")

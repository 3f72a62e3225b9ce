"""Diagnostic (dev tool): where algo 11 (persistent GEMM) differs from algo 7 on the LN-consumer / bf16 / residual
epilogues -- mismatch counts by tile-local column and row."""
import sys
import torch
sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib as lib  # noqa: E402

L = lib.load()
M, N, K = 4133, 1024, 1024
g = torch.Generator(device="cuda").manual_seed(1)
x = torch.randn(M, K, device="cuda", generator=g) * 1.5 + 3.0
w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
b = torch.randn(N, device="cuda", generator=g)
colsum = w.double().sum(1).float()
xb, st = lib.rowstats(x)
for kind in ("ln", "plain"):
    outs = {}
    for algo in (7, 11):
        L.pdm_set_gemm_algo(algo)
        if kind == "ln":
            outs[algo] = lib.gemm_ln(xb, w, b, lib.EPI_BF16, ln_stats=st, ln_colsum=colsum).float()
        else:
            outs[algo] = lib.gemm(xb, w, b, lib.EPI_BF16).float()
    L.pdm_set_gemm_algo(0)
    torch.cuda.synchronize()
    bad = ~torch.isclose(outs[7], outs[11], rtol=0, atol=0, equal_nan=True)
    print(kind, "mismatches", int(bad.sum()), "of", bad.numel())
    if bad.any():
        cols = bad.sum(0).view(-1, 256).sum(0)   # per local column
        rows = bad[: (M // 256) * 256].view(-1, 256, N).sum(0).sum(1)
        print(" local cols with mismatches:", torch.nonzero(cols).flatten().tolist()[:80])
        print(" local rows with mismatches:", torch.nonzero(rows).flatten().tolist()[:80])
        print(" col tiles:", bad.view(M, -1, 256).sum((0, 2)).tolist())
        t0 = bad[:256, :256].float()
        print(" tile(0,0) mismatch fraction by 8-col group:", [round(float(v), 2) for v in t0.view(256, 32, 8).mean((0, 2))])
        print(" tile(0,0) mismatch fraction by 16-row group:", [round(float(v), 2) for v in t0.view(16, 16, 256).mean((1, 2))])
        d = (outs[11] - outs[7])[:256, :256]
        rr = outs[11][:256, :256] / outs[7][:256, :256]
        print(" ratio sample row 0 cols 32..40:", [round(float(v), 3) for v in rr[0, 32:40]])
        r, c = torch.nonzero(bad)[0].tolist()
        print(" first", r, c, outs[7][r, c].item(), outs[11][r, c].item())

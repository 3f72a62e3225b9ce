"""Run one GEMM shape repeatedly (profiling target): python tools/gemm_one.py ALGO M N K EPI [ITERS]
(env PDM_RASTER: tile-order raster, pdm_set_gemm_tuning; 1 = row-major; PDM_DBG: its timing bits, e.g. 16 = no epilogue)"""
import os
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

algo, M, N, K, epi = (int(v) for v in sys.argv[1:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 20
lib = _lib.load()
assert lib.pdm_set_gemm_algo(algo) == 0, lib.pdm_last_error()
if os.environ.get("PDM_RASTER") or os.environ.get("PDM_DBG"):
    assert lib.pdm_set_gemm_tuning(int(os.environ.get("PDM_RASTER", "0")), int(os.environ.get("PDM_DBG", "0"))) == 0, \
        lib.pdm_last_error()
g = torch.Generator(device="cuda").manual_seed(0)
a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
b = torch.randn(N, device="cuda", generator=g)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
of = torch.zeros(M, N, device="cuda")
for _ in range(iters):
    if epi == 2:
        _lib.gemm(a, w, b, epi, out_f32=of, accumulate=True)
    else:
        _lib.gemm(a, w, b, epi, out=out)
torch.cuda.synchronize()
print("done")

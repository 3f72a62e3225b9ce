"""Run one attention structure repeatedly (profiling target): python tools/attn_one.py ALGO [rows L H Dh ITERS]"""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

algo = int(sys.argv[1])
rows, L, H, Dh, iters = (int(v) for v in (sys.argv[2:7] if len(sys.argv) > 6 else (190, 258, 16, 64, 10)))
lib = _lib.load()
assert lib.pdm_set_attention_algo(algo) == 0, lib.pdm_last_error()
g = torch.Generator(device="cuda").manual_seed(0)
qkv = torch.randn(rows * L, 3 * H * Dh, device="cuda", generator=g).bfloat16()
for _ in range(iters):
    _lib.attention(qkv, rows, L, H, Dh)
torch.cuda.synchronize()
print("done")

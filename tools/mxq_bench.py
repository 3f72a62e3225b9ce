"""pdm_mx_quantize at the H/4 fp8 forward's attention-output shape (rows x 258 tokens, K = 1152, bf16), GPU time of
graph replays (dev tool; A/B two builds with PDM_LIB_PATH).  Usage: python3 tools/mxq_bench.py [rows]"""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 50
M, K = rows * 258, 1152
x = torch.randn(M, K, device="cuda").bfloat16()
q = torch.empty(M, K, dtype=torch.float8_e4m3fn, device="cuda")
s = torch.zeros((K + 127) // 128, M, dtype=torch.int32, device="cuda")
lib = _lib.load()


def fn():
    _lib.check(lib.pdm_mx_quantize(_lib.ptr(x), _lib.PDM_BF16, K, M, K, _lib.ptr(q), K, _lib.ptr(s), M,
                                   _lib.stream_ptr()), "pdm_mx_quantize")


st = torch.cuda.Stream()
st.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(st):
    fn()
torch.cuda.current_stream().wait_stream(st)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for _ in range(20):
        fn()
ts = []
for _ in range(9):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 20 * 1e3)
t = sorted(ts)[4]
byt = M * K * 2 + M * K + M * K // 32
print(f"mx_quantize M={M} K={K}: {t:.1f} us, {byt / t / 1e3:.0f} GB/s", flush=True)

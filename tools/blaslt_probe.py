"""Which hipBLASLt kernels torch.nn.functional.linear picks on the U-ViT block GEMM shapes (run under rocprofv3
--kernel-trace --stats; the kernel names encode the macro tile / MFMA / depth the vendor library chose)."""
import sys

import torch

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 190
D = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
M = rows * 258
g = torch.Generator(device="cuda").manual_seed(0)
A = torch.randn(M, 4 * D, device="cuda", generator=g).bfloat16()
for name, N, K in (("qkv", 3 * D, D), ("proj", D, D), ("fc1", 4 * D, D), ("fc2", D, 4 * D)):
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g).bfloat16()
    a = A[:, :K].contiguous()
    for _ in range(20):
        torch.nn.functional.linear(a, W, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        torch.nn.functional.linear(a, W, b)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"{name}: M={M} N={N} K={K} {ms * 1e3:.1f} us {2 * M * N * K / ms / 1e9:.0f} TF/s", flush=True)

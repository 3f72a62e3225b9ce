"""Decoder conv3x3 shapes under each GEMM tile policy (dev tool): python tools/conv_bench.py [B]
Shapes: the KL-f8 decoder's 512^2 / 256^2 levels (libs/autoencoder.py:303-409, ch 128, ch_mult 1 2 4 4)."""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

lib = _lib.load()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)


def timeit(fn, n=5, rounds=3):
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / n)
    return sorted(ts)[rounds // 2] * 1e3


# (name, source res, cin, cout, up, epi)
shapes = [("L0 conv 128->128", 512, 128, 128, 0, "bf16"), ("L0 conv2 128->128 acc", 512, 128, 128, 0, "f32acc"),
          ("L0 conv1 256->128", 512, 256, 128, 0, "bf16"), ("L1 up 256 @512", 256, 256, 256, 1, "f32"),
          ("L1 conv 256->256", 256, 256, 256, 0, "bf16"), ("L2 up 512 @256", 128, 512, 512, 1, "f32")]
for name, r, cin, cout, up, epi in shapes:
    x = torch.randn(B, r, r, cin, device=dev, generator=g).bfloat16()
    w = (torch.randn(cout, cin, 3, 3, device=dev, generator=g) * (9 * cin) ** -0.5).bfloat16()
    bias = torch.randn(cout, device=dev, generator=g)
    R = r << up
    flops = 2.0 * B * R * R * cout * 9 * cin
    acc = torch.zeros(B * R * R, cout, device=dev) if epi != "bf16" else None
    ob = torch.empty(B * R * R, cout, device=dev, dtype=torch.bfloat16) if epi == "bf16" else None
    line = f"{name:24s} B={B} M={B * R * R}"
    for algo in [0, 1, 7, 8, 9]:
        lib.pdm_set_gemm_algo(algo)
        try:
            fn = (lambda: _lib.gemm_conv3x3(x, w, bias, _lib.EPI_BF16, up=up, out=ob)) if epi == "bf16" else \
                 (lambda: _lib.gemm_conv3x3(x, w, bias, _lib.EPI_F32, up=up, out_f32=acc, accumulate=epi == "f32acc"))
            fn()
            t = timeit(fn)
        finally:
            lib.pdm_set_gemm_algo(0)
        line += f" | a{algo} {t:8.1f}us {flops / t / 1e6:5.0f}TF"
    print(line, flush=True)

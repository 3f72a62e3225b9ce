"""Quick timing of one U-ViT forward at a given batch (dev tool)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import configs, weights  # noqa: E402
from panopticdiffusionmodels_amd.utils import get_nnet  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "imagenet256_uvit_large"
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 100
n = int(sys.argv[3]) if len(sys.argv) > 3 else 10   # timed forwards
precision = sys.argv[4] if len(sys.argv) > 4 else "bf16"
dev = torch.device("cuda")
cfg = configs.nnet_kwargs(name)
sd = weights.nnet_state_dict(cfg, seed=0, device=dev)
net = get_nnet(**cfg).to(dev)
net.load_state_dict(sd)
if precision != "bf16":
    net.set_precision(precision)
zs = configs.get_config(name)["z_shape"]
x = torch.randn(rows, *zs, device=dev)
t = torch.rand(rows, device=dev) * 999
if cfg["name"] == "uvit_t2i":   # context + panoptic mask token (libs/uvit_t2i.py:378)
    extra = (torch.randn(rows, cfg["num_clip_token"], cfg["clip_dim"], device=dev),
             torch.randn(rows, cfg["num_panoptic_class"], *zs[1:], device=dev))
else:
    extra = (torch.randint(0, 1000, (rows,), device=dev) if cfg.get("num_classes", -1) > 0 else None,)
with torch.no_grad():
    for _ in range(3):
        net.forward_pre(x, t, *extra)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        net.forward_pre(x, t, *extra)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
D, depth = cfg["embed_dim"], cfg["depth"]
L = (cfg["img_size"] // cfg["patch_size"]) ** 2 + (2 if cfg.get("num_classes", -1) > 0 else 1)
gemm_flops = rows * L * (depth + 1) * 2 * (3 * D * D + D * D + 8 * D * D) + rows * L * (depth // 2) * 2 * 2 * D * D
attn_flops = rows * (depth + 1) * 4 * L * L * D
print(f"{name} {precision} rows={rows}: {dt*1e3:.2f} ms/forward, {(gemm_flops+attn_flops)/dt/1e12:.1f} TFLOP/s")

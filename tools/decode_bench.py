"""Time the HIP KL-f8 decode (dev tool): python tools/decode_bench.py [B latent]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd.libs.autoencoder import get_model  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
s = int(sys.argv[2]) if len(sys.argv) > 2 else 32
dev = torch.device("cuda")
ae = get_model(None, seed=1, latent_size=s).to(dev)
z = torch.randn(B, 4, s, s, device=dev)
for _ in range(2):
    ae.decode(z)
torch.cuda.synchronize()
n = 5
t0 = time.perf_counter()
for _ in range(n):
    img = ae.decode(z)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / n
gf = 622.2 if s == 32 else 2514.5
print(f"decode B={B} latent={s}: {dt*1e3:.1f} ms, {B/dt:.1f} img/s, {B*gf/dt/1e3:.1f} TFLOP/s, finite={bool(torch.isfinite(img).all())}")

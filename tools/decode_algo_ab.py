"""A/B of the GEMM tile policy inside the HIP KL-f8 decode (dev tool): auto policy (128-tile kernel for the
N = 128 convs of the 256^2 level) vs the 256-tile kernel forced for every decoder GEMM.
usage: python tools/decode_algo_ab.py [B latent]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402
from panopticdiffusionmodels_amd.libs.autoencoder import get_model  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
s = int(sys.argv[2]) if len(sys.argv) > 2 else 32
lib = _lib.load()
dev = torch.device("cuda")
ae = get_model(None, seed=1, latent_size=s).to(dev)
z = torch.randn(B, 4, s, s, device=dev)
outs, times = {}, {0: [], 7: []}
for rnd in range(4):
    for algo in (0, 7):
        assert lib.pdm_set_gemm_algo(algo) == 0, lib.pdm_last_error()
        ae.decode(z)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            img = ae.decode(z)
        torch.cuda.synchronize()
        times[algo].append((time.perf_counter() - t0) / 3)
        outs[algo] = img.float()
lib.pdm_set_gemm_algo(0)
err = float((outs[0] - outs[7]).norm() / outs[0].norm())
for algo in (0, 7):
    t = sorted(times[algo])[1]
    print(f"decode B={B} latent={s} algo={algo}: {t*1e3:.1f} ms  (rounds: {[round(x*1e3, 1) for x in times[algo]]})")
print(f"rel-L2 between the two policies: {err:.2e}")

"""Speed-of-light decomposition of one eager U-ViT forward (dev tool): the same forward timed with parts of the
GEMM family switched off by pdm_set_gemm_tuning timing bits (wrong results, timing only), interleaved in one
process so the variants share the box's clock state.
  a11 / a7    the forward with the persistent GEMM (algo 11, the default) / the per-tile GEMM (algo 7)
  noepi11/7   timing bit 16: every 256-tile GEMM skips its epilogue (main loops only; nothing written)
usage: python tools/sol_forward.py [config] [rows] [rounds] [precision]"""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib, configs, weights  # noqa: E402
from panopticdiffusionmodels_amd.utils import get_nnet  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "imagenet256_uvit_large"
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 100
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
precision = sys.argv[4] if len(sys.argv) > 4 else "bf16"
lib = _lib.load()
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
if cfg["name"] == "uvit_t2i":
    extra = (torch.randn(rows, cfg["num_clip_token"], cfg["clip_dim"], device=dev),
             torch.randn(rows, cfg["num_panoptic_class"], *zs[1:], device=dev))
else:
    extra = (torch.randint(0, 1000, (rows,), device=dev) if cfg.get("num_classes", -1) > 0 else None,)
modes = {"a11": (11, 0), "a7": (7, 0), "noepi11": (11, 16), "noepi7": (7, 16)}
if os.environ.get("SOL_MODES"):   # e.g. "a11:11:0,a12:12:0" = name:algo:timing bits
    modes = {m.split(":")[0]: (int(m.split(":")[1]), int(m.split(":")[2])) for m in os.environ["SOL_MODES"].split(",")}
res = {k: [] for k in modes}
with torch.no_grad():
    for _ in range(20):
        net.forward_pre(x, t, *extra)
    torch.cuda.synchronize()
    for r in range(rounds):
        for k, (algo, dbg) in modes.items():
            lib.pdm_set_gemm_algo(algo)
            lib.pdm_set_gemm_tuning(0, dbg)
            net.forward_pre(x, t, *extra)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                net.forward_pre(x, t, *extra)
            torch.cuda.synchronize()
            res[k].append((time.perf_counter() - t0) / 5 * 1e3)
    lib.pdm_set_gemm_tuning(0, 0)
    lib.pdm_set_gemm_algo(0)
for k, v in res.items():
    v = sorted(v)
    print(f"{name} {precision} rows={rows} {k:8s} median {v[len(v) // 2]:.2f} ms/forward  min {v[0]:.2f}", flush=True)

"""U-ViT forward time per GEMM algo override, interleaved rounds (dev tool):
  python tools/forward_algo_ab.py CONFIG ROWS PRECISION ALGO[,ALGO...]   (0 = automatic)"""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib, configs, weights  # noqa: E402
from panopticdiffusionmodels_amd.utils import get_nnet  # noqa: E402

name, rows, precision = sys.argv[1], int(sys.argv[2]), sys.argv[3]
algos = [int(a) for a in sys.argv[4].split(",")]
lib = _lib.load()
dev = torch.device("cuda")
cfg = configs.nnet_kwargs(name)
net = get_nnet(**cfg).to(dev)
net.load_state_dict(weights.nnet_state_dict(cfg, seed=0, device=dev))
if precision != "bf16":
    net.set_precision(precision)
zs = configs.get_config(name)["z_shape"]
x = torch.randn(rows, *zs, device=dev)
t = torch.rand(rows, device=dev) * 999
extra = (torch.randint(0, 1000, (rows,), device=dev),)
outs, ts = {}, {a: [] for a in algos}
with torch.no_grad():
    for rnd in range(6):
        for a in algos:
            assert lib.pdm_set_gemm_algo(a) == 0
            for _ in range(2):
                o = net.forward_pre(x, t, *extra)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                o = net.forward_pre(x, t, *extra)
            e1.record()
            torch.cuda.synchronize()
            ts[a].append(e0.elapsed_time(e1) / 5)
            outs[a] = o.float()
    lib.pdm_set_gemm_algo(0)
ref = outs[algos[0]]
for a in algos:
    v = sorted(ts[a])
    print(f"{name} {precision} rows={rows} algo {a}: median {v[len(v) // 2]:.3f} ms/forward (min {v[0]:.3f}), "
          f"rel-L2 vs algo {algos[0]} {float((outs[a] - ref).norm() / ref.norm()):.2e}", flush=True)

"""Speed-of-light of the bench's sampling configuration (dev tool): the 50-NFE CFG sample of B images as `lanes`
concurrent lanes (graph replay, as bench.py times it), with the GEMM family switched by algo / timing bits --
wrong results for the timing modes, timing only.  Modes are interleaved in one process; each builds its own sampler
(the graphs capture the GEMM policy at capture time).
usage: python tools/sol_lanes.py [config] [B] [lanes] [rounds] [modes: name=algo:dbg,...]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib, configs, parallel, weights  # noqa: E402
from panopticdiffusionmodels_amd.sampler import ClassCondSampler  # noqa: E402
from panopticdiffusionmodels_amd.utils import get_nnet  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "imagenet256_uvit_large"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 50
lanes = int(sys.argv[3]) if len(sys.argv) > 3 else 2
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 2
spec = sys.argv[5] if len(sys.argv) > 5 else "a11=11:0,a7=7:0,noepi11=11:16"
modes = {}
for item in spec.split(","):
    k, v = item.split("=")
    a, d = v.split(":")
    modes[k] = (int(a), int(d))
lib = _lib.load()
dev = torch.device("cuda")
full = configs.get_config(name)
ncfg = dict(full["nnet"])
net = get_nnet(**ncfg).to(dev).eval()
net.load_state_dict(weights.nnet_state_dict(ncfg, seed=0, init="reference", device=dev))
if hasattr(net, "set_precision"):
    net.set_precision(full.get("precision", "bf16"))
null_label = ncfg["num_classes"] - 1 if ncfg.get("num_classes", -1) > 0 else None
z, y = parallel.sample_inputs(list(range(B)), full["z_shape"], num_classes=1000 if null_label is not None else None)
z = z.to(dev)
y = y.to(dev) if y is not None else None
samplers = {}
for k, (algo, dbg) in modes.items():
    lib.pdm_set_gemm_algo(algo)
    lib.pdm_set_gemm_tuning(0, dbg)
    s = ClassCondSampler(net, front_end=full["front_end"], cfg_scale=full["cfg_scale"], null_label=null_label,
                         steps=full["sample_steps"], eps=full.get("eps"), lanes=lanes)
    s.sample(z, y)   # captures the graphs under this mode
    torch.cuda.synchronize()
    samplers[k] = s
lib.pdm_set_gemm_algo(0)
lib.pdm_set_gemm_tuning(0, 0)
res = {k: [] for k in modes}
for r in range(rounds):
    for k, s in samplers.items():
        s.sample(z, y)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            s.sample(z, y)
        torch.cuda.synchronize()
        res[k].append((time.perf_counter() - t0) / 3 * 1e3)
for k, v in res.items():
    v = sorted(v)
    print(f"{name} B={B} lanes={lanes} {k:8s} sampling median {v[len(v) // 2]:.1f} ms  min {v[0]:.1f}", flush=True)

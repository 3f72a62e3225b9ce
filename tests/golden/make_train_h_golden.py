"""Generate tests/golden/train_h_golden.npz: the REFERENCE's training loop at head dim 72 (tiny_uvit_train_h, 8 heads
x 72 as U-ViT-H/2 and H/4; build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_train_h_golden.py [/root/reference]

Three iterations of train_ldm_discrete.py's train_step (159-175) exactly as make_train_golden.py runs them for the
head-dim-64 configs.  A head-dim-72 net is at least 576 wide (the GEMMs' 64-multiple widths), ~8.6 M parameters, so
instead of whole tensors each gradient / displacement is stored as a sketch: its norm and its inner products with 8
seeded N(0, 1) vectors (seed crc32(key) + i), plus every tensor of <= 4096 elements whole.  A relative error e of a
tensor shows up as the same relative error of its sketch (the projections are a random embedding).  Nothing here is
imported by the product or run on the GPU box; the .npz is data.
"""
import os
import sys
import zlib

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import C, W, _import_reference, _np, _sd_checksum  # noqa: E402
from make_train_golden import SEEDS, _ref_defs, batch  # noqa: E402

NAME = "tiny_uvit_train_h"
S = 8


def sketch(key, v):
    """(norm, S projections) of tensor v: inner products with N(0, 1) vectors seeded crc32(key) + i."""
    v = v.detach().double().flatten()
    pr = [float(torch.randn(v.numel(), generator=torch.Generator().manual_seed(zlib.crc32(key.encode()) + i),
                            dtype=torch.float64) @ v) for i in range(S)]
    return np.array([float(v.norm())] + pr)


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    uvit = _import_reference(ref)[0]
    ns = {"torch": torch, "np": np, "nn": torch.nn}
    _ref_defs(os.path.join(ref, "train_ldm_discrete.py"),
              {"stable_diffusion_beta_schedule", "get_skip", "stp", "mos", "Schedule", "LSimple"}, ns)
    _ref_defs(os.path.join(ref, "utils.py"), {"customized_lr_scheduler", "ema"}, ns)
    full = C.get_config(NAME)
    cfg = full["nnet"]
    sd = W.nnet_state_dict(cfg, seed=11, init="random")
    kw = dict(cfg)
    kw.pop("name")
    net = uvit.UViT(**kw)
    net.load_state_dict(sd)
    net.train()
    opt = full["optimizer"]
    optimizer = torch.optim.AdamW(net.parameters(), lr=opt["lr"], weight_decay=opt["weight_decay"],
                                  betas=tuple(opt["betas"]))
    sched = ns["customized_lr_scheduler"](optimizer, warmup_steps=full["lr_scheduler"]["warmup_steps"])
    x0, y = batch(NAME)
    schedule = ns["Schedule"](ns["stable_diffusion_beta_schedule"]())
    out = {"sd_checksum": _sd_checksum(sd), "x0": _np(x0), "y": _np(y)}
    for i, (nps, ts) in enumerate(SEEDS):
        optimizer.zero_grad()
        np.random.seed(nps)
        torch.manual_seed(ts)
        loss = ns["LSimple"](x0, net, schedule, y=y)
        np.random.seed(nps)
        torch.manual_seed(ts)
        n, eps, xn = schedule.sample(x0)
        out[f"it{i}_t"] = _np(n.float())
        out[f"it{i}_eps"] = _np(eps)
        out[f"it{i}_xt"] = _np(xn)
        out[f"it{i}_loss"] = _np(loss)
        out[f"it{i}_lr"] = np.array(optimizer.param_groups[0]["lr"])
        loss.mean().backward()
        if i == 0:
            for k, p in net.named_parameters():
                g = p.grad if p.grad is not None else torch.zeros_like(p)
                out[f"gsk/{k}"] = sketch(k, g)
                if g.numel() <= 4096:
                    out[f"grad/{k}"] = _np(g)
        optimizer.step()
        sched.step()
    for k, p in net.named_parameters():
        out[f"dsk/{k}"] = sketch(k, p.detach() - sd[k])
    path = os.path.join(HERE, "train_h_golden.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays, {os.path.getsize(path) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()

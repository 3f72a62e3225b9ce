"""Generate tests/golden/t2i_train_golden.npz: the REFERENCE's panoptic t2i training iterations on tiny_t2i_train
(build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_t2i_train_golden.py [/root/reference]

Two iterations of train_t2i_discrete.py's train_step (446-478) on one batch: seeded draws (np.random.seed /
torch.manual_seed per iteration), optimizer.zero_grad, LSimple's panoptic branch (148-224: utils.int2bits analog bits
* 2 - 1, the t2i Schedule.sample with the mask noise 2 randn, nnet(xn, n, context=..., mask_token=mask_n)),
(loss_eps.mean() + loss_mask.mean()).backward(), torch.optim.AdamW.step().  The reference's UViT (libs/uvit_t2i.py)
computes the forward / gradients; Schedule, LSimple, stp, mos, get_skip, stable_diffusion_beta_schedule (from
train_t2i_discrete.py) and int2bits (utils.py) run from the reference source with `ast` (both files import packages
absent here), with the module-level flags the script sets (use_panoptic True, p_uncond 0, use_ground_truth False,
use_twophases False).  Stored: per-iteration draws (t, eps, xt, mask_n), losses, LR; the first iteration's gradients
(parameters the forward uses); the final parameters' displacement (float16); input checksums.  Nothing here is
imported by the product or run on the GPU box; the .npz is data.
"""
import os
import random
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import C, W, _import_reference, _np, _sd_checksum  # noqa: E402
from make_train_golden import _ref_defs  # noqa: E402

ITERS = 2
SEEDS = [(300 + i, 400 + i) for i in range(ITERS)]
NAME = "tiny_t2i_train"


def batch(B=2, seed=31):
    full = C.get_config(NAME)
    n = full["nnet"]
    g = torch.Generator().manual_seed(seed)
    x0 = torch.randn(B, *full["z_shape"], generator=g)
    ctx = torch.randn(B, n["num_clip_token"], n["clip_dim"], generator=g)
    pan = torch.randint(0, 201, (B, 1, n["img_size"], n["img_size"]), generator=g)
    return x0, ctx, pan


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    mods = _import_reference(ref)
    uvit_t2i = mods[1]
    ns = {"torch": torch, "np": np, "nn": torch.nn, "random": random, "p_uncond": 0.0, "use_panoptic": True,
          "use_ground_truth": False, "use_twophases": False}
    uns = _ref_defs(os.path.join(ref, "utils.py"), {"int2bits"}, {"torch": torch, "np": np})
    ns["utils"] = types.SimpleNamespace(int2bits=uns["int2bits"])
    _ref_defs(os.path.join(ref, "train_t2i_discrete.py"),
              {"stable_diffusion_beta_schedule", "get_skip", "stp", "mos", "Schedule", "LSimple"}, ns)
    full = C.get_config(NAME)
    cfg = full["nnet"]
    sd = W.nnet_state_dict(cfg, seed=11, init="random")
    kw = dict(cfg)
    kw.pop("name")
    net = uvit_t2i.UViT(**kw)
    net.load_state_dict(sd)
    net.train()
    opt = full["optimizer"]
    optimizer = torch.optim.AdamW(net.parameters(), lr=opt["lr"], weight_decay=opt["weight_decay"],
                                  betas=tuple(opt["betas"]))
    x0, ctx, pan = batch()
    schedule = ns["Schedule"](ns["stable_diffusion_beta_schedule"]())
    out = {"sd_checksum": _sd_checksum(sd), "x0": _np(x0), "context": _np(ctx), "panoptic": _np(pan)}
    for i, (nps, ts) in enumerate(SEEDS):
        optimizer.zero_grad()
        np.random.seed(nps)
        torch.manual_seed(ts)
        random.seed(0)
        loss_eps, loss_mask = ns["LSimple"](x0, net, schedule, panoptic=pan, context=ctx)
        # the same draw, recorded (LSimple: int2bits * 2 - 1, then Schedule.sample)
        scaled = ns["utils"].int2bits(pan, out_dtype=torch.float) * 2.0 - 1.0
        np.random.seed(nps)
        torch.manual_seed(ts)
        n, eps, xn, eps_m, mask_n = schedule.sample(x0, scaled, phaseone=True)
        out[f"it{i}_t"] = _np(n.float())
        out[f"it{i}_eps"] = _np(eps)
        out[f"it{i}_xt"] = _np(xn)
        out[f"it{i}_mask_n"] = _np(mask_n)
        out[f"it{i}_loss"] = _np(loss_eps)
        out[f"it{i}_loss_mask"] = _np(loss_mask)
        out[f"it{i}_lr"] = np.array(optimizer.param_groups[0]["lr"])
        (loss_eps.mean() + loss_mask.mean()).backward()
        if i == 0:
            out["scaled"] = _np(scaled)
            for k, p in net.named_parameters():
                if p.grad is not None:
                    out[f"grad/{k}"] = _np(p.grad)
        optimizer.step()
    for k, p in net.named_parameters():
        out[f"delta/{k}"] = (p.detach() - sd[k]).numpy().astype(np.float16)
    path = os.path.join(HERE, "t2i_train_golden.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays, {os.path.getsize(path) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()

"""Generate tests/golden/train_golden.npz: the REFERENCE's own training loop on the tiny training configs (build
container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_train_golden.py [/root/reference]

For each of tiny_uvit_train (class-conditional, discrete SD schedule: train_ldm_discrete.py Schedule + LSimple) and
tiny_uvit_train_uncond (unconditional, qkv bias, no final conv, continuous VPSDE: sde.LSimple + ScoreModel
'noise_pred'), three iterations of the reference's train_step (train_ldm_discrete.py:159-175) run on one batch:
seeded noise draw (np.random.seed / torch.manual_seed per iteration), optimizer.zero_grad, loss.mean().backward(),
torch.optim.AdamW.step() under utils.customized_lr_scheduler, lr_scheduler.step(), utils.ema(nnet_ema, nnet, rate).
The reference's UViT module (libs/uvit.py) computes the forward / gradients; Schedule, LSimple, stp, mos (from
train_ldm_discrete.py) and customized_lr_scheduler, ema (from utils.py) are executed from the reference source with
`ast` (both files import packages absent here).  Stored: per-iteration losses and noise draws, the first
iteration's gradients, the final parameters and EMA parameters (all keys), input checksums.  Nothing here is
imported by the product or run on the GPU box; the .npz is data.
"""
import ast
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import C, W, _import_reference, _np, _sd_checksum  # noqa: E402

ITERS = 3
SEEDS = [(100 + i, 200 + i) for i in range(ITERS)]   # (np.random.seed, torch.manual_seed) per iteration


def _ref_defs(path, names, ns):
    """Execute the named top-level functions / classes of a reference file that cannot be imported whole."""
    tree = ast.parse(open(path).read())
    keep = [n for n in tree.body if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and n.name in names]
    exec(compile(ast.Module(body=keep, type_ignores=[]), path, "exec"), ns)
    return ns


def batch(name, B=4, seed=21):
    full = C.get_config(name)
    n = full["nnet"]
    g = torch.Generator().manual_seed(seed)
    x0 = torch.randn(B, *full["z_shape"], generator=g)
    y = None
    if n.get("num_classes", -1) > 0:
        y = torch.randint(0, n["num_classes"] - 1, (B,), generator=g)
        y[-1] = n["num_classes"] - 1   # a dropped (null) label, as CFGDataset produces
    return x0, y


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    mods = _import_reference(ref)
    uvit, sde_mod = mods[0], mods[5]
    ns = {"torch": torch, "np": np, "nn": torch.nn}
    _ref_defs(os.path.join(ref, "train_ldm_discrete.py"),
              {"stable_diffusion_beta_schedule", "get_skip", "stp", "mos", "Schedule", "LSimple"}, ns)
    _ref_defs(os.path.join(ref, "utils.py"), {"customized_lr_scheduler", "ema"}, ns)
    out = {}
    for name in ("tiny_uvit_train", "tiny_uvit_train_uncond"):
        full = C.get_config(name)
        cfg = full["nnet"]
        sd = W.nnet_state_dict(cfg, seed=11, init="random")
        kw = dict(cfg)
        kw.pop("name")
        net = uvit.UViT(**kw)
        net.load_state_dict(sd)
        net_ema = uvit.UViT(**kw)
        net_ema.load_state_dict(sd)   # utils.initialize_train_state: ema_update(0)
        net.train()
        opt = full["optimizer"]
        optimizer = torch.optim.AdamW(net.parameters(), lr=opt["lr"], weight_decay=opt["weight_decay"],
                                      betas=tuple(opt["betas"]))
        sched = ns["customized_lr_scheduler"](optimizer, warmup_steps=full["lr_scheduler"]["warmup_steps"])
        x0, y = batch(name)
        kwargs = {"y": y} if y is not None else {}
        objective = full["train"]["objective"]
        schedule = ns["Schedule"](ns["stable_diffusion_beta_schedule"]())
        score_model = sde_mod.ScoreModel(net, pred="noise_pred", sde=sde_mod.VPSDE())
        out[f"{name}/sd_checksum"] = _sd_checksum(sd)
        out[f"{name}/x0"] = _np(x0)
        if y is not None:
            out[f"{name}/y"] = _np(y)
        for i, (nps, ts) in enumerate(SEEDS):
            optimizer.zero_grad()
            np.random.seed(nps)
            torch.manual_seed(ts)
            if objective == "discrete":
                loss = ns["LSimple"](x0, net, schedule, **kwargs)
                np.random.seed(nps)
                torch.manual_seed(ts)
                n, eps, xn = schedule.sample(x0)   # the same draw, recorded
                out[f"{name}/it{i}_t"] = _np(n.float())
            else:
                loss = sde_mod.LSimple(score_model, x0, pred="noise_pred", **kwargs)
                torch.manual_seed(ts)
                t, eps, xn = score_model.sde.sample(x0)
                out[f"{name}/it{i}_t"] = _np(t * 999)
            out[f"{name}/it{i}_eps"] = _np(eps)
            out[f"{name}/it{i}_xt"] = _np(xn)
            out[f"{name}/it{i}_loss"] = _np(loss)
            out[f"{name}/it{i}_lr"] = np.array(optimizer.param_groups[0]["lr"])
            loss.mean().backward()
            if i == 0:
                for k, p in net.named_parameters():
                    out[f"{name}/grad/{k}"] = _np(p.grad if p.grad is not None else torch.zeros_like(p))
            optimizer.step()
            sched.step()
            ns["ema"](net_ema, net, full["train"]["ema_rate"])
        for k, p in net.named_parameters():
            out[f"{name}/param/{k}"] = _np(p)
        for k, p in net_ema.named_parameters():
            out[f"{name}/ema/{k}"] = _np(p)
    path = os.path.join(HERE, "train_golden.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays, {os.path.getsize(path) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()

"""ORACLE (test infrastructure): fp32 CPU restatement of the LSimple training step.

Follows train_ldm_discrete.py:54-90 (Schedule, LSimple), 159-175 (train_step), train_t2i_discrete.py:111-142,148-224,
446-473 (the panoptic Schedule.sample, LSimple's mask branch, loss_eps.mean() + loss_mask.mean()), utils.py:475-488
(int2bits), sde.py:64-69,270-279 (VPSDE sample,
LSimple with ScoreModel.noise_pred: the net sees t * 999), utils.py:308-345 (torch.optim.AdamW, the 'customized'
warm-up LambdaLR, ema).  Gradients are torch autograd through oracle/uvit_ref.uvit_forward (itself pinned to the
reference's UViT at full size); the whole step is pinned to the reference's own training loop by
tests/golden/train_golden.npz (tests/golden/make_train_golden.py imports the reference).  Only tests/ use this.
"""
import numpy as np
import torch

from . import uvit_ref


def mos(a):
    """mean of squares per sample (train_ldm_discrete.py:49-50)."""
    return a.pow(2).flatten(1).mean(-1)


def lsimple_grads(sd, cfg, xt, t_in, y, target):
    """Per-sample loss mos(target - nnet(xt, t_in, y)) and d loss.mean() / d params (every key; zeros where a
    parameter does not reach the loss, e.g. unused label rows)."""
    params = {k: v.detach().clone().float().requires_grad_(True) for k, v in sd.items()}
    pred = uvit_ref.uvit_forward(params, cfg, xt, t_in, y)
    loss = mos(target - pred)
    loss.mean().backward()
    grads = {k: (p.grad if p.grad is not None else torch.zeros_like(p)).detach() for k, p in params.items()}
    return loss.detach(), grads


def adamw_step(p, g, m, v, step, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
    """torch.optim.AdamW single-tensor update (decoupled decay, bias-corrected moments); returns (p, m, v)."""
    b1, b2 = betas
    p = p * (1 - lr * weight_decay)
    m = b1 * m + (1 - b1) * g
    v = b2 * v + (1 - b2) * g * g
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = v.sqrt() / (bc2 ** 0.5) + eps
    p = p - (lr / bc1) * m / denom
    return p, m, v


def customized_lr(base_lr, step, warmup_steps):
    """utils.customized_lr_scheduler: factor min(step / warmup, 1) (1 without warm-up) at scheduler step `step`."""
    return base_lr * (min(step / warmup_steps, 1) if warmup_steps > 0 else 1)


def ema(e, p, rate):
    """utils.ema: e <- rate e + (1 - rate) p."""
    return rate * e + (1 - rate) * p


def sd_betas():
    return (torch.linspace(0.00085 ** 0.5, 0.0120 ** 0.5, 1000, dtype=torch.float64) ** 2).numpy()


def discrete_sample(x0, np_seed, torch_seed):
    """Schedule.sample (train_ldm_discrete.py:75-80) under np.random.seed / torch.manual_seed: (n, eps, xn)."""
    betas = np.append(0., sd_betas())
    cum = (1. - betas).cumprod()
    np.random.seed(np_seed)
    torch.manual_seed(torch_seed)
    n = np.random.choice(list(range(1, 1001)), (len(x0),))
    eps = torch.randn_like(x0)
    a = torch.from_numpy(cum[n] ** 0.5).float().view(-1, 1, 1, 1)
    s = torch.from_numpy((1. - cum[n]) ** 0.5).float().view(-1, 1, 1, 1)
    return torch.tensor(n), eps, a * x0 + s * eps


def sde_sample(x0, torch_seed, beta_min=0.1, beta_max=20.0):
    """VPSDE sample (sde.py:64-69,72-113) under torch.manual_seed: (t, eps, xt)."""
    torch.manual_seed(torch_seed)
    t = torch.rand(x0.shape[0])
    integ = beta_min * t + (beta_max - beta_min) * t ** 2 * 0.5
    alpha = torch.exp(-integ)
    mean = alpha.sqrt().view(-1, 1, 1, 1) * x0
    std = (1. - alpha).sqrt()
    eps = torch.randn_like(x0)
    return t, eps, mean + std.view(-1, 1, 1, 1) * eps


def train_steps(sd, cfg, x0, y, draws, objective, opt, warmup_steps, ema_rate):
    """`len(draws)` reference training iterations on one batch: draws[i] = seeds of iteration i.  Returns (losses per
    iteration, the first iteration's grads, final params, final ema)."""
    p = {k: v.detach().clone().float() for k, v in sd.items()}
    m = {k: torch.zeros_like(v) for k, v in p.items()}
    v2 = {k: torch.zeros_like(v) for k, v in p.items()}
    e = {k: v.clone() for k, v in p.items()}
    losses, g0 = [], None
    for i, seeds in enumerate(draws):
        if objective == "discrete":
            n, eps, xt = discrete_sample(x0, *seeds)
            t_in = n.float()
        else:
            t, eps, xt = sde_sample(x0, seeds[1])
            t_in = t * 999
        loss, g = lsimple_grads(p, cfg, xt, t_in, y, eps)
        losses.append(loss)
        if g0 is None:
            g0 = g
        lr = customized_lr(opt["lr"], i, warmup_steps)
        for k in p:
            p[k], m[k], v2[k] = adamw_step(p[k], g[k], m[k], v2[k], i + 1, lr, opt["betas"], opt.get("eps", 1e-8),
                                           opt["weight_decay"])
            e[k] = ema(e[k], p[k], ema_rate)
    return losses, g0, p, e


def int2bits(x, n=8):
    """utils.int2bits (utils.py:475-488): integer masks (b, 1, h, w) -> bits (b, n, h, w), channel 0 = the most
    significant bit (x >> (n-1)), channel n-1 = x mod 2."""
    x = x.to(torch.int64)
    y = torch.cat([torch.bitwise_right_shift(x, i) for i in range(n - 1, -1, -1)], dim=1)
    return torch.remainder(y, 2).float()


def t2i_sample(x0, scaled, np_seed, torch_seed):
    """The t2i Schedule.sample with a panoptic mask (train_t2i_discrete.py:111-142) under np.random.seed /
    torch.manual_seed: n ~ U{1..1000}, eps = randn_like(x0), xn; eps_m = 2 randn_like(scaled), mask_n."""
    betas = np.append(0., sd_betas())
    cum = (1. - betas).cumprod()
    np.random.seed(np_seed)
    torch.manual_seed(torch_seed)
    n = np.random.choice(list(range(1, 1001)), (len(x0),))
    eps = torch.randn_like(x0)
    a = torch.from_numpy(cum[n] ** 0.5).float().view(-1, 1, 1, 1)
    s = torch.from_numpy((1. - cum[n]) ** 0.5).float().view(-1, 1, 1, 1)
    xn = a * x0 + s * eps
    eps_m = 2.0 * torch.randn_like(scaled)
    mask_n = a * scaled + s * eps_m
    return torch.tensor(n), eps, xn, eps_m, mask_n


def lsimple_t2i_grads(sd, cfg, xt, t_in, context, mask_n, eps, scaled):
    """Per-sample loss_eps = mos(eps - eps_pred), loss_mask = mos(mask_pred - scaled) of the separate-stream panoptic
    net (mask_token = mask_n) and d(loss_eps.mean() + loss_mask.mean()) / d params.  Returns (loss_eps, loss_mask,
    grads, used): grads are zeros for parameters the forward never touches, `used` the keys that got a gradient
    (torch.optim skips the others)."""
    params = {k: v.detach().clone().float().requires_grad_(True) for k, v in sd.items()}
    noise, y = uvit_ref.uvit_t2i_forward(params, cfg, xt, t_in, context, mask_token=mask_n, enable_panoptic=True)
    le, lm = mos(eps - noise), mos(y - scaled)
    (le.mean() + lm.mean()).backward()
    used = {k for k, p in params.items() if p.grad is not None}
    grads = {k: (p.grad if p.grad is not None else torch.zeros_like(p)).detach() for k, p in params.items()}
    return le.detach(), lm.detach(), grads, used


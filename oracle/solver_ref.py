"""ORACLE (test infrastructure): fp32 CPU restatement of the two DPM-Solver front-ends + CFG closures.

* Front-end A (U-ViT-H/2, H/4, panoptic t2i): dpm_solver_pp.py — discrete SD beta schedule
  (eval_ldm_discrete.py:15-19,94), piecewise-linear `interpolate_fn` (9-52), data prediction
  (`predict_x0=True`, model_fn 310-328), 'fast' method (927-1044) on a time-uniform 51-point grid,
  first/second/third single-step updates (420-494, 496-599, 679-829) including the mask co-update
  quirks.
* Front-end B (U-ViT-L/2, CIFAR S/2): dpm_solver_pytorch.py — linear VP schedule (6-102), noise
  prediction through model_wrapper(time_input_type='0') (105-218) and sde.ScoreModel.noise_pred
  (sde.py:155-184, nnet(x, t*999)), fast orders on a logSNR-uniform K+1 grid (270-299), updates
  301-432.
All arithmetic is fp32 torch like the reference (coefficient vectors of shape [B]).
"""
import math

import torch


# ----------------------------------------------------------------------------------------------
# schedules

def sd_betas(linear_start=0.00085, linear_end=0.0120, n_timestep=1000):
    """eval_ldm_discrete.py:15-19 — linspace(sqrt(b0), sqrt(b1), N)^2 in fp64 (returned as numpy fp64)."""
    return (torch.linspace(linear_start ** 0.5, linear_end ** 0.5, n_timestep, dtype=torch.float64) ** 2).numpy()


def interp(x, xp, yp):
    """dpm_solver_pp.py:9-52 — piecewise-linear interpolation with linear extrapolation from the first /
    last segment.  x [N], xp/yp [K] increasing xp."""
    K = xp.shape[0]
    idx = torch.searchsorted(xp.contiguous(), x.contiguous())  # number of knots < x
    lo = torch.where(idx == 0, torch.zeros_like(idx), torch.where(idx == K, torch.full_like(idx, K - 2), idx - 1))
    x0, x1 = xp[lo], xp[lo + 1]
    y0, y1 = yp[lo], yp[lo + 1]
    return y0 + (x - x0) * (y1 - y0) / (x1 - x0)


class DiscreteSchedule:
    """dpm_solver_pp.py:55-169, schedule='discrete' with `betas`."""

    def __init__(self, betas):
        betas = torch.as_tensor(betas).float()
        self.log_alpha = 0.5 * torch.log(1 - betas).cumsum(dim=0)
        N = self.log_alpha.shape[0]
        self.t_knots = torch.linspace(1.0 / N, 1.0, N)
        self.T = 1.0

    def log_mean(self, t):
        return interp(t.reshape(-1), self.t_knots, self.log_alpha).reshape(-1)

    def alpha(self, t):
        return torch.exp(self.log_mean(t))

    def std(self, t):
        return torch.sqrt(1.0 - torch.exp(2.0 * self.log_mean(t)))

    def lam(self, t):
        lm = self.log_mean(t)
        return lm - 0.5 * torch.log(1.0 - torch.exp(2.0 * lm))

    def inv_lam(self, lamb):
        la = -0.5 * torch.logaddexp(torch.zeros(1), -2.0 * lamb)
        return interp(la.reshape(-1), torch.flip(self.log_alpha, [0]), torch.flip(self.t_knots, [0])).reshape(-1)


class LinearSchedule:
    """dpm_solver_pytorch.py:6-102, schedule='linear' (beta_0 = 0.1, beta_1 = 20)."""

    def __init__(self):
        self.b0, self.b1, self.T = 0.1, 20.0, 1.0

    def log_mean(self, t):
        return -0.25 * t ** 2 * (self.b1 - self.b0) - 0.5 * t * self.b0

    def std(self, t):
        return torch.sqrt(1.0 - torch.exp(2.0 * self.log_mean(t)))

    def lam(self, t):
        lm = self.log_mean(t)
        return lm - 0.5 * torch.log(1.0 - torch.exp(2.0 * lm))

    def inv_lam(self, lamb):
        tmp = 2.0 * (self.b1 - self.b0) * torch.logaddexp(-2.0 * lamb, torch.zeros((1,)))
        delta = self.b0 ** 2 + tmp
        return tmp / (torch.sqrt(delta) + self.b0) / (self.b1 - self.b0)


def fast_orders(steps, order=3):
    """dpm_solver_pp.py:365-405 / dpm_solver_pytorch.py:270-299."""
    if order == 3:
        K = steps // 3 + 1
        if steps % 3 == 0:
            return [3] * (K - 2) + [2, 1], K
        if steps % 3 == 1:
            return [3] * (K - 1) + [1], K
        return [3] * (K - 1) + [2], K
    if order == 2:
        K = steps // 2
        return ([2] * K if steps % 2 == 0 else [2] * K + [1]), K
    raise ValueError("order must >= 2")


# ----------------------------------------------------------------------------------------------
# front-end A: dpm_solver_pp fast, predict_x0

def pp_sample(model, betas, x, steps=50, eps=None, T=1.0, order=3, mask_token=None,
              enable_mask_opt=False, trace=None):
    """dpm_solver_pp.py:927-1044 (method='fast', skip_type='time_uniform', solver_type='dpm_solver',
    predict_x0=True, thresholding=False).

    `model(x, t_cont, mask_token)` returns (eps, pred_mask) — the eval closure's output (CFG already
    applied, t_cont * N fed to the net).  Returns (x, pred_mask).  `trace` (list) receives x after each step.
    """
    ns = DiscreteSchedule(betas)
    N = ns.log_alpha.shape[0]
    eps = 1.0 / N if eps is None else eps
    B = x.shape[0]
    orders, _ = fast_orders(steps, order)
    ts = torch.linspace(T, eps, steps + 1)  # get_time_steps('time_uniform') 330-363

    def bc(v):
        return v[:, None, None, None]

    def model_x0(xx, t, m):  # 310-328
        noise, pm = model(xx, t, m)
        return (xx - bc(ns.std(t)) * noise) / bc(ns.alpha(t)), pm

    pred_mask = mask_token
    mask_t = mask_token
    i = 0
    for o in orders:
        s = torch.ones(B) * ts[i]
        t = torch.ones(B) * ts[i + o]
        h_ = ns.lam(ts[i + o].reshape(1)) - ns.lam(ts[i].reshape(1))
        r1 = None if o <= 1 else (ns.lam(ts[i + 1].reshape(1)) - ns.lam(ts[i].reshape(1))) / h_
        r2 = None if o <= 2 else (ns.lam(ts[i + 2].reshape(1)) - ns.lam(ts[i].reshape(1))) / h_
        m = mask_t
        lam_s, lam_t = ns.lam(s), ns.lam(t)
        h = lam_t - lam_s
        sig_s, sig_t = ns.std(s), ns.std(t)
        a_t = torch.exp(ns.log_mean(t))
        if o == 1:  # 420-494
            phi1 = (torch.exp(-h) - 1.0) / (-1.0)
            x0, pm = model_x0(x, s, m)
            x_new = bc(sig_t / sig_s) * x + bc(a_t * phi1) * x0
            if enable_mask_opt:
                m_new = bc(sig_t / sig_s) * m + bc(a_t * phi1) * pm
            else:
                m_new = pm
        elif o == 2:  # 496-599
            r1 = 0.5 if r1 is None else r1
            s1 = ns.inv_lam(lam_s + r1 * h)
            sig_s1 = ns.std(s1)
            a_s1 = torch.exp(ns.log_mean(s1))
            phi11, phi1 = torch.expm1(-r1 * h), torch.expm1(-h)
            x0, pm = model_x0(x, s, m)
            x_s1 = bc(sig_s1 / sig_s) * x - bc(a_s1 * phi11) * x0
            m_s1 = bc(sig_s1 / sig_s) * m + bc(a_s1 * phi11) * pm if enable_mask_opt else m
            x0_1, pm1 = model_x0(x_s1, s1, m_s1)
            x_new = bc(sig_t / sig_s) * x - bc(a_t * phi1) * x0 - (0.5 / r1) * bc(a_t * phi1) * (x0_1 - x0)
            if enable_mask_opt:
                m_new = bc(sig_t / sig_s) * m - bc(a_t * phi1) * pm - (0.5 / r1) * bc(a_t * phi1) * (pm1 - pm)
            else:
                m_new = pm
        else:  # 679-829
            r1 = 1.0 / 3.0 if r1 is None else r1
            r2 = 2.0 / 3.0 if r2 is None else r2
            s1 = ns.inv_lam(lam_s + r1 * h)
            s2 = ns.inv_lam(lam_s + r2 * h)
            sig_s1, sig_s2 = ns.std(s1), ns.std(s2)
            a_s1, a_s2 = torch.exp(ns.log_mean(s1)), torch.exp(ns.log_mean(s2))
            phi11, phi12, phi1 = torch.expm1(-r1 * h), torch.expm1(-r2 * h), torch.expm1(-h)
            phi22 = torch.expm1(-r2 * h) / (r2 * h) + 1.0
            phi2 = phi1 / h + 1.0
            x0, pm = model_x0(x, s, m)
            x_s1 = bc(sig_s1 / sig_s) * x - bc(a_s1 * phi11) * x0
            m_s1 = bc(sig_s1 / sig_s) * m + bc(a_s1 * phi11) * pm if enable_mask_opt else m
            x0_1, pm1 = model_x0(x_s1, s1, m_s1)
            x_s2 = bc(sig_s2 / sig_s) * x - bc(a_s2 * phi12) * x0 + r2 / r1 * bc(a_s2 * phi22) * (x0_1 - x0)
            if enable_mask_opt:
                m_s2 = bc(sig_s2 / sig_s) * m - bc(a_s2 * phi12) * pm + r2 / r1 * bc(a_s2 * phi22) * (pm1 - pm)
            else:
                m_s2 = m
            x0_2, pm2 = model_x0(x_s2, s2, m_s2)
            x_new = bc(sig_t / sig_s) * x - bc(a_t * phi1) * x0 + (1.0 / r2) * bc(a_t * phi2) * (x0_2 - x0)
            if enable_mask_opt:
                m_new = bc(sig_t / sig_s) * m - bc(a_t * phi1) * pm + (1.0 / r2) * bc(a_t * phi2) * (pm2 - pm)
            else:
                m_new = pm
        x, pred_mask, mask_t = x_new, pm, m_new
        if trace is not None:
            trace.append(x.clone())
        i += o
    return x, pred_mask


# ----------------------------------------------------------------------------------------------
# front-end B: dpm_solver_pytorch fast, noise prediction

def pytorch_sample(model, x, steps=50, eps=1e-4, T=None, order=3, trace=None):
    """dpm_solver_pytorch.py:509-589 (fast_version=True, adaptive_step_size=False) with the linear schedule.
    `model(x, t_cont)` returns the noise prediction (eval closure, CFG applied)."""
    ns = LinearSchedule()
    t_T = ns.T if T is None else T
    K = steps // 3 + 1
    if steps % 3 == 0:
        orders = [3] * (K - 2) + [2, 1]
    elif steps % 3 == 1:
        orders = [3] * (K - 1) + [1]
    else:
        orders = [3] * (K - 1) + [2]
    lam_T = ns.lam(torch.tensor(t_T))
    lam_0 = ns.lam(torch.tensor(eps))
    ts = ns.inv_lam(torch.linspace(lam_T, lam_0, K + 1))  # get_time_steps('logSNR') 237-268
    B = x.shape[0]

    def bc(v):
        return v[:, None, None, None]

    for i, o in enumerate(orders):
        s = torch.ones(B) * ts[i]
        t = torch.ones(B) * ts[i + 1]
        lam_s, lam_t = ns.lam(s), ns.lam(t)
        h = lam_t - lam_s
        la_s, la_t = ns.log_mean(s), ns.log_mean(t)
        sig_t = ns.std(t)
        if o == 1:  # 301-330
            phi1 = torch.expm1(h)
            e = model(x, s)
            x = bc(torch.exp(la_t - la_s)) * x - bc(sig_t * phi1) * e
        elif o == 2:  # 332-375
            r1 = 0.5
            s1 = ns.inv_lam(lam_s + r1 * h)
            la_s1 = ns.log_mean(s1)
            sig_s1 = ns.std(s1)
            phi11, phi1 = torch.expm1(r1 * h), torch.expm1(h)
            e = model(x, s)
            x_s1 = bc(torch.exp(la_s1 - la_s)) * x - bc(sig_s1 * phi11) * e
            e1 = model(x_s1, s1)
            x = bc(torch.exp(la_t - la_s)) * x - bc(sig_t * phi1) * e - (0.5 / r1) * bc(sig_t * phi1) * (e1 - e)
        else:  # 377-432
            r1, r2 = 1.0 / 3.0, 2.0 / 3.0
            s1 = ns.inv_lam(lam_s + r1 * h)
            s2 = ns.inv_lam(lam_s + r2 * h)
            la_s1, la_s2 = ns.log_mean(s1), ns.log_mean(s2)
            sig_s1, sig_s2 = ns.std(s1), ns.std(s2)
            phi11, phi12, phi1 = torch.expm1(r1 * h), torch.expm1(r2 * h), torch.expm1(h)
            phi22 = torch.expm1(r2 * h) / (r2 * h) - 1.0
            phi2 = torch.expm1(h) / h - 1.0
            e = model(x, s)
            x_s1 = bc(torch.exp(la_s1 - la_s)) * x - bc(sig_s1 * phi11) * e
            e1 = model(x_s1, s1)
            x_s2 = bc(torch.exp(la_s2 - la_s)) * x - bc(sig_s2 * phi12) * e - r2 / r1 * bc(sig_s2 * phi22) * (e1 - e)
            e2 = model(x_s2, s2)
            x = bc(torch.exp(la_t - la_s)) * x - bc(sig_t * phi1) * e - (1.0 / r2) * bc(sig_t * phi2) * (e2 - e)
        if trace is not None:
            trace.append(x.clone())
    return x


# ----------------------------------------------------------------------------------------------
# eval closures (CFG)

def cfg_class_closure(nnet, y, scale, null_label, time_scale):
    """eval_ldm_discrete.py:72-81,96-98 (time_scale = N = 1000) and eval_ldm.py:66-74 + sde.py:168-184
    (time_scale = 999): eps = c + s (c - u), uncond label = dataset.K."""
    def fn(x, t_cont):
        tt = t_cont * time_scale
        c = nnet(x, tt, y)
        if scale > 0:
            u = nnet(x, tt, torch.full_like(y, null_label))
            return c + scale * (c - u)
        return c
    return fn


def cfg_t2i_closure(nnet, context, empty_context, scale, time_scale=1000):
    """train_t2i_discrete.py:387-439 + 506-513 (use_panoptic=True, cfg=True, use_ground_truth=False):
    eps = c + s(c - u), pred_mask = pm + s(pm - pm_u); uncond = empty_context broadcast."""
    def fn(x, t_cont, mask_token):
        tt = t_cont * time_scale
        ec = empty_context.unsqueeze(0).expand(x.shape[0], -1, -1)
        if mask_token is None:
            c = nnet(x, tt, context)
            u = nnet(x, tt, ec)
            return c + scale * (c - u), None
        c, pm = nnet(x, tt, context, mask_token)
        u, pmu = nnet(x, tt, ec, mask_token)
        pm = pm + scale * (pm - pmu)
        return c + scale * (c - u), pm
    return fn

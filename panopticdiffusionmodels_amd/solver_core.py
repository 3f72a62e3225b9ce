"""Host-side DPM-Solver arithmetic: noise schedules as float64 scalar functions and the per-stage linear
coefficients of every single-step update.

Every update of the reference solvers is a linear combination of the step's starting state and the
model outputs of its stages, with scalar coefficients that depend only on the time grid.  They are
computed here once, in float64 on the host, from the reference's fp32 grid values, and executed on the
GPU by one fused epilogue kernel per model evaluation (pdm_stage_epilogue) or by pdm_lincomb.

Stage record (one model evaluation):
  time      continuous time of the model call
  ax, ae    model-output transform m = ax * x_in + ae * out  (data prediction: 1/alpha, -sigma/alpha)
  nx        coefficient of the step's starting state x in the NEXT state
  nm        coefficients of the earlier stage outputs m_0..m_{k-1} in the next state
  cm        coefficient of this stage's own output m_k
  mask      same (mx, mm, mc) for the panoptic mask co-update (dpm_solver_pp.py:536-564,730-766)
The next state after the last stage of a step is the step's result x_t.
"""
import math

import numpy as np
import torch


# ------------------------------------------------------------------------------------------------
# schedules (float64 scalars)

def _interp(x, xp, yp):
    """dpm_solver_pp.py:9-52 on host scalars: piecewise linear, extrapolating from the end segments."""
    K = len(xp)
    i = int(np.searchsorted(xp, x, side="left"))
    lo = 0 if i == 0 else (K - 2 if i == K else i - 1)
    x0, x1, y0, y1 = xp[lo], xp[lo + 1], yp[lo], yp[lo + 1]
    return y0 + (x - x0) * (y1 - y0) / (x1 - x0)


class HostDiscrete:
    """dpm_solver_pp.py:55-169 schedule='discrete' (knots built in fp32 exactly like the reference)."""

    def __init__(self, betas=None, alphas_cumprod=None):
        if betas is not None:
            la = 0.5 * torch.log(1 - torch.as_tensor(betas).float().cpu()).cumsum(dim=0)
        else:
            la = 0.5 * torch.log(torch.as_tensor(alphas_cumprod).float().cpu())
        N = la.shape[0]
        self.N = N
        self.log_alpha = la.double().numpy()
        self.t_knots = torch.linspace(1.0 / N, 1.0, N).double().numpy()
        self.T = 1.0

    def log_mean(self, t):
        return _interp(t, self.t_knots, self.log_alpha)

    def inv_lam(self, lamb):
        la = -0.5 * np.logaddexp(0.0, -2.0 * lamb)
        return _interp(la, self.log_alpha[::-1], self.t_knots[::-1])

    # fp32 tensor versions (grid construction exactly as the reference computes it)
    def lam_f32(self, t):
        xp = torch.from_numpy(self.t_knots).float()
        yp = torch.from_numpy(self.log_alpha).float()
        lm = torch.tensor([_interp(float(t), xp.double().numpy(), yp.double().numpy())], dtype=torch.float32)
        return lm - 0.5 * torch.log(1.0 - torch.exp(2.0 * lm))

    def inv_lam_f32(self, lamb):
        return torch.tensor([self.inv_lam(float(v)) for v in lamb], dtype=torch.float32)


class HostLinear:
    """Linear VP schedule: dpm_solver_pytorch.py:6-102 (beta in [0.1, 20]) and dpm_solver_pp.py's
    'linear' (beta_0/1 given per 1000 steps)."""

    def __init__(self, beta_0=0.1, beta_1=20.0):
        self.b0, self.b1, self.T = beta_0, beta_1, 1.0

    def log_mean(self, t):
        return -0.25 * t * t * (self.b1 - self.b0) - 0.5 * t * self.b0

    def inv_lam(self, lamb):
        tmp = 2.0 * (self.b1 - self.b0) * np.logaddexp(-2.0 * lamb, 0.0)
        delta = self.b0 ** 2 + tmp
        return tmp / (math.sqrt(delta) + self.b0) / (self.b1 - self.b0)

    def lam_f32(self, t):
        t = torch.tensor(t, dtype=torch.float32)
        lm = -0.25 * t ** 2 * (self.b1 - self.b0) - 0.5 * t * self.b0
        return lm - 0.5 * torch.log(1.0 - torch.exp(2.0 * lm))

    def inv_lam_f32(self, lamb):
        tmp = 2.0 * (self.b1 - self.b0) * torch.logaddexp(-2.0 * lamb, torch.zeros((1,)))
        delta = self.b0 ** 2 + tmp
        return tmp / (torch.sqrt(delta) + self.b0) / (self.b1 - self.b0)


class HostCosine:
    """Cosine VP schedule (dpm_solver_pytorch.py:62-102)."""

    def __init__(self, s=0.008):
        self.s = s
        self.la0 = math.log(math.cos(s / (1.0 + s) * math.pi / 2.0))
        self.T = 0.9946

    def log_mean(self, t):
        return math.log(math.cos((t + self.s) / (1.0 + self.s) * math.pi / 2.0)) - self.la0

    def inv_lam(self, lamb):
        la = -0.5 * np.logaddexp(-2.0 * lamb, 0.0)
        return math.acos(math.exp(la + self.la0)) * 2.0 * (1.0 + self.s) / math.pi - self.s

    def lam_f32(self, t):
        t = torch.tensor(t, dtype=torch.float32)
        lm = torch.log(torch.cos((t + self.s) / (1.0 + self.s) * math.pi / 2.0)) - self.la0
        return lm - 0.5 * torch.log(1.0 - torch.exp(2.0 * lm))

    def inv_lam_f32(self, lamb):
        la = -0.5 * torch.logaddexp(-2.0 * lamb, torch.zeros((1,)))
        return torch.arccos(torch.exp(la + self.la0)) * 2.0 * (1.0 + self.s) / math.pi - self.s


def alpha(hs, t):
    return math.exp(hs.log_mean(t))


def sigma(hs, t):
    return math.sqrt(1.0 - math.exp(2.0 * hs.log_mean(t)))


def lam(hs, t):
    lm = hs.log_mean(t)
    return lm - 0.5 * math.log(1.0 - math.exp(2.0 * lm))


# ------------------------------------------------------------------------------------------------
# time grids

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


def time_steps(hs, skip_type, t_T, t_0, N):
    """dpm_solver_pp.py:330-363 / dpm_solver_pytorch.py:237-268, reproduced in fp32 like the reference and
    returned as python floats (exact fp32 values)."""
    if skip_type == "logSNR":
        # fp32 like the reference (its lambda has fp32 cancellation near t_0; reproduced on purpose so the
        # net sees the reference's time inputs)
        lT = hs.lam_f32(t_T).reshape(())
        l0 = hs.lam_f32(t_0).reshape(())
        ls = torch.linspace(float(lT), float(l0), N + 1)
        return [float(v) for v in hs.inv_lam_f32(ls)]
    if skip_type == "time_uniform":
        return [float(v) for v in torch.linspace(t_T, t_0, N + 1)]
    if skip_type == "t2":
        return [float(v) for v in torch.linspace(t_T ** 0.5, t_0 ** 0.5, N + 1).pow(2)]
    if skip_type == "time_quadratic":
        t = torch.linspace(t_0, t_T, 10000000)
        qt = torch.sqrt(t)
        qs = torch.linspace(float(qt[0]), float(qt[-1]), N + 1)
        out = torch.flip(torch.cat([t[torch.searchsorted(qt, qs)[:-1]], t_T * torch.ones((1,))]), dims=[0])
        return [float(v) for v in out]
    raise ValueError(f"Unsupported skip_type {skip_type}, need to be 'logSNR' or 'time_uniform' or 'time_quadratic'")


# ------------------------------------------------------------------------------------------------
# per-step stage coefficients

def _stage(time, ax, ae, nx, nm, cm, mask=None):
    return dict(time=time, ax=ax, ae=ae, nx=nx, nm=list(nm), cm=cm, mask=mask)


def _m(mx, mm, mc):
    return dict(mx=mx, mm=list(mm), mc=mc)


def step_stages(hs, s, t, order, predict_x0=True, r1=None, r2=None, solver_type="dpm_solver",
                enable_mask_opt=False):
    """Coefficients of dpm_solver_{first,second,third}_update (dpm_solver_pp.py:420-829 for both
    predict_x0 branches; dpm_solver_pytorch.py:301-432 is the predict_x0=False branch with the default
    r1/r2).  Returns a list of stage records (module docstring)."""
    if solver_type not in ("dpm_solver", "taylor"):
        raise ValueError(f"solver_type must be either dpm_solver or taylor, got {solver_type}")
    if enable_mask_opt and solver_type == "taylor":
        raise NotImplementedError("the mask co-update is only defined for solver_type='dpm_solver'")
    ls, lt = lam(hs, s), lam(hs, t)
    h = lt - ls
    sg_s, sg_t = sigma(hs, s), sigma(hs, t)
    la_s, la_t = hs.log_mean(s), hs.log_mean(t)
    a_s, a_t = math.exp(la_s), math.exp(la_t)
    if predict_x0:
        tr = lambda tt: (1.0 / alpha(hs, tt), -sigma(hs, tt) / alpha(hs, tt))  # noqa: E731 (model_fn 310-328)
    else:
        tr = lambda tt: (0.0, 1.0)  # noqa: E731
    keep = _m(1.0, [], 0.0)  # mask passes through unchanged

    if order == 1:
        ax, ae = tr(s)
        if predict_x0:
            phi1 = -math.expm1(-h)  # (exp(-h) - 1) / (-1)
            st = _stage(s, ax, ae, sg_t / sg_s, [], a_t * phi1,
                        _m(sg_t / sg_s, [], a_t * phi1) if enable_mask_opt else "pred")
        else:
            phi1 = math.expm1(h)
            st = _stage(s, ax, ae, math.exp(la_t - la_s), [], -sg_t * phi1, "pred")
        return [st]

    if order == 2:
        r1 = 0.5 if r1 is None else r1
        s1 = hs.inv_lam(ls + r1 * h)
        sg_1, la_1 = sigma(hs, s1), hs.log_mean(s1)
        a_1 = math.exp(la_1)
        ax0, ae0 = tr(s)
        ax1, ae1 = tr(s1)
        if predict_x0:
            phi11, phi1 = math.expm1(-r1 * h), math.expm1(-h)
            st0 = _stage(s, ax0, ae0, sg_1 / sg_s, [], -a_1 * phi11,
                         _m(sg_1 / sg_s, [], a_1 * phi11) if enable_mask_opt else keep)
            if solver_type == "dpm_solver":
                c = (0.5 / r1) * a_t * phi1
                st1 = _stage(s1, ax1, ae1, sg_t / sg_s, [-a_t * phi1 + c], -c,
                             _m(sg_t / sg_s, [-a_t * phi1 + c], -c) if enable_mask_opt else "pred")
            else:
                c = (1.0 / r1) * a_t * ((math.exp(-h) - 1.0) / h + 1.0)
                st1 = _stage(s1, ax1, ae1, sg_t / sg_s, [-a_t * phi1 - c], c, "pred")
        else:
            phi11, phi1 = math.expm1(r1 * h), math.expm1(h)
            st0 = _stage(s, ax0, ae0, math.exp(la_1 - la_s), [], -sg_1 * phi11, keep)
            if solver_type == "dpm_solver":
                c = (0.5 / r1) * sg_t * phi1
            else:
                c = (1.0 / r1) * sg_t * ((math.exp(h) - 1.0) / h - 1.0)
            st1 = _stage(s1, ax1, ae1, math.exp(la_t - la_s), [-sg_t * phi1 + c], -c, "pred")
        return [st0, st1]

    if order == 3:
        r1 = 1.0 / 3.0 if r1 is None else r1
        r2 = 2.0 / 3.0 if r2 is None else r2
        s1 = hs.inv_lam(ls + r1 * h)
        s2 = hs.inv_lam(ls + r2 * h)
        sg_1, sg_2 = sigma(hs, s1), sigma(hs, s2)
        la_1, la_2 = hs.log_mean(s1), hs.log_mean(s2)
        a_1, a_2 = math.exp(la_1), math.exp(la_2)
        (ax0, ae0), (ax1, ae1), (ax2, ae2) = tr(s), tr(s1), tr(s2)
        if predict_x0:
            phi11, phi12, phi1 = math.expm1(-r1 * h), math.expm1(-r2 * h), math.expm1(-h)
            phi22 = math.expm1(-r2 * h) / (r2 * h) + 1.0
            phi2 = phi1 / h + 1.0
            phi3 = phi2 / h - 0.5
            st0 = _stage(s, ax0, ae0, sg_1 / sg_s, [], -a_1 * phi11,
                         _m(sg_1 / sg_s, [], a_1 * phi11) if enable_mask_opt else keep)
            c2 = (r2 / r1) * a_2 * phi22
            st1 = _stage(s1, ax1, ae1, sg_2 / sg_s, [-a_2 * phi12 - c2], c2,
                         _m(sg_2 / sg_s, [-a_2 * phi12 - c2], c2) if enable_mask_opt else keep)
            if solver_type == "dpm_solver":
                c3 = (1.0 / r2) * a_t * phi2
                # x_t does not use m_1 (dpm_solver_pp.py:753-758)
                st2 = _stage(s2, ax2, ae2, sg_t / sg_s, [-a_t * phi1 - c3, 0.0], c3,
                             _m(sg_t / sg_s, [-a_t * phi1 - c3, 0.0], c3) if enable_mask_opt else "pred")
            else:  # taylor, dpm_solver_pp.py:767-777
                d = r2 - r1
                # D1 = (r2 (m1-m0)/r1 - r1 (m2-m0)/r2) / d ; D2 = 2 ((m2-m0)/r2 - (m1-m0)/r1) / d
                k1 = a_t * phi2
                k2 = a_t * phi3
                c_m1 = k1 * (r2 / r1) / d - k2 * (-2.0 / r1) / d
                c_m2 = k1 * (-r1 / r2) / d - k2 * (2.0 / r2) / d
                c_m0 = -a_t * phi1 - c_m1 - c_m2
                st2 = _stage(s2, ax2, ae2, sg_t / sg_s, [c_m0, c_m1], c_m2, "pred")
        else:
            phi11, phi12, phi1 = math.expm1(r1 * h), math.expm1(r2 * h), math.expm1(h)
            phi22 = math.expm1(r2 * h) / (r2 * h) - 1.0
            phi2 = phi1 / h - 1.0
            phi3 = phi2 / h - 0.5
            st0 = _stage(s, ax0, ae0, math.exp(la_1 - la_s), [], -sg_1 * phi11, keep)
            c2 = (r2 / r1) * sg_2 * phi22
            st1 = _stage(s1, ax1, ae1, math.exp(la_2 - la_s), [-sg_2 * phi12 + c2], -c2, keep)
            if solver_type == "dpm_solver":
                c3 = (1.0 / r2) * sg_t * phi2
                st2 = _stage(s2, ax2, ae2, math.exp(la_t - la_s), [-sg_t * phi1 + c3, 0.0], -c3, "pred")
            else:
                d = r2 - r1
                k1 = sg_t * phi2
                k2 = sg_t * phi3
                # x_t = e x - sg phi1 m0 - k1 D1 - k2 D2
                c_m1 = -(k1 * (r2 / r1) / d) - k2 * (-2.0 / r1) / d
                c_m2 = -(k1 * (-r1 / r2) / d) - k2 * (2.0 / r2) / d
                c_m0 = -sg_t * phi1 - c_m1 - c_m2
                st2 = _stage(s2, ax2, ae2, math.exp(la_t - la_s), [c_m0, c_m1], c_m2, "pred")
        return [st0, st1, st2]
    raise ValueError(f"Solver order must be 1 or 2 or 3, got {order}")


def pp_fast_plan(hs, steps, t_0, t_T, order=3, skip_type="time_uniform", predict_x0=True,
                 solver_type="dpm_solver", enable_mask_opt=False):
    """DPM_Solver.sample(method='fast') of dpm_solver_pp.py:1018-1044: the step grid is `steps`+1 points,
    a step of order o spans o grid intervals and r1/r2 come from the grid's lambda spacing."""
    orders, _ = fast_orders(steps, order)
    ts = time_steps(hs, skip_type, t_T, t_0, steps)
    plan = []
    i = 0
    for o in orders:
        if i + o > len(ts) - 1:
            raise ValueError("time grid too short for the order schedule")
        h = lam(hs, ts[i + o]) - lam(hs, ts[i])
        r1 = None if o <= 1 else (lam(hs, ts[i + 1]) - lam(hs, ts[i])) / h
        r2 = None if o <= 2 else (lam(hs, ts[i + 2]) - lam(hs, ts[i])) / h
        plan.append(step_stages(hs, ts[i], ts[i + o], o, predict_x0, r1, r2, solver_type, enable_mask_opt))
        i += o
    return plan


def pp_singlestep_plan(hs, steps, t_0, t_T, order, skip_type="time_uniform", predict_x0=True,
                       solver_type="dpm_solver", enable_mask_opt=False):
    """DPM_Solver.sample(method='singlestep') of dpm_solver_pp.py:1045-1078."""
    n = steps // order
    ts = time_steps(hs, skip_type, t_T, t_0, n)
    return [step_stages(hs, ts[i], ts[i + 1], order, predict_x0, None, None, solver_type, enable_mask_opt)
            for i in range(n)]


def pt_fast_plan(hs, steps, t_0, t_T):
    """dpm_solver_pytorch DPM_Solver.sample(fast_version=True) (509-589): logSNR grid of K+1 points, one
    step per interval, default r1/r2, noise prediction."""
    orders, K = fast_orders(steps, 3)
    ts = time_steps(hs, "logSNR", t_T, t_0, K)
    return [step_stages(hs, ts[i], ts[i + 1], o, predict_x0=False) for i, o in enumerate(orders)]


def pt_plan(hs, steps, t_0, t_T, order=3, skip_type="logSNR"):
    """dpm_solver_pytorch DPM_Solver.sample(fast_version=False)."""
    n = steps // order
    ts = time_steps(hs, skip_type, t_T, t_0, n)
    return [step_stages(hs, ts[i], ts[i + 1], order, predict_x0=False) for i in range(n)]


def nfe(plan):
    return sum(len(st) for st in plan)

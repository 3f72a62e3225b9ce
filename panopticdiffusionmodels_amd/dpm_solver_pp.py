"""DPM-Solver(++) with the discrete schedule and the panoptic mask co-update — API of dpm_solver_pp.py.

`NoiseScheduleVP`, `model_wrapper` and `DPM_Solver` keep the reference signatures (dpm_solver_pp.py:55,
172, 291, 927).  The schedule methods are tensor functions like the reference.  The solver computes every
update's coefficients on the host in float64 (solver_core.step_stages) and applies them to the GPU tensors
with libpdm's fused linear-combination kernel; the model is whatever `model_fn` the caller passes.

Caller-contract fixes ("Contract conflict"): `DPM_Solver.model_fn` forwards the panoptic
keyword arguments only when a mask token is in play and accepts a tensor or an (out, pred_mask) tuple, and
`sample()` returns a tensor when `mask_token is None` (so eval_ldm_discrete.py / sample_t2i_discrete.py run
unchanged) and `(x, pred_mask)` otherwise (`return_tuple=True` forces the reference's tuple).

The multistep and adaptive methods are outside the sampling hot path (never called; the reference's
multistep references an undefined `timesteps`, dpm_solver_pp.py:997) and raise NotImplementedError.
"""
import math

import torch
import torch.nn.functional as F

from . import _lib
from . import solver_core as sc


def interpolate_fn(x, xp, yp):
    """dpm_solver_pp.py:9-52: x [N, C], xp/yp [C, K] (or [1, K]) -> [N, C], linear extrapolation at the ends."""
    N, K = x.shape[0], xp.shape[1]
    xp_b = xp.expand(x.shape[1], -1) if xp.shape[0] == 1 else xp
    yp_b = yp.expand(x.shape[1], -1) if yp.shape[0] == 1 else yp
    out = torch.empty_like(x)
    for c in range(x.shape[1]):
        xc = x[:, c].contiguous()
        idx = torch.searchsorted(xp_b[c].contiguous(), xc)
        lo = torch.where(idx == 0, torch.zeros_like(idx),
                         torch.where(idx == K, torch.full_like(idx, K - 2), idx - 1))
        x0, x1 = xp_b[c][lo], xp_b[c][lo + 1]
        y0, y1 = yp_b[c][lo], yp_b[c][lo + 1]
        out[:, c] = y0 + (xc - x0) * (y1 - y0) / (x1 - x0)
    return out


class NoiseScheduleVP:
    """dpm_solver_pp.py:55-169 API as tensor functions over ONE schedule object: the float64 host schedule
    (solver_core.HostDiscrete / HostLinear / HostCosine) that the fused samplers' coefficients come from.  The
    discrete knots are that object's (built in fp32 exactly like the reference), the linear / cosine constants
    its attributes, so the tensor API and the samplers cannot drift apart."""

    def __init__(self, schedule='discrete', beta_0=1e-4, beta_1=2e-2, total_N=1000, betas=None, alphas_cumprod=None):
        """dpm_solver_pp.py:56-119."""
        if schedule not in ['linear', 'discrete', 'cosine']:
            raise ValueError("Unsupported noise schedule {}. The schedule needs to be 'linear' or 'cosine'".format(schedule))
        self.schedule = schedule
        self.total_N = total_N
        self.beta_0 = beta_0 * 1000.
        self.beta_1 = beta_1 * 1000.
        if schedule == 'discrete':
            if betas is not None:
                self._host = sc.HostDiscrete(betas=betas)
            else:
                assert alphas_cumprod is not None
                self._host = sc.HostDiscrete(alphas_cumprod=alphas_cumprod)
            self.total_N = self._host.N
            self.t_discrete = torch.from_numpy(self._host.t_knots).float().reshape((1, -1))
            self.log_alpha_discrete = torch.from_numpy(self._host.log_alpha).float().reshape((1, -1))
        elif schedule == 'linear':
            self._host = sc.HostLinear(self.beta_0, self.beta_1)
        else:
            self._host = sc.HostCosine()
        cos = self._host if schedule == 'cosine' else sc.HostCosine()
        self.cosine_s = cos.s
        self.cosine_beta_max = 999.
        self.cosine_t_max = math.atan(self.cosine_beta_max * (1. + self.cosine_s) / math.pi) * 2. * (1. + self.cosine_s) / math.pi - self.cosine_s
        self.cosine_log_alpha_0 = cos.la0
        self.T = self._host.T

    def marginal_log_mean_coeff(self, t):
        if self.schedule == 'linear':
            return -0.25 * t ** 2 * (self._host.b1 - self._host.b0) - 0.5 * t * self._host.b0
        if self.schedule == 'discrete':
            return interpolate_fn(t.reshape((-1, 1)), self.t_discrete.to(t.device),
                                  self.log_alpha_discrete.to(t.device)).reshape((-1,))
        log_alpha_fn = lambda s: torch.log(torch.cos((s + self.cosine_s) / (1. + self.cosine_s) * math.pi / 2.))  # noqa: E731
        return log_alpha_fn(t) - self.cosine_log_alpha_0

    def marginal_alpha(self, t):
        return torch.exp(self.marginal_log_mean_coeff(t))

    def marginal_std(self, t):
        return torch.sqrt(1. - torch.exp(2. * self.marginal_log_mean_coeff(t)))

    def marginal_lambda(self, t):
        log_mean_coeff = self.marginal_log_mean_coeff(t)
        log_std = 0.5 * torch.log(1. - torch.exp(2. * log_mean_coeff))
        return log_mean_coeff - log_std

    def inverse_lambda(self, lamb):
        if self.schedule == 'linear':
            b0, b1 = self._host.b0, self._host.b1
            tmp = 2. * (b1 - b0) * torch.logaddexp(-2. * lamb, torch.zeros((1,)).to(lamb))
            Delta = b0 ** 2 + tmp
            return tmp / (torch.sqrt(Delta) + b0) / (b1 - b0)
        if self.schedule == 'discrete':
            log_alpha = -0.5 * torch.logaddexp(torch.zeros((1,)).to(lamb.device), -2. * lamb)
            t = interpolate_fn(log_alpha.reshape((-1, 1)), torch.flip(self.log_alpha_discrete.to(lamb.device), [1]),
                               torch.flip(self.t_discrete.to(lamb.device), [1]))
            return t.reshape((-1,))
        log_alpha = -0.5 * torch.logaddexp(-2. * lamb, torch.zeros((1,)).to(lamb))
        t_fn = lambda log_alpha_t: torch.arccos(torch.exp(log_alpha_t + self.cosine_log_alpha_0)) * 2. * (1. + self.cosine_s) / math.pi - self.cosine_s  # noqa: E731
        return t_fn(log_alpha)


def model_wrapper(model, noise_schedule=None, is_cond_classifier=False, classifier_fn=None, classifier_scale=1.,
                  time_input_type='1', total_N=1000, model_kwargs={}, is_deis=False):
    """dpm_solver_pp.py:172-288: continuous-time noise-prediction wrapper with optional classifier guidance."""
    def get_model_input_time(t_continuous):
        if time_input_type == '0':
            return t_continuous
        if time_input_type == '1':
            return 1000. * torch.max(t_continuous - 1. / total_N, torch.zeros_like(t_continuous).to(t_continuous))
        if time_input_type == '2':
            return (total_N - 1) / total_N * 1000. * t_continuous
        raise ValueError("Unsupported time input type {}, must be '0' or '1' or '2'".format(time_input_type))

    def cond_fn(x, t_discrete, y):
        assert y is not None
        with torch.enable_grad():
            x_in = x.detach().requires_grad_(True)
            log_probs = F.log_softmax(classifier_fn(x_in, t_discrete), dim=-1)
            selected = log_probs[range(len(log_probs)), y.view(-1)]
            return classifier_scale * torch.autograd.grad(selected.sum(), x_in)[0]

    def model_fn(x, t_continuous):
        if t_continuous.reshape((-1,)).shape[0] == 1:
            t_continuous = torch.ones((x.shape[0],)).to(x.device) * t_continuous
        if is_cond_classifier:
            y = model_kwargs.get("y", None)
            if y is None:
                raise ValueError("For classifier guidance, the label y has to be in the input.")
            t_discrete = get_model_input_time(t_continuous)
            noise_uncond = model(x, t_discrete, **model_kwargs)
            cond_grad = cond_fn(x, t_discrete, y)
            sigma_t = noise_schedule.marginal_std(t_continuous / 1000. if is_deis else t_continuous)
            return noise_uncond - sigma_t[(...,) + (None,) * (len(cond_grad.shape) - 1)] * cond_grad
        return model(x, get_model_input_time(t_continuous), **model_kwargs)

    return model_fn


def _lin(terms, coeffs):
    """sum_i c_i * T_i on the GPU (libpdm lincomb), skipping zero coefficients."""
    pairs = [(t, c) for t, c in zip(terms, coeffs) if c != 0.0]
    if not pairs:
        return torch.zeros_like(terms[0])
    return _lib.lincomb([p[0].float().contiguous() for p in pairs], [p[1] for p in pairs])


def _scalar(t):
    """The (uniform) time of a per-sample time vector, as a python float."""
    if isinstance(t, torch.Tensor):
        return float(t.reshape(-1)[0])
    return float(t)


class DPM_Solver:
    def __init__(self, model_fn, noise_schedule, predict_x0=False, thresholding=False, max_val=1.):
        self.model = model_fn
        self.noise_schedule = noise_schedule
        self.predict_x0 = predict_x0
        self.thresholding = thresholding
        self.max_val = max_val

    # ---- model call (dpm_solver_pp.py:310-328) ----------------------------------------------------
    def _call_model(self, x, t, panoptic=None, mask_token=None, use_ground_truth=False, enable_panoptic=False):
        if mask_token is None:
            out = self.model(x, t)
        else:
            out = self.model(x, t, panoptic=panoptic, mask_token=mask_token, use_ground_truth=use_ground_truth,
                             enable_panoptic=enable_panoptic)
        if isinstance(out, (tuple, list)):
            return out[0], out[1]
        return out, None

    def _data_pred(self, x, t, noise):
        ts = _scalar(t)
        hs = self.noise_schedule._host
        a, s = sc.alpha(hs, ts), sc.sigma(hs, ts)
        x0 = _lin([x, noise], [1.0 / a, -s / a])
        if self.thresholding:
            p = 0.995
            dims = len(x0.shape) - 1
            q = torch.quantile(torch.abs(x0).reshape((x0.shape[0], -1)), p, dim=1)
            q = torch.maximum(q, torch.ones_like(q))[(...,) + (None,) * dims]
            x0 = torch.clamp(x0, -q, q) / (q / self.max_val)
        return x0

    def model_fn(self, x, t, panoptic=None, mask_token=None, use_ground_truth=False, enable_panoptic=False):
        noise, pred_mask = self._call_model(x, t, panoptic, mask_token, use_ground_truth, enable_panoptic)
        if self.predict_x0:
            return self._data_pred(x, t, noise), pred_mask
        return noise, pred_mask

    # ---- time grids ---------------------------------------------------------------------------
    def get_time_steps(self, skip_type, t_T, t_0, N, device):
        return torch.tensor(sc.time_steps(self.noise_schedule._host, skip_type, t_T, t_0, N),
                            dtype=torch.float32).to(device)

    def get_time_steps_for_dpm_solver_fast(self, skip_type, t_T, t_0, steps, order, device):
        orders, K = sc.fast_orders(steps, order)
        return orders, self.get_time_steps(skip_type, t_T, t_0, K, device)

    def denoise_fn(self, x, s, noise_s=None):
        if noise_s is None:
            noise_s, _ = self._call_model(x, s)
        return self._data_pred(x, s, noise_s)

    # ---- single-step updates (dpm_solver_pp.py:420-850) -----------------------------------------
    def _run_step(self, x, s, t, order, r1=None, r2=None, solver_type='dpm_solver', panoptic=None, mask_token=None,
                  enable_mask_opt=True, use_ground_truth=False, enable_panoptic=False, noise_s=None):
        if mask_token is not None and not self.predict_x0:
            raise NotImplementedError("the mask co-update is only defined for predict_x0=True")
        opt = enable_mask_opt and mask_token is not None
        stages = sc.step_stages(self.noise_schedule._host, _scalar(s), _scalar(t), order, self.predict_x0, r1, r2,
                                solver_type, opt)
        B = x.shape[0]
        ms, pms = [], []
        x_in, m_in = x, mask_token
        pm0 = None
        for k, st in enumerate(stages):
            tvec = torch.full((B,), st["time"], dtype=torch.float32, device=x.device)
            if k == 0 and noise_s is not None:
                out, pm = noise_s, panoptic
            else:
                out, pm = self._call_model(x_in, tvec, panoptic, m_in, use_ground_truth, enable_panoptic)
            if self.predict_x0:
                m = self._data_pred(x_in, tvec, out)
            else:
                m = out.float()
            ms.append(m)
            pms.append(pm)
            if k == 0:
                pm0 = pm
            x_in = _lin([x] + ms, [st["nx"]] + st["nm"] + [st["cm"]])
            mk = st["mask"]
            if mask_token is not None:
                if mk == "pred":
                    m_in = pm0
                elif opt:
                    m_in = _lin([mask_token] + pms, [mk["mx"]] + mk["mm"] + [mk["mc"]])
                else:
                    m_in = mask_token
        return x_in, pm0, m_in

    def dpm_solver_first_update(self, x, s, t, noise_s=None, return_noise=False, panoptic=None, mask_token=None,
                                enable_mask_opt=True, use_ground_truth=False, enable_panoptic=False):
        x_t, pm, mt = self._run_step(x, s, t, 1, panoptic=panoptic, mask_token=mask_token,
                                     enable_mask_opt=enable_mask_opt, use_ground_truth=use_ground_truth,
                                     enable_panoptic=enable_panoptic, noise_s=noise_s)
        return (x_t, {'noise_s': noise_s}) if return_noise else (x_t, pm, mt)

    def dpm_solver_second_update(self, x, s, t, r1=0.5, noise_s=None, return_noise=False, solver_type='dpm_solver',
                                 panoptic=None, mask_token=None, enable_mask_opt=True, use_ground_truth=False,
                                 enable_panoptic=False):
        x_t, pm, mt = self._run_step(x, s, t, 2, r1=r1, solver_type=solver_type, panoptic=panoptic,
                                     mask_token=mask_token, enable_mask_opt=enable_mask_opt,
                                     use_ground_truth=use_ground_truth, enable_panoptic=enable_panoptic,
                                     noise_s=noise_s)
        return (x_t, {'noise_s': noise_s}) if return_noise else (x_t, pm, mt)

    def dpm_solver_third_update(self, x, s, t, r1=1. / 3., r2=2. / 3., noise_s=None, noise_s1=None, noise_s2=None,
                                return_noise=False, solver_type='dpm_solver', panoptic=None, mask_token=None,
                                enable_mask_opt=True, use_ground_truth=False, enable_panoptic=False):
        if noise_s1 is not None or noise_s2 is not None:
            raise NotImplementedError("precomputed noise_s1 / noise_s2 (adaptive solver only)")
        x_t, pm, mt = self._run_step(x, s, t, 3, r1=r1, r2=r2, solver_type=solver_type, panoptic=panoptic,
                                     mask_token=mask_token, enable_mask_opt=enable_mask_opt,
                                     use_ground_truth=use_ground_truth, enable_panoptic=enable_panoptic,
                                     noise_s=noise_s)
        return (x_t, {'noise_s': noise_s}) if return_noise else (x_t, pm, mt)

    def dpm_solver_update(self, x, s, t, order, return_noise=False, solver_type='dpm_solver', r1=None, r2=None,
                          panoptic=None, mask_token=None, enable_mask_opt=True, use_ground_truth=False,
                          enable_panoptic=False):
        if order not in (1, 2, 3):
            raise ValueError("Solver order must be 1 or 2 or 3, got {}".format(order))
        return self._run_step(x, s, t, order, r1=r1, r2=r2, solver_type=solver_type, panoptic=panoptic,
                              mask_token=mask_token, enable_mask_opt=enable_mask_opt,
                              use_ground_truth=use_ground_truth, enable_panoptic=enable_panoptic)

    def dpm_multistep_update(self, *args, **kwargs):
        raise NotImplementedError("multistep DPM-Solver is outside the sampling hot path (SURVEY.md §2 row 5)")

    def dpm_solver_adaptive(self, *args, **kwargs):
        raise NotImplementedError("adaptive DPM-Solver is outside the sampling hot path (SURVEY.md §2 row 5)")

    # ---- sample (dpm_solver_pp.py:927-1081) ---------------------------------------------------
    def sample(self, x, steps=10, eps=1e-4, T=None, order=3, panoptic=None, skip_type='time_uniform', denoise=False,
               method='fast', solver_type='dpm_solver', atol=0.0078, rtol=0.05, mask_token=None, use_twophases=False,
               use_ground_truth=False, enable_panoptic=False, enable_mask_opt=False, return_tuple=None):
        _lib.require_gpu(x)
        t_0 = eps
        t_T = self.noise_schedule.T if T is None else T
        hs = self.noise_schedule._host
        if method in ('adaptive', 'multistep'):
            raise NotImplementedError(f"method={method!r} is outside the sampling hot path (SURVEY.md §2 row 5)")
        if method == 'fast':
            orders, _ = sc.fast_orders(steps, order)
            ts = sc.time_steps(hs, skip_type, t_T, t_0, steps)
            spans = []
            i = 0
            for o in orders:
                h = sc.lam(hs, ts[i + o]) - sc.lam(hs, ts[i])
                r1 = None if o <= 1 else (sc.lam(hs, ts[i + 1]) - sc.lam(hs, ts[i])) / h
                r2 = None if o <= 2 else (sc.lam(hs, ts[i + 2]) - sc.lam(hs, ts[i])) / h
                spans.append((ts[i], ts[i + o], o, r1, r2))
                i += o
        elif method == 'singlestep':
            n = steps // order
            ts = sc.time_steps(hs, skip_type, t_T, t_0, n)
            spans = [(ts[i], ts[i + 1], order, None, None) for i in range(n)]
        else:
            raise ValueError(f"Unsupported method {method}")
        x = x.float()
        pred_mask = mask_token.to(x.device) if mask_token is not None else None
        mask_t = pred_mask
        with torch.no_grad():
            for s, t, o, r1, r2 in spans:
                B = x.shape[0]
                vs = torch.full((B,), s, dtype=torch.float32, device=x.device)
                vt = torch.full((B,), t, dtype=torch.float32, device=x.device)
                x, pred_mask, mask_t = self._run_step(x, vs, vt, o, r1=r1, r2=r2, solver_type=solver_type,
                                                      panoptic=pred_mask, mask_token=mask_t,
                                                      enable_mask_opt=enable_mask_opt,
                                                      use_ground_truth=use_ground_truth,
                                                      enable_panoptic=enable_panoptic)
            if method == 'singlestep' and use_twophases:
                for s, t, o, r1, r2 in spans:
                    B = x.shape[0]
                    vs = torch.full((B,), s, dtype=torch.float32, device=x.device)
                    vt = torch.full((B,), t, dtype=torch.float32, device=x.device)
                    x, _, _ = self._run_step(x, vs, vt, o, solver_type=solver_type, panoptic=panoptic,
                                             mask_token=mask_t, enable_mask_opt=False, use_ground_truth=True,
                                             enable_panoptic=True)
            if denoise:
                x = self.denoise_fn(x, torch.full((x.shape[0],), t_0, device=x.device))
        want_tuple = (mask_token is not None) if return_tuple is None else return_tuple
        return (x, pred_mask) if want_tuple else x

"""Original DPM-Solver (noise prediction, continuous VP schedules) — API of dpm_solver_pytorch.py.

Used by the U-ViT-L/2 and CIFAR callers (eval_ldm.py:94-108, eval.py:72-86).  Same design as
dpm_solver_pp: host float64 coefficients (solver_core), GPU linear combinations through libpdm, the model
is the caller's `model_fn`.  Adaptive step size is outside the hot path (never used by the callers) and
raises NotImplementedError.
"""
import torch

from . import _lib
from . import solver_core as sc
from .dpm_solver_pp import _lin, _scalar
from .dpm_solver_pp import model_wrapper as _pp_model_wrapper


class NoiseScheduleVP:
    """dpm_solver_pytorch.py:6-102: 'linear' (beta 0.1 .. 20) or 'cosine'."""

    def __init__(self, schedule='linear'):
        if schedule not in ['linear', 'cosine']:
            raise ValueError("Unsupported noise schedule {}. The schedule needs to be 'linear' or 'cosine'".format(schedule))
        self.schedule = schedule
        self.beta_0, self.beta_1 = 0.1, 20
        self._host = sc.HostLinear(0.1, 20.0) if schedule == 'linear' else sc.HostCosine()
        self.cosine_s = 0.008
        self.cosine_beta_max = 999.
        self.cosine_log_alpha_0 = self._host.la0 if schedule == 'cosine' else sc.HostCosine().la0
        self.T = self._host.T

    def marginal_log_mean_coeff(self, t):
        if self.schedule == 'linear':
            return -0.25 * t ** 2 * (self.beta_1 - self.beta_0) - 0.5 * t * self.beta_0
        s = self.cosine_s
        return torch.log(torch.cos((t + s) / (1. + s) * torch.pi / 2.)) - self.cosine_log_alpha_0

    def marginal_std(self, t):
        return torch.sqrt(1. - torch.exp(2. * self.marginal_log_mean_coeff(t)))

    def marginal_lambda(self, t):
        lm = self.marginal_log_mean_coeff(t)
        return lm - 0.5 * torch.log(1. - torch.exp(2. * lm))

    def inverse_lambda(self, lamb):
        zero = torch.zeros((1,)).to(lamb)
        if self.schedule == 'linear':
            tmp = 2. * (self.beta_1 - self.beta_0) * torch.logaddexp(-2. * lamb, zero)
            return tmp / (torch.sqrt(self.beta_0 ** 2 + tmp) + self.beta_0) / (self.beta_1 - self.beta_0)
        la = -0.5 * torch.logaddexp(-2. * lamb, zero)
        s = self.cosine_s
        return torch.arccos(torch.exp(la + self.cosine_log_alpha_0)) * 2. * (1. + s) / torch.pi - s


def model_wrapper(model, noise_schedule=None, is_cond_classifier=False, classifier_fn=None, classifier_scale=1.,
                  time_input_type='1', total_N=1000, model_kwargs={}):
    """dpm_solver_pytorch.py:105-218 (same behaviour as the pp wrapper)."""
    return _pp_model_wrapper(model, noise_schedule, is_cond_classifier, classifier_fn, classifier_scale,
                             time_input_type, total_N, model_kwargs)


class DPM_Solver:
    def __init__(self, model_fn, noise_schedule):
        self.model_fn = model_fn
        self.noise_schedule = noise_schedule

    def get_time_steps(self, skip_type, t_T, t_0, N, device):
        return torch.tensor(sc.time_steps(self.noise_schedule._host, skip_type, t_T, t_0, N),
                            dtype=torch.float32).to(device)

    def get_time_steps_for_dpm_solver_fast(self, t_T, t_0, steps, device):
        orders, K = sc.fast_orders(steps, 3)
        return orders, self.get_time_steps('logSNR', t_T, t_0, K, device)

    def _step(self, x, s, t, order, r1=None, r2=None, noise_s=None):
        stages = sc.step_stages(self.noise_schedule._host, _scalar(s), _scalar(t), order, predict_x0=False,
                                r1=r1, r2=r2)
        B = x.shape[0]
        ms = []
        x_in = x
        for k, st in enumerate(stages):
            if k == 0 and noise_s is not None:
                e = noise_s
            else:
                e = self.model_fn(x_in, torch.full((B,), st["time"], dtype=torch.float32, device=x.device))
            ms.append(e.float())
            x_in = _lin([x] + ms, [st["nx"]] + st["nm"] + [st["cm"]])
        return x_in

    def dpm_solver_first_update(self, x, s, t, return_noise=False):
        return self._step(x, s, t, 1)

    def dpm_solver_second_update(self, x, s, t, r1=0.5, noise_s=None, return_noise=False):
        return self._step(x, s, t, 2, r1=r1, noise_s=noise_s)

    def dpm_solver_third_update(self, x, s, t, r1=1. / 3., r2=2. / 3., noise_s=None, noise_s1=None, noise_s2=None):
        if noise_s1 is not None or noise_s2 is not None:
            raise NotImplementedError("precomputed noise_s1 / noise_s2 (adaptive solver only)")
        return self._step(x, s, t, 3, r1=r1, r2=r2, noise_s=noise_s)

    def dpm_solver_update(self, x, s, t, order):
        if order not in (1, 2, 3):
            raise ValueError("Solver order must be 1 or 2 or 3, got {}".format(order))
        return self._step(x, s, t, order)

    def dpm_solver_adaptive(self, *args, **kwargs):
        raise NotImplementedError("adaptive DPM-Solver is outside the sampling hot path (SURVEY.md §2 row 6)")

    def sample(self, x, steps=10, eps=1e-4, T=None, order=3, skip_type='logSNR', adaptive_step_size=False,
               fast_version=True, atol=0.0078, rtol=0.05):
        _lib.require_gpu(x)
        if adaptive_step_size:
            raise NotImplementedError("adaptive DPM-Solver is outside the sampling hot path (SURVEY.md §2 row 6)")
        hs = self.noise_schedule._host
        t_0, t_T = eps, (self.noise_schedule.T if T is None else T)
        plan = sc.pt_fast_plan(hs, steps, t_0, t_T) if fast_version else sc.pt_plan(hs, steps, t_0, t_T, order, skip_type)
        x = x.float()
        with torch.no_grad():
            for stages in plan:
                B = x.shape[0]
                ms = []
                x0 = x
                x_in = x
                for st in stages:
                    e = self.model_fn(x_in, torch.full((B,), st["time"], dtype=torch.float32, device=x.device))
                    ms.append(e.float())
                    x_in = _lin([x0] + ms, [st["nx"]] + st["nm"] + [st["cm"]])
                x = x_in
        return x

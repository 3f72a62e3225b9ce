"""VP-SDE bookkeeping and ScoreModel — the hot-path subset of sde.py (VPSDE 72-113, ScoreModel 155-199).

`ScoreModel.predict` feeds the net `t * 999` (sde.py:174); `noise_pred` is what eval_ldm.py / eval.py hand
to dpm_solver_pytorch.model_wrapper.  The Euler-Maruyama sampler and LSimple (training) are outside the
sampling hot path.
"""
import numpy as np
import torch


def stp(s, ts):
    """scalar-tensor product broadcasting s [B] over ts [B, ...] (sde.py:18-22)."""
    if isinstance(s, np.ndarray):
        s = torch.from_numpy(s).type_as(ts)
    return s.view(-1, *([1] * (ts.dim() - 1))) * ts


def mos(a, start_dim=1):
    return a.pow(2).flatten(start_dim=start_dim).mean(dim=-1)


def duplicate(tensor, *size):
    return tensor.unsqueeze(dim=0).expand(*size, *tensor.shape)


class VPSDE:
    """Linear VP-SDE, beta(t) = beta_0 + t (beta_1 - beta_0)."""

    def __init__(self, beta_min=0.1, beta_max=20):
        self.beta_0, self.beta_1 = beta_min, beta_max

    def squared_diffusion(self, t):
        return self.beta_0 + t * (self.beta_1 - self.beta_0)

    def diffusion(self, t):
        return self.squared_diffusion(t) ** 0.5

    def drift(self, x, t):
        return -0.5 * stp(self.squared_diffusion(t), x)

    def squared_diffusion_integral(self, s, t):
        return self.beta_0 * (t - s) + (self.beta_1 - self.beta_0) * (t ** 2 - s ** 2) * 0.5

    def skip_alpha(self, s, t):
        return (-self.squared_diffusion_integral(s, t)).exp()

    def skip_beta(self, s, t):
        return 1. - self.skip_alpha(s, t)

    def cum_alpha(self, t):
        return self.skip_alpha(0, t)

    def cum_beta(self, t):
        return self.skip_beta(0, t)

    def nsr(self, t):
        return self.squared_diffusion_integral(0, t).expm1()

    def snr(self, t):
        return 1. / self.nsr(t)

    def marginal_prob(self, x0, t):
        return stp(self.cum_alpha(t) ** 0.5, x0), self.cum_beta(t) ** 0.5

    def __repr__(self):
        return f'vpsde beta_0={self.beta_0} beta_1={self.beta_1}'

    __str__ = __repr__


class ScoreModel:
    def __init__(self, nnet, pred, sde, T=1):
        assert T == 1
        self.nnet, self.pred, self.sde, self.T = nnet, pred, sde, T

    def predict(self, xt, t, **kwargs):
        if not isinstance(t, torch.Tensor):
            t = torch.tensor(t)
        t = t.to(xt.device)
        if t.dim() == 0:
            t = duplicate(t, xt.size(0))
        return self.nnet(xt, t * 999, **kwargs)

    def noise_pred(self, xt, t, **kwargs):
        pred = self.predict(xt, t, **kwargs)
        if self.pred == 'noise_pred':
            return pred
        if self.pred == 'x0_pred':
            return -stp(self.sde.snr(t).sqrt(), pred) + stp(self.sde.cum_beta(t).rsqrt(), xt)
        raise NotImplementedError(self.pred)

    def x0_pred(self, xt, t, **kwargs):
        pred = self.predict(xt, t, **kwargs)
        if self.pred == 'noise_pred':
            return stp(self.sde.cum_alpha(t).rsqrt(), xt) - stp(self.sde.nsr(t).sqrt(), pred)
        if self.pred == 'x0_pred':
            return pred
        raise NotImplementedError(self.pred)

    def score(self, xt, t, **kwargs):
        return stp(-self.sde.cum_beta(t).rsqrt(), self.noise_pred(xt, t, **kwargs))

"""LSimple training step on the HIP path.

Restates, behind the reference's own names, what one training iteration does:
  * `Schedule` / `stable_diffusion_beta_schedule` / `LSimple` — train_ldm_discrete.py:23-27,54-90 (discrete SD
    betas, n ~ U{1..1000}, xn = sqrt(a_n) x0 + sqrt(1 - a_n) eps, loss = mos(eps - nnet(xn, n, y)));
  * `LSimple_sde` — sde.py:64-69,270-279 with ScoreModel.noise_pred (sde.py:168-184): t ~ U(0, 1), the VPSDE
    marginal, the net sees t * 999 (train_ldm.py, the U-ViT-L/2 config);
  * `HipTrainState.train_step` — train_ldm_discrete.py:159-175: zero_grad, loss.mean().backward(), AdamW step
    (utils.get_optimizer, torch.optim.AdamW semantics), the `customized` warm-up LR (utils.py:319-326), then the
    EMA update (utils.py:339-345, rate config.ema_rate, default 0.9999);
  * label dropout for classifier-free guidance — datasets.py:45-61 CFGDataset (p_uncond, the null label);
  * the panoptic t2i step — train_t2i_discrete.py:111-142 (Schedule.sample with a mask: eps_m = 2 randn, mask_n),
    148-224 (LSimple: analog bits utils.int2bits * 2 - 1, nnet(xn, n, context, mask_token=mask_n), loss_eps and
    loss_mask = mos(mask_pred - bits)), 446-473 (loss_eps.mean() + loss_mask.mean() backpropagated).
The noise draw (n / t, eps) is host-side torch RNG, as in the reference; the network forward, the loss, the whole
backward and the optimizer run on libpdm's HIP kernels (csrc/train.hip, csrc/train_kernels.hip).  Data parallel:
one process per GPU, the gradient buffer all-reduced (average, RCCL) between backward and optimizer step — the
DDP semantics accelerate gives the reference (train_ldm_discrete.py:130-132).
"""
import ctypes

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .native import cfg_struct
from .sde import VPSDE, mos, stp


def stable_diffusion_beta_schedule(linear_start=0.00085, linear_end=0.0120, n_timestep=1000):
    """train_ldm_discrete.py:23-27."""
    return (torch.linspace(linear_start ** 0.5, linear_end ** 0.5, n_timestep, dtype=torch.float64) ** 2).numpy()


class Schedule:
    """Discrete-time forward process (train_ldm_discrete.py:54-84): betas[0] = 0, cum_alphas = prod(1 - betas)."""

    def __init__(self, _betas):
        self._betas = _betas
        self.betas = np.append(0., _betas)
        self.alphas = 1. - self.betas
        self.N = len(_betas)
        self.cum_alphas = self.alphas.cumprod()
        self.cum_betas = 1. - self.cum_alphas

    def sample(self, x0, rng=None, panoptic=None):
        """(n, eps, xn), n uniform in {1..N} (np.random.choice as the reference; `rng` a numpy Generator /
        RandomState for reproducible draws), eps ~ N(0, 1).  With the scaled analog-bit mask `panoptic`
        (train_t2i_discrete.py:130-142) also (eps_m, mask_n): eps_m = 2 N(0, 1), mask_n noised like xn."""
        choice = (rng or np.random).choice
        n = choice(list(range(1, self.N + 1)), (len(x0),))
        eps = torch.randn_like(x0)
        xn = stp(self.cum_alphas[n] ** 0.5, x0) + stp(self.cum_betas[n] ** 0.5, eps)
        if panoptic is None:
            return torch.tensor(n, device=x0.device), eps, xn
        eps_m = 2.0 * torch.randn_like(panoptic)
        mask_n = stp(self.cum_alphas[n] ** 0.5, panoptic) + stp(self.cum_betas[n] ** 0.5, eps_m)
        return torch.tensor(n, device=x0.device), eps, xn, eps_m, mask_n


def int2bits(x, n=8):
    """utils.int2bits (utils.py:475-488): integer masks (b, 1, h, w) -> float bits (b, n, h, w), channel 0 the most
    significant bit."""
    x = x.to(torch.int64)
    return torch.remainder(torch.cat([torch.bitwise_right_shift(x, i) for i in range(n - 1, -1, -1)], 1), 2).float()


def drop_labels(y, p_uncond, null_label, generator=None):
    """CFGDataset (datasets.py:45-61): each label replaced by the null class with probability p_uncond."""
    if not p_uncond:
        return y
    r = torch.rand(y.shape, generator=generator, device=y.device if generator is None else "cpu").to(y.device)
    return torch.where(r < p_uncond, torch.full_like(y, null_label), y)


def customized_lr(base_lr, step, warmup_steps=-1):
    """utils.customized_lr_scheduler (utils.py:319-326): LambdaLR factor min(step / warmup, 1) at scheduler step
    `step` (the number of optimizer steps already taken)."""
    return base_lr * (min(step / warmup_steps, 1) if warmup_steps > 0 else 1)


class HipTrainState:
    """Parameters, gradients, AdamW moments and the EMA copy of one U-ViT in flat device buffers (pdm_train_*).

    `state_dict()` / `ema_state_dict()` hand back reference-keyed tensors (views copied out), so checkpoints
    interoperate with utils.TrainState's nnet / nnet_ema files."""

    def __init__(self, nnet_kwargs, device="cuda", optimizer=None, lr_scheduler=None, ema_rate=0.9999, lanes=1):
        """lanes=2 splits each batch into two halves run concurrently on their own streams (a second pdm_train
        handle sharing the parameters and bf16 copies, with its own workspace and gradient buffer; AdamW sums the
        two), so one half's GEMM tiles fill the CUs the other half's partly filled last wave leaves idle -- the
        sampler lanes (sampler.py) applied to the training step."""
        _lib.require_gpu()
        kw = dict(nnet_kwargs)
        name = kw.pop("name", "uvit")
        if name not in ("uvit", "uvit_t2i"):
            raise ValueError(f"HipTrainState: libs/uvit.py or libs/uvit_t2i.py networks, not {name!r}")
        self.t2i = name == "uvit_t2i"
        self.kw = kw
        self.device = torch.device(device)
        self.lib = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(self.lib.pdm_train_create(ctypes.byref(cfg_struct(kw, self.t2i)), ctypes.byref(h)),
                   "pdm_train_create")
        self.h = h
        n, nwt = ctypes.c_longlong(), ctypes.c_longlong()
        _lib.check(self.lib.pdm_train_sizes(h, ctypes.byref(n), ctypes.byref(nwt)), "pdm_train_sizes")
        self.n = n.value
        self.index = {}
        buf = ctypes.create_string_buffer(256)
        for i in range(self.lib.pdm_train_param_count(h)):
            off, numel = ctypes.c_longlong(), ctypes.c_longlong()
            _lib.check(self.lib.pdm_train_param_info(h, i, buf, 256, ctypes.byref(off), ctypes.byref(numel)))
            self.index[buf.value.decode()] = (off.value, numel.value)
        dev = self.device
        self.P = torch.zeros(self.n, dtype=torch.float32, device=dev)
        self.G = torch.zeros(self.n, dtype=torch.float32, device=dev)
        self.M = torch.zeros(self.n, dtype=torch.float32, device=dev)
        self.V = torch.zeros(self.n, dtype=torch.float32, device=dev)
        self.E = torch.zeros(self.n, dtype=torch.float32, device=dev)
        self.WB = torch.zeros(self.n, dtype=torch.bfloat16, device=dev)
        self.WT = torch.zeros(max(nwt.value, 1), dtype=torch.bfloat16, device=dev)
        _lib.check(self.lib.pdm_train_set_buffers(h, _lib.ptr(self.P), _lib.ptr(self.G), _lib.ptr(self.WB),
                                                  _lib.ptr(self.WT)), "pdm_train_set_buffers")
        self.optimizer = dict(name="adamw", lr=2e-4, weight_decay=0.03, betas=(0.99, 0.99), eps=1e-8)
        self.optimizer.update(optimizer or {})
        if self.optimizer["name"] != "adamw":
            raise NotImplementedError(self.optimizer["name"])
        self.lr_scheduler = dict(name="customized", warmup_steps=-1)
        self.lr_scheduler.update(lr_scheduler or {})
        if self.lr_scheduler["name"] != "customized":
            raise NotImplementedError(self.lr_scheduler["name"])
        self.ema_rate = ema_rate
        self.step = 0
        self.shapes = {}
        self.ws = None
        self.lanes = max(1, min(2, int(lanes)))
        self.h2 = self.G2 = self.ws2 = None
        self._streams = []
        if self.lanes == 2:
            h2 = ctypes.c_void_p()
            _lib.check(self.lib.pdm_train_create(ctypes.byref(cfg_struct(kw, self.t2i)), ctypes.byref(h2)),
                       "pdm_train_create")
            self.h2 = h2
            self.G2 = torch.zeros(self.n, dtype=torch.float32, device=dev)
            _lib.check(self.lib.pdm_train_set_buffers(h2, _lib.ptr(self.P), _lib.ptr(self.G2), _lib.ptr(self.WB),
                                                      _lib.ptr(self.WT)), "pdm_train_set_buffers")
            self._streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]

    def __del__(self):
        try:
            if getattr(self, "h", None):
                self.lib.pdm_train_destroy(self.h)
            if getattr(self, "h2", None):
                self.lib.pdm_train_destroy(self.h2)
        except Exception:
            pass

    # ---- parameters ----------------------------------------------------------------------------------------
    def _view(self, flat, name):
        off, numel = self.index[name]
        return flat[off: off + numel].view(self.shapes.get(name, (numel,)))

    def load_state_dict(self, sd, ema_sd=None):
        """Reference-keyed state_dict -> parameters (strict), bf16 working copies; the EMA copy starts equal to the
        parameters (utils.initialize_train_state: ema_update(0)) unless ema_sd is given."""
        missing = set(self.index) - set(sd)
        extra = set(sd) - set(self.index)
        if missing or extra:
            raise KeyError(f"state_dict mismatch: missing {sorted(missing)[:5]}, unexpected {sorted(extra)[:5]}")
        with torch.no_grad():
            for k, v in sd.items():
                self.shapes[k] = tuple(v.shape)
                self._view(self.P, k).copy_(v.to(self.device, torch.float32).view(self.shapes[k]))
            self.E.copy_(self.P)
            if ema_sd is not None:
                for k, v in ema_sd.items():
                    self._view(self.E, k).copy_(v.to(self.device, torch.float32))
        _lib.check(self.lib.pdm_train_refresh(self.h, _lib.stream_ptr(self.device)), "pdm_train_refresh")

    def state_dict(self):
        return {k: self._view(self.P, k).clone() for k in self.index}

    def ema_state_dict(self):
        return {k: self._view(self.E, k).clone() for k in self.index}

    def grads(self):
        g = self.G + self.G2 if self.G2 is not None else self.G
        return {k: self._view(g, k).clone() for k in self.index}

    # ---- one step --------------------------------------------------------------------------------------------
    def _workspace(self, rows, lane=0):
        need = ctypes.c_size_t()
        _lib.check(self.lib.pdm_train_workspace_size(self.h, rows, ctypes.byref(need)), "pdm_train_workspace_size")
        ws = self.ws if lane == 0 else self.ws2
        if ws is None or ws.numel() < need.value:
            ws = None
            if lane == 0:
                self.ws = None
            else:
                self.ws2 = None
            ws = torch.empty(need.value, dtype=torch.uint8, device=self.device)
            if lane == 0:
                self.ws = ws
            else:
                self.ws2 = ws
        return ws

    def _step_call(self, h, xt, t_in, y, target, loss, gscale, ws, stream):
        B = xt.shape[0]
        _lib.check(self.lib.pdm_train_step(h, _lib.ptr(xt), _lib.ptr(t_in), _lib.ptr(y), _lib.ptr(target),
                                           _lib.ptr(loss), B, float(gscale), _lib.ptr(ws), ws.numel(),
                                           ctypes.c_void_p(stream.cuda_stream)), "pdm_train_step")

    def forward_backward(self, xt, t_in, y, target, gscale=None):
        """loss[b] = mos(target - nnet(xt, t_in, y)) and d(gscale * sum(loss)) / d(params) into the gradient buffer
        (gscale default 1/B = loss.mean()).  Returns the per-sample losses."""
        B = xt.shape[0]
        xt = xt.to(self.device, torch.float32).contiguous()
        target = target.to(self.device, torch.float32).contiguous()
        t_in = t_in.to(self.device, torch.float32).contiguous().reshape(B)
        if y is not None:
            # the reference's nn.Embedding raises IndexError on an out-of-range label; the kernels would read the
            # neighbouring parameter (pos_embed) as the embedding and scatter its gradient there.  Host labels (the
            # data loader's) are checked here; device-resident labels are clamped into range on the stream (the
            # kernels never read outside label_emb) and their range error is kept in a device flag that
            # _raise_label_error reads once the step that set it has finished -- no synchronisation per step
            nc = int(self.kw.get("num_classes", -1))
            if nc <= 0:
                raise ValueError("HipTrainState: labels given to an unconditional U-ViT (num_classes <= 0)")
            self._raise_label_error(block=False)
            if y.numel() and y.device.type == "cpu":
                lo, hi = (int(v) for v in torch.stack([y.min(), y.max()]).cpu())
                if lo < 0 or hi >= nc:
                    raise IndexError(f"HipTrainState: label out of range [0, {nc}): min {lo}, max {hi}")
                y = y.to(self.device, torch.int64).contiguous()
            elif y.numel():
                y = y.to(self.device, torch.int64)
                bad = ((y < 0) | (y >= nc)).any()
                self._label_bad = bad if getattr(self, "_label_bad", None) is None else self._label_bad | bad
                self._label_ev = torch.cuda.Event()
                self._label_ev.record(torch.cuda.current_stream(self.device))
                y = y.clamp(0, nc - 1).contiguous()
            else:
                y = y.to(self.device, torch.int64).contiguous()
        gs = float(1.0 / B if gscale is None else gscale)
        loss = torch.empty(B, dtype=torch.float32, device=self.device)
        self._lanes(B, lambda h, a, b, ws, s: self._step_call(h, xt[a:b], t_in[a:b], y[a:b] if y is not None else None,
                                                              target[a:b], loss[a:b], gs, ws, s),
                    (xt, t_in, target, loss) + ((y,) if y is not None else ()))
        return loss

    def _raise_label_error(self, block=True):
        """IndexError if a device-resident label of an earlier step was out of range [0, num_classes) (those steps ran
        on clamped labels).  block=False reads the flag only once the step that set it has finished."""
        bad = getattr(self, "_label_bad", None)
        if bad is None or (not block and not self._label_ev.query()):
            return
        self._label_bad = None
        if bool(bad):
            raise IndexError(f"HipTrainState: a device label of an earlier step was out of range "
                             f"[0, {int(self.kw.get('num_classes', -1))}) (that step ran on clamped labels)")

    check_labels = _raise_label_error

    def _lanes(self, B, call, tensors):
        """call(handle, row0, row1, workspace, stream) for the whole batch on the current stream, or (lanes = 2) for
        its two halves on the lanes' own streams, joined back into the current stream."""
        cur = torch.cuda.current_stream(self.device)
        if self.lanes == 1 or B < 2:
            if self.G2 is not None:
                self.G2.zero_()
            call(self.h, 0, B, self._workspace(B), cur)
            return
        h0 = B // 2
        ready = torch.cuda.Event()
        ready.record(cur)
        for lane, (a, b) in enumerate([(0, h0), (h0, B)]):
            s = self._streams[lane]
            s.wait_event(ready)
            ws = self._workspace(b - a, lane)
            with torch.cuda.stream(s):
                call(self.h if lane == 0 else self.h2, a, b, ws, s)
            done = torch.cuda.Event()
            done.record(s)
            cur.wait_event(done)
            for t in tuple(tensors) + (ws,):
                t.record_stream(s)

    def forward_backward_t2i(self, xt, t_in, context, mask_token, target, mask_target, gscale=None):
        """The panoptic t2i step (pdm_train_step_t2i): loss[b] = mos(target - eps_pred), loss_mask[b] =
        mos(mask_pred - mask_target) and d(gscale * sum(loss + loss_mask)) / d(params) into the gradient buffer
        (gscale default 1/B: loss_eps.mean() + loss_mask.mean()).  Returns (loss, loss_mask)."""
        if not self.t2i:
            raise ValueError("forward_backward_t2i: not a t2i trainer")
        B = xt.shape[0]
        f32 = lambda v: v.to(self.device, torch.float32).contiguous()
        xt, target, context, mask_token, mask_target = (f32(v) for v in (xt, target, context, mask_token, mask_target))
        t_in = f32(t_in).reshape(B)
        gs = float(1.0 / B if gscale is None else gscale)
        loss = torch.empty(B, dtype=torch.float32, device=self.device)
        loss_m = torch.empty(B, dtype=torch.float32, device=self.device)

        def call(h, a, b, ws, s):
            _lib.check(self.lib.pdm_train_step_t2i(h, _lib.ptr(xt[a:b]), _lib.ptr(t_in[a:b]), _lib.ptr(context[a:b]),
                                                   _lib.ptr(mask_token[a:b]), _lib.ptr(target[a:b]),
                                                   _lib.ptr(mask_target[a:b]), _lib.ptr(loss[a:b]),
                                                   _lib.ptr(loss_m[a:b]), b - a, gs, _lib.ptr(ws), ws.numel(),
                                                   ctypes.c_void_p(s.cuda_stream)), "pdm_train_step_t2i")
        self._lanes(B, call, (xt, t_in, context, mask_token, target, mask_target, loss, loss_m))
        return loss, loss_m

    def all_reduce_grads(self):
        """DDP: average the gradient buffer over the process group (RCCL on the GPU); with two lanes the second
        lane's gradients are folded in first (at world size 1 AdamW sums the two buffers itself)."""
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            if self.G2 is not None:
                self.G.add_(self.G2)
                self.G2.zero_()
            average_gradients(self.G)

    def optimizer_step(self):
        """AdamW at the current scheduled LR, then the EMA update; advances the step counter.  Returns the LR this
        step applied (train_step reports the next one, as the reference logs it)."""
        o = self.optimizer
        lr = customized_lr(o["lr"], self.step, self.lr_scheduler.get("warmup_steps", -1))
        b1, b2 = o["betas"]
        _lib.check(self.lib.pdm_train_adamw(self.h, _lib.ptr(self.M), _lib.ptr(self.V), _lib.ptr(self.E),
                                            _lib.ptr(self.G2), float(lr),
                                            float(b1), float(b2), float(o.get("eps", 1e-8)), float(o["weight_decay"]),
                                            self.step + 1, float(self.ema_rate), _lib.stream_ptr(self.device)),
                   "pdm_train_adamw")
        self.step += 1
        return lr

    def current_lr(self):
        """The rate the next optimizer_step applies (optimizer.param_groups[0]['lr'] after lr_scheduler.step())."""
        return customized_lr(self.optimizer["lr"], self.step, self.lr_scheduler.get("warmup_steps", -1))

    def train_step(self, x0, y=None, objective="discrete", schedule=None, sde=None, rng=None, context=None,
                   panoptic=None):
        """One iteration of train_ldm_discrete.py:159-175 (objective 'discrete', Schedule) or train_ldm.py
        (objective 'sde', VPSDE + noise_pred); a t2i trainer runs train_t2i_discrete.py:446-478 on (x0, context,
        panoptic integer masks).  Returns dict(loss=mean loss over the global batch, lr=...) (+ loss_mask)."""
        if self.t2i:
            schedule = schedule or Schedule(stable_diffusion_beta_schedule())
            scaled = int2bits(panoptic).to(x0.device) * 2.0 - 1.0
            n, eps, xn, eps_m, mask_n = schedule.sample(x0, rng, panoptic=scaled)
            loss, loss_m = self.forward_backward_t2i(xn, n.float(), context, mask_n, eps, scaled)
            self.all_reduce_grads()
            self.optimizer_step()
            ms = torch.stack([loss.mean(), loss_m.mean()])
            if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
                dist.all_reduce(ms, op=dist.ReduceOp.SUM)
                ms /= dist.get_world_size()
            return dict(loss=ms[0], loss_mask=ms[1], lr=self.current_lr())
        if objective == "discrete":
            schedule = schedule or Schedule(stable_diffusion_beta_schedule())
            n, eps, xn = schedule.sample(x0, rng)
            loss = self.forward_backward(xn, n.float(), y, eps)
        elif objective == "sde":
            t, eps, xt = LSimple_sde_sample(sde or VPSDE(), x0)
            loss = self.forward_backward(xt, t * 999, y, eps)
        else:
            raise NotImplementedError(objective)
        self.all_reduce_grads()
        self.optimizer_step()
        m = loss.mean()
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(m, op=dist.ReduceOp.SUM)
            m /= dist.get_world_size()
        # the reference returns optimizer.param_groups[0]['lr'] read after lr_scheduler.step()
        # (train_ldm_discrete.py:174-177): the rate of the NEXT step
        return dict(loss=m, lr=self.current_lr())


def average_gradients(g):
    """All-reduce-average a flat gradient tensor over the default process group (no-op at world size 1)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(g, op=dist.ReduceOp.SUM)
        g /= dist.get_world_size()
    return g


def LSimple_sde_sample(sde, x0, t_init=0):
    """SDE.sample (sde.py:64-69): t ~ U(t_init, 1), xt = sqrt(cum_alpha(t)) x0 + sqrt(cum_beta(t)) eps."""
    t = torch.rand(x0.shape[0], device=x0.device) * (1. - t_init) + t_init
    mean = stp(sde.cum_alpha(t) ** 0.5, x0)
    std = sde.cum_beta(t) ** 0.5
    eps = torch.randn_like(x0)
    return t, eps, mean + stp(std, eps)


def LSimple(x0, nnet, schedule, **kwargs):
    """train_ldm_discrete.py:87-90 on any callable net (e.g. the HIP U-ViT's forward): per-sample losses."""
    n, eps, xn = schedule.sample(x0)
    eps_pred = nnet(xn, n, **kwargs)
    return mos(eps - eps_pred)


__all__ = ["Schedule", "stable_diffusion_beta_schedule", "LSimple", "LSimple_sde_sample", "HipTrainState",
           "drop_labels", "customized_lr", "average_gradients", "int2bits"]

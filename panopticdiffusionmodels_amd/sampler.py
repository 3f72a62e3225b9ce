"""Fused sampling loops: the whole DPM-Solver trajectory with classifier-free guidance on the GPU.

What the reference does per model evaluation (eval_ldm.py:66-108 / eval_ldm_discrete.py:72-102):
two `nnet` calls (cond, uncond), the CFG combine, the x0 conversion and a handful of linear combinations,
each a separate PyTorch launch, plus host syncs inside the discrete schedule.  Here one evaluation is:

  pdm_uvit_forward on the 2B-row batch [cond rows | uncond rows]   (one native call, ~130 kernels)
  pdm_stage_epilogue                                                (final conv + CFG + x0 + next input,
                                                                     written into both halves of the batch)

with every coefficient precomputed on the host (solver_core).  Nothing in the loop synchronises with the
host, so the 50-NFE loop for a fixed batch is captured once into a HIP graph and replayed.
"""

import torch

from . import _lib
from . import solver_core as sc


def sd_betas(linear_start=0.00085, linear_end=0.0120, n_timestep=1000):
    """eval_ldm_discrete.py:15-19 (fp64 -> numpy)."""
    return (torch.linspace(linear_start ** 0.5, linear_end ** 0.5, n_timestep, dtype=torch.float64) ** 2).numpy()


def build_plan(front_end, steps=50, eps=None, betas=None):
    """Returns (plan, time_scale).

    'dpm_solver_pp'      : eval_ldm_discrete.py:90-102 — discrete SD betas, predict_x0, time_uniform grid,
                           eps = 1/N, T = 1, net time = t * N.
    'dpm_solver_pytorch' : eval_ldm.py:93-108 (+ sde.ScoreModel) — linear VP, noise prediction, logSNR grid,
                           eps = 1e-4, net time = t * 999.
    """
    if front_end == "dpm_solver_pp":
        hs = sc.HostDiscrete(betas=sd_betas() if betas is None else betas)
        e = 1.0 / hs.N if eps is None else eps
        return sc.pp_fast_plan(hs, steps, e, 1.0, order=3, predict_x0=True), float(hs.N)
    if front_end == "dpm_solver_pytorch":
        hs = sc.HostLinear(0.1, 20.0)
        return sc.pt_fast_plan(hs, steps, 1e-4 if eps is None else eps, 1.0), 999.0
    raise ValueError(f"unknown solver front-end {front_end!r}")


def _drop_stale_graph(st, nnet):
    """A captured graph holds the device addresses of the net's packed weights and workspace.  Anything that
    rebuilds the native handle (load_state_dict, .to(), set_precision, set_residual) frees those, so the graph is
    dropped and recaptured on the new handle rather than replayed on freed memory; a lane's private workspace is
    re-sized for the new handle (an fp8 or fp32-residual handle needs more than the one it was sized for)."""
    handle = nnet.native()   # (re)builds the handle first, so `generation` names the one the loop will use
    if st.get("generation") != nnet.generation:
        st["graph"] = None
        if st.get("ws") is not None:
            need = handle.workspace_bytes(st["rows"])
            if st["ws"].numel() < need:
                st["ws"] = None
                st["ws"] = torch.empty(need, dtype=torch.uint8, device=st["xin"].device)
        st["generation"] = nnet.generation


def _lane_streams(owner, main):
    """Streams of the concurrent lanes: lane 0 runs on the caller's stream, lanes 1.. on the process's shared side
    streams (_lib.lane_streams: high priority, so a lane never waits behind another lane's kernels in a shared
    hardware queue).  Lane 0 on a side stream as well (equal priorities) measured 0.2-0.3 % slower."""
    return [main] + _lib.lane_streams(main.device, owner.lanes - 1)


def _fork(main, streams):
    for s in streams:
        if s is not main:
            s.wait_stream(main)


def _join(main, streams, outs):
    for s, o in zip(streams, outs):
        if s is not main:
            main.wait_stream(s)
            for t in (o if isinstance(o, tuple) else (o,)):
                t.record_stream(main)


class ClassCondSampler:
    """z_T -> z_0 for a class-conditional (or unconditional) UViT with CFG, fully on the GPU.

    nnet: panopticdiffusionmodels_amd.libs.uvit.UViT on the GPU.  cfg_scale > 0 batches the uncond rows
    (label = null_label, the dataset's K: eval_ldm_discrete.py:76) behind the cond rows.
    """

    def __init__(self, nnet, front_end="dpm_solver_pytorch", cfg_scale=0.4, null_label=1000, steps=50, eps=None,
                 betas=None, use_graph=True, lanes=1):
        self.nnet = nnet
        self.plan, self.time_scale = build_plan(front_end, steps, eps, betas)
        self.cfg = cfg_scale is not None and cfg_scale > 0
        self.cfg_scale = float(cfg_scale or 0.0)
        self.null_label = null_label
        self.use_graph = use_graph
        # lanes > 1 (graph mode): the batch is cut into `lanes` sub-batches sampled concurrently on their own
        # streams, each with a private workspace and graph, so one lane's GEMMs fill the CUs the other's leave
        # idle in a partly filled last wave (batches whose 2B * L rows tile the 256-row GEMM unevenly)
        self.lanes = max(1, int(lanes))
        self._state = {}
        self.nfe = sc.nfe(self.plan)

    def _buffers(self, B, device, lane=None):
        key = (B, device, lane)
        if key in self._state:
            return self._state[key]
        n = self.nnet
        rows = 2 * B if self.cfg else B
        shp = (n.in_chans, n.img_size, n.img_size)
        st = dict(
            # a lane's private workspace (concurrent lanes must not share the handle's)
            ws=None if lane is None else torch.empty(n.native().workspace_bytes(rows), dtype=torch.uint8,
                                                     device=device),
            rows=rows, generation=n.generation,
            xin=torch.empty(rows, *shp, device=device),           # batched model input [cond | uncond]
            pre=torch.empty(rows, *shp, device=device),           # model output before the final conv
            x=torch.empty(B, *shp, device=device),                # solver state at the step start
            m=[torch.empty(B, *shp, device=device) for _ in range(3)],
            y=torch.empty(rows, dtype=torch.int64, device=device) if n.num_classes > 0 else None,
            t=torch.empty(self.nfe, rows, device=device),         # per-evaluation net time inputs
            graph=None,
        )
        k = 0
        for stages in self.plan:
            for s in stages:
                st["t"][k].fill_(s["time"] * self.time_scale)
                k += 1
        self._state[key] = st
        return st

    def _loop(self, st, B):
        n = self.nnet
        w, b = n.final_conv_params()
        xin, pre, x, ms = st["xin"], st["pre"], st["x"], st["m"]
        cond = xin[:B]
        unc = xin[B:] if self.cfg else None
        k = 0
        for stages in self.plan:
            for j, s in enumerate(stages):
                n.forward_pre(xin, st["t"][k], st["y"], out=pre, workspace=st["ws"])
                last = j == len(stages) - 1
                terms = [x] + ms[:j]
                coeffs = [s["nx"]] + s["nm"]
                _lib.stage_epilogue(pre, B, conv_w=w, conv_b=b, cfg_scale=self.cfg_scale if self.cfg else None,
                                    xin=cond, ax=s["ax"], ae=s["ae"], m_out=ms[j], terms=terms, coeffs=coeffs,
                                    cm=s["cm"], x_out=cond, x_out2=unc, x_out3=x if last else None)
                k += 1

    @torch.no_grad()
    def sample(self, z, y=None, eager=False):
        """z [B, C, H, W] fp32 on the GPU; y [B] int64 labels (num_classes > 0).  Returns z_0 [B, C, H, W].
        eager=True runs this call without the HIP graph (e.g. with the GEMM profiling hook enabled)."""
        _lib.require_gpu(z)
        B = z.shape[0]
        if self.lanes > 1 and B >= self.lanes and self.use_graph and not eager:
            return self._sample_lanes(z, y)
        return self._sample_one(z, y, eager)

    def _sample_lanes(self, z, y):
        main = torch.cuda.current_stream(z.device)
        streams = _lane_streams(self, main)
        _fork(main, streams)   # before lane 0's work is queued on main
        bounds = [round(i * z.shape[0] / self.lanes) for i in range(self.lanes + 1)]
        outs = []
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                zi = z[bounds[i]:bounds[i + 1]]
                yi = y[bounds[i]:bounds[i + 1]] if y is not None else None
                outs.append(self._sample_one(zi, yi, False, lane=i))
        _join(main, streams, outs)
        return torch.cat(outs)

    def _sample_one(self, z, y, eager, lane=None):
        B = z.shape[0]
        st = self._buffers(B, z.device, lane)
        st["x"].copy_(z)
        st["xin"][:B].copy_(z)
        if self.cfg:
            st["xin"][B:].copy_(z)
        if st["y"] is not None:
            if y is None:
                raise ValueError("labels required for a class-conditional net")
            st["y"][:B].copy_(y)
            if self.cfg:
                st["y"][B:].fill_(self.null_label)
        if not self.use_graph or eager:
            self._loop(st, B)
            return st["x"].clone()
        _drop_stale_graph(st, self.nnet)
        if st["graph"] is None:
            # warm-up outside capture: builds the native handle, workspace and conv params
            self._loop(st, B)
            st["x"].copy_(z)
            st["xin"][:B].copy_(z)
            if self.cfg:
                st["xin"][B:].copy_(z)
            torch.cuda.synchronize(z.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._loop(st, B)
            st["graph"] = g
        st["graph"].replay()
        return st["x"].clone()


class T2ISampler:
    """Text-conditioned panoptic co-generation sampler (train_t2i_discrete.py:387-439 cfg_nnet + 480-546
    dpm_solver_sample, use_panoptic=True, use_ground_truth=False): dpm_solver_pp fast, predict_x0, discrete SD
    betas, CFG on both the noise and the predicted mask (uncond = empty_context), mask co-update with
    `enable_mask_opt`.  Returns (z_0, pred_mask)."""

    def __init__(self, nnet, cfg_scale=1.0, steps=50, betas=None, enable_mask_opt=True, use_graph=True, lanes=1):
        self.nnet = nnet
        self.lanes = max(1, int(lanes))   # concurrent sub-batches (ClassCondSampler)
        hs = sc.HostDiscrete(betas=sd_betas() if betas is None else betas)
        self.plan = sc.pp_fast_plan(hs, steps, 1.0 / hs.N, 1.0, order=3, predict_x0=True,
                                    enable_mask_opt=enable_mask_opt)
        self.time_scale = float(hs.N)
        self.cfg = cfg_scale is not None and cfg_scale > 0
        self.cfg_scale = float(cfg_scale or 0.0)
        self.use_graph = use_graph
        self.nfe = sc.nfe(self.plan)
        self._state = {}

    def _buffers(self, B, device, lane=None):
        key = (B, device, lane)
        if key in self._state:
            return self._state[key]
        n = self.nnet
        rows = 2 * B if self.cfg else B
        S, K = n.img_size, n.num_panoptic_class
        shp, mshp = (n.in_chans, S, S), (K, S, S)
        st = dict(
            ws=None if lane is None else torch.empty(n.native().workspace_bytes(rows), dtype=torch.uint8,
                                                     device=device),
            rows=rows, generation=n.generation,
            xin=torch.empty(rows, *shp, device=device), pre=torch.empty(rows, *shp, device=device),
            x=torch.empty(B, *shp, device=device), m=[torch.empty(B, *shp, device=device) for _ in range(3)],
            min=torch.empty(rows, *mshp, device=device), mpre=torch.empty(rows, *mshp, device=device),
            mask=torch.empty(B, *mshp, device=device), pm=[torch.empty(B, *mshp, device=device) for _ in range(3)],
            ctx=torch.empty(rows, n.num_clip_token, n.clip_dim, device=device),
            t=torch.empty(self.nfe, rows, device=device), graph=None)
        k = 0
        for stages in self.plan:
            for s in stages:
                st["t"][k].fill_(s["time"] * self.time_scale)
                k += 1
        self._state[key] = st
        return st

    def _loop(self, st, B):
        n = self.nnet
        wx, bx = n.conv_params()
        wm, bm = n.conv_params(mask=True)
        xin, x, ms = st["xin"], st["x"], st["m"]
        mn, mask, pms = st["min"], st["mask"], st["pm"]
        scale = self.cfg_scale if self.cfg else None
        k = 0
        for stages in self.plan:
            for j, s in enumerate(stages):
                n.forward_pre(xin, st["t"][k], st["ctx"], mn, out=st["pre"], mask_out=st["mpre"], workspace=st["ws"])
                last = j == len(stages) - 1
                _lib.stage_epilogue(st["pre"], B, conv_w=wx, conv_b=bx, cfg_scale=scale, xin=xin[:B], ax=s["ax"],
                                    ae=s["ae"], m_out=ms[j], terms=[x] + ms[:j], coeffs=[s["nx"]] + s["nm"],
                                    cm=s["cm"], x_out=xin[:B], x_out2=xin[B:] if self.cfg else None,
                                    x_out3=x if last else None)
                mk = s["mask"]
                if mk == "pred":   # mask state := pred_mask of the step's first evaluation
                    terms, coeffs, cm = [pms[0]], [1.0], 0.0
                else:
                    terms, coeffs, cm = [mask] + pms[:j], [mk["mx"]] + mk["mm"], mk["mc"]
                _lib.stage_epilogue(st["mpre"], B, conv_w=wm, conv_b=bm, cfg_scale=scale, act_tanh=True, ae=1.0,
                                    m_out=pms[j], terms=terms, coeffs=coeffs, cm=cm, x_out=mn[:B],
                                    x_out2=mn[B:] if self.cfg else None, x_out3=mask if last else None)
                k += 1

    @torch.no_grad()
    def sample(self, z, context, empty_context, mask_token):
        _lib.require_gpu(z)
        B = z.shape[0]
        if self.lanes > 1 and B >= self.lanes and self.use_graph:
            main = torch.cuda.current_stream(z.device)
            streams = _lane_streams(self, main)
            _fork(main, streams)
            bounds = [round(i * B / self.lanes) for i in range(self.lanes + 1)]
            outs = []
            for i, s in enumerate(streams):
                lo, hi = bounds[i], bounds[i + 1]
                with torch.cuda.stream(s):
                    outs.append(self._sample_one(z[lo:hi], context[lo:hi], empty_context, mask_token[lo:hi], i))
            _join(main, streams, outs)
            return torch.cat([a for a, _ in outs]), torch.cat([b for _, b in outs])
        return self._sample_one(z, context, empty_context, mask_token)

    def _sample_one(self, z, context, empty_context, mask_token, lane=None):
        B = z.shape[0]
        st = self._buffers(B, z.device, lane)

        def load():
            st["x"].copy_(z)
            st["xin"][:B].copy_(z)
            st["mask"].copy_(mask_token)
            st["min"][:B].copy_(mask_token)
            st["ctx"][:B].copy_(context)
            if self.cfg:
                st["xin"][B:].copy_(z)
                st["min"][B:].copy_(mask_token)
                st["ctx"][B:].copy_(empty_context.expand(B, -1, -1))
        load()
        if not self.use_graph:
            self._loop(st, B)
        else:
            _drop_stale_graph(st, self.nnet)
            if st["graph"] is None:
                self._loop(st, B)
                load()
                torch.cuda.synchronize(z.device)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self._loop(st, B)
                st["graph"] = g
            st["graph"].replay()
        return st["x"].clone(), st["pm"][0].clone()

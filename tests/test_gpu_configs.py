"""Every BASELINE config exercised on the HIP path at its full shape.

* configs[3] mscoco_uvit_small: the full panoptic t2i forward (77 x 768 context, 334-token image stream,
  590-token mask stream, 13 zeroconv injections) vs the fp32 CPU oracle, with and without mask tokens and in
  ground-truth mode (libs/uvit_t2i.py:378-525); the 50-NFE panoptic sampler (train_t2i_discrete.py:480-546).
* configs[2] imagenet256_uvit_huge / configs[4] imagenet512_uvit_huge: the 50-NFE dpm_solver_pp front end
  (eval_ldm_discrete.py:90-107) through the fused sampler: finite, graph == eager, batch-shard invariance,
  and agreement with the reference-API DPM_Solver driving the same HIP network.
Tolerances: per forward rel-L2 <= 2e-2 (bf16), final latent of two samplers over the same network <= 1e-2
(bf16), graph vs eager bit-exact, batch-shard invariance <= 1e-6."""
import pytest
import torch

from oracle import uvit_ref
from panopticdiffusionmodels_amd import configs as C
from panopticdiffusionmodels_amd import weights as W
from panopticdiffusionmodels_amd.sampler import ClassCondSampler, T2ISampler, sd_betas
from panopticdiffusionmodels_amd.utils import get_nnet

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _net(name, dev, seed=3, init="random"):
    cfg = C.nnet_kwargs(name)
    sd = W.nnet_state_dict(cfg, seed=seed, init=init)
    net = get_nnet(**cfg)
    net.load_state_dict(sd)
    return net.to(dev).eval(), sd, cfg


@pytest.fixture(scope="module")
def coco(dev):
    return _net("mscoco_uvit_small", dev)


def _t2i_inputs(B, seed=1):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, 4, 32, 32, generator=g)
    t = torch.rand(B, generator=g) * 999 + 1
    ctx = torch.randn(B, 77, 768, generator=g)
    mt = torch.randn(B, 8, 32, 32, generator=g)
    return x, t, ctx, mt


def test_full_t2i_forward_with_mask_vs_oracle(dev, coco):
    torch.set_num_threads(min(16, torch.get_num_threads()))
    net, sd, cfg = coco
    kw = dict(cfg)
    kw.pop("name")
    x, t, ctx, mt = _t2i_inputs(2)
    with torch.no_grad():
        eps, pm = net(x.to(dev), t.to(dev), ctx.to(dev), mask_token=mt.to(dev))
        ref_eps, ref_pm = uvit_ref.uvit_t2i_forward(sd, kw, x, t, ctx, mask_token=mt)
    assert torch.isfinite(eps).all() and torch.isfinite(pm).all()
    assert rel(eps, ref_eps) < 2e-2
    assert rel(pm, ref_pm) < 2e-2


def test_full_t2i_forward_grouped_rows_vs_oracle(dev, coco):
    """At >= 13 rows every image- / mask-stream Linear pair of a layer is ONE grouped persistent launch (capi.hip
    run_block16_pair -> pdm::gemm_launch_pair: both problems >= 4096 rows); the B <= 3 tests above take its two-launch
    fallback.  The grouped forward at B = 14 against the fp32 oracle (2e-2, as above) and against the same forward
    with grouping off (pdm_set_gemm_algo(7): separate whole-tile launches) to bf16 rounding (1e-2)."""
    torch.set_num_threads(min(16, torch.get_num_threads()))
    from panopticdiffusionmodels_amd import _lib
    net, sd, cfg = coco
    kw = dict(cfg)
    kw.pop("name")
    x, t, ctx, mt = _t2i_inputs(14, seed=3)
    with torch.no_grad():
        eps, pm = net(x.to(dev), t.to(dev), ctx.to(dev), mask_token=mt.to(dev))
        _lib.check(_lib.load().pdm_set_gemm_algo(7), "pdm_set_gemm_algo")
        try:
            eps7, pm7 = net(x.to(dev), t.to(dev), ctx.to(dev), mask_token=mt.to(dev))
        finally:
            _lib.load().pdm_set_gemm_algo(0)
        ref_eps, ref_pm = uvit_ref.uvit_t2i_forward(sd, kw, x, t, ctx, mask_token=mt)
    assert torch.isfinite(eps).all() and torch.isfinite(pm).all()
    assert rel(eps, ref_eps) < 2e-2
    assert rel(pm, ref_pm) < 2e-2
    assert rel(eps, eps7) < 1e-2
    assert rel(pm, pm7) < 1e-2


def test_full_t2i_forward_no_mask_and_ground_truth_vs_oracle(dev, coco):
    net, sd, cfg = coco
    kw = dict(cfg)
    kw.pop("name")
    x, t, ctx, mt = _t2i_inputs(2, seed=2)
    with torch.no_grad():
        eps = net(x.to(dev), t.to(dev), ctx.to(dev))
        ref = uvit_ref.uvit_t2i_forward(sd, kw, x, t, ctx)
        assert rel(eps, ref) < 2e-2
        eps_gt, y = net(x.to(dev), t.to(dev), ctx.to(dev), mask_token=mt.to(dev), use_ground_truth=True)
        ref_gt, _ = uvit_ref.uvit_t2i_forward(sd, kw, x, t, ctx, mask_token=mt, use_ground_truth=True)
        assert rel(eps_gt, ref_gt) < 2e-2
        assert torch.equal(y.cpu(), mt)


def test_full_t2i_sampler_properties(dev, coco):
    """50-NFE panoptic co-generation at the mscoco shape: finite, graph == eager, batch invariance."""
    net, _, _ = coco
    g = torch.Generator().manual_seed(7)
    z = torch.randn(3, 4, 32, 32, generator=g).to(dev)
    ctx = torch.randn(3, 77, 768, generator=g).to(dev)
    empty = torch.randn(77, 768, generator=g).to(dev)
    mt = torch.randn(3, 8, 32, 32, generator=g).to(dev)
    scale = C.get_config("mscoco_uvit_small")["cfg_scale"]
    sg = T2ISampler(net, cfg_scale=scale, steps=50, use_graph=True)
    se = T2ISampler(net, cfg_scale=scale, steps=50, use_graph=False)
    a, pa = sg.sample(z, ctx, empty, mt)
    b, pb = se.sample(z, ctx, empty, mt)
    assert torch.isfinite(a).all() and torch.isfinite(pa).all()
    assert torch.equal(a, b) and torch.equal(pa, pb)
    c, pc = se.sample(z[:1], ctx[:1], empty, mt[:1])
    assert rel(c, a[:1]) < 1e-6 and rel(pc, pa[:1]) < 1e-6
    # concurrent sub-batch lanes (two streams, private workspaces / graphs) give the single-lane result
    s2 = T2ISampler(net, cfg_scale=scale, steps=50, use_graph=True, lanes=2)
    d, pd = s2.sample(z, ctx, empty, mt)
    assert rel(d, a) < 1e-6 and rel(pd, pa) < 1e-6


@pytest.mark.parametrize("name,B", [("imagenet256_uvit_huge", 3), ("imagenet512_uvit_huge", 2)])
def test_full_huge_pp_sampler(dev, name, B):
    """H/2 and H/4 through the dpm_solver_pp front end: fused sampler (graph and eager) vs the reference-API
    DPM_Solver (eval_ldm_discrete.py:72-102 as written) on the same HIP network, plus batch invariance."""
    from panopticdiffusionmodels_amd.dpm_solver_pp import DPM_Solver, NoiseScheduleVP
    net, _, cfg = _net(name, dev, seed=0, init="reference")
    full = C.get_config(name)
    scale = full["cfg_scale"]
    g = torch.Generator().manual_seed(1234)
    z = torch.randn(B, *full["z_shape"], generator=g).to(dev)
    y = torch.randint(0, 1000, (B,), generator=g).to(dev)
    sg = ClassCondSampler(net, front_end="dpm_solver_pp", cfg_scale=scale, null_label=1000, steps=50, use_graph=True)
    se = ClassCondSampler(net, front_end="dpm_solver_pp", cfg_scale=scale, null_label=1000, steps=50,
                          use_graph=False)
    a = sg.sample(z, y)
    b = se.sample(z, y)
    assert torch.isfinite(a).all()
    assert torch.equal(a, b)
    c = se.sample(z[:1], y[:1])
    assert rel(c, a[:1]) < 1e-6

    def cfg_nnet(x, timesteps, y):
        _cond = net(x, timesteps, y=y)
        _uncond = net(x, timesteps, y=torch.tensor([1000] * x.size(0), device=dev))
        return _cond + scale * (_cond - _uncond)

    ns = NoiseScheduleVP(schedule='discrete', betas=torch.tensor(sd_betas(), device=dev).float())

    def model_fn(x, t_continuous):
        return cfg_nnet(x, t_continuous * 1000, y=y)
    r = DPM_Solver(model_fn, ns, predict_x0=True, thresholding=False).sample(z, steps=50, eps=1. / 1000, T=1.)
    # the reference API runs cond / uncond as two B-row forwards (other GEMM tilings, other bf16 roundings)
    # against the fused 2B-row forward: the bf16 final-latent tolerance applies
    err = rel(a, r)
    assert err < 1e-2, err

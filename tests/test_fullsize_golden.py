"""Full-size parity against the REFERENCE's own outputs (tests/golden/fullsize.npz, made by
tests/golden/make_fullsize_golden.py with the reference imported): every BASELINE config's forward at B = 2
and full 50-NFE CFG samples (L/2 through dpm_solver_pytorch, H/2 and H/4 through dpm_solver_pp, the panoptic t2i
with the mask co-update).  configs[4] (H/4, 512²) is checked at both precisions: the bf16 HIP sampler and the
MXFP8 one the bench runs (UViT.set_precision('fp8')), each against the reference's fp32 latent.

CPU: the oracle (oracle/uvit_ref.py) vs the reference forwards, rel-L2 <= 1e-5 — the oracle is pinned at full
size, not only on tiny nets.  GPU: the HIP forward (rel-L2 <= 2e-2) and the fused HIP-graph samplers (final
latent <= 1e-2, panoptic mask <= 2e-2), SURVEY.md §8c tolerances.
"""
import os

import numpy as np
import pytest
import torch

from oracle import uvit_ref
from panopticdiffusionmodels_amd import configs as C
from panopticdiffusionmodels_amd import weights as W

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FWD = ["cifar10_uvit_small", "imagenet256_uvit_large", "imagenet256_uvit_huge", "imagenet512_uvit_huge",
       "mscoco_uvit_small"]
SAMPLE = ["cifar10_uvit_small", "imagenet256_uvit_large", "imagenet256_uvit_huge", "imagenet512_uvit_huge", "mscoco_uvit_small"]
TOL_SAMPLE = {"bf16": 1e-2, "fp8": 3e-2}   # final latent after 50 NFE vs the reference


@pytest.fixture(scope="module")
def fs():
    return np.load(os.path.join(REPO, "tests", "golden", "fullsize.npz"))


def rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _checksum(sd):
    return np.array([float(v.double().sum()) for v in sd.values()] + [float(v.double().abs().sum()) for v in sd.values()])


def fwd_inputs(name, B=2, seed=5):
    """= make_golden._inputs (the fixture stores their checksum)."""
    cfg = C.get_config(name)
    n = cfg["nnet"]
    g = torch.Generator().manual_seed(seed)
    Cc, H, Wd = cfg["z_shape"]
    out = {"x": torch.randn(B, Cc, H, Wd, generator=g), "t": torch.rand(B, generator=g) * 998.0 + 1.0}
    if n["name"] == "uvit" and n.get("num_classes", -1) > 0:
        y = torch.randint(0, n["num_classes"] - 1, (B,), generator=g)
        y[-1] = n["num_classes"] - 1
        out["y"] = y
    if n["name"] == "uvit_t2i":
        out["context"] = torch.randn(B, n["num_clip_token"], n["clip_dim"], generator=g)
        out["mask_token"] = torch.randn(B, n["num_panoptic_class"], H, Wd, generator=g)
    return out


def sample_inputs(name, seed=99):
    """= make_fullsize_golden.sample_inputs (configs[0], CIFAR-10: the BASELINE batch of 4 images)."""
    full = C.get_config(name)
    n = full["nnet"]
    g = torch.Generator().manual_seed(seed)
    nb = 4 if name == "cifar10_uvit_small" else 1
    out = {"z": torch.randn(nb, *full["z_shape"], generator=g)}
    if n.get("num_classes", -1) > 0:
        out["y"] = torch.randint(0, n["num_classes"] - 1, (1,), generator=g)
    if n["name"] == "uvit_t2i":
        out["context"] = torch.randn(1, n["num_clip_token"], n["clip_dim"], generator=g)
        out["empty_context"] = torch.randn(n["num_clip_token"], n["clip_dim"], generator=g)
        out["mask_token"] = torch.randn(1, n["num_panoptic_class"], *full["z_shape"][1:], generator=g)
    return out


def cfg_scale_zero(full):
    return not (full.get("cfg_scale") or 0) > 0


def _sd(name, seed, init):
    cfg = C.nnet_kwargs(name)
    return cfg, W.nnet_state_dict(cfg, seed=seed, init=init)


@pytest.mark.parametrize("name", FWD)
def test_oracle_vs_reference_fullsize_forward(fs, name):
    torch.set_num_threads(min(8, os.cpu_count() or 8))
    cfg, sd = _sd(name, 3, "random")
    np.testing.assert_allclose(_checksum(sd), fs[f"fwd/{name}/sd_checksum"], rtol=1e-9)
    inp = fwd_inputs(name)
    np.testing.assert_allclose([float(v.double().sum()) for v in inp.values()], fs[f"fwd/{name}/in_checksum"],
                               rtol=1e-9)
    kw = dict(cfg)
    kind = kw.pop("name")
    with torch.no_grad():
        if kind == "uvit_t2i":
            eps, pm = uvit_ref.uvit_t2i_forward(sd, kw, inp["x"], inp["t"], inp["context"],
                                                mask_token=inp["mask_token"])
            assert rel(pm, fs[f"fwd/{name}/pred_mask"]) < 1e-5
        else:
            eps = uvit_ref.uvit_forward(sd, kw, inp["x"], inp["t"], inp.get("y"))
    assert rel(eps, fs[f"fwd/{name}/eps"]) < 1e-5


def test_oracle_vs_reference_cifar_sample(fs):
    """configs[0] (eval.py:47-86): CIFAR-10 U-ViT-S/2, pixel space, unconditional, no CFG, 50-NFE
    dpm_solver_pytorch (ScoreModel noise_pred, time fed as t * 999) -- the oracle's trajectory (solver_ref +
    uvit_ref) against the reference's own final sample of 4 images."""
    from oracle import solver_ref
    torch.set_num_threads(min(8, os.cpu_count() or 8))
    name = "cifar10_uvit_small"
    cfg, sd = _sd(name, 0, "reference")
    np.testing.assert_allclose(_checksum(sd), fs[f"sample/{name}/sd_checksum"], rtol=1e-9)
    kw = dict(cfg)
    kw.pop("name")
    fn = solver_ref.cfg_class_closure(lambda x, t, y: uvit_ref.uvit_forward(sd, kw, x, t, y), None, 0.0, None, 999.0)
    with torch.no_grad():
        z = solver_ref.pytorch_sample(fn, sample_inputs(name)["z"].clone(), steps=50, eps=1e-4)
    assert rel(z, fs[f"sample/{name}/z"]) < 1e-5, rel(z, fs[f"sample/{name}/z"])


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.mark.gpu
@pytest.mark.parametrize("name,residual", [(n, "bf16") for n in FWD] + [("imagenet256_uvit_large", "fp32"),
                                                                         ("mscoco_uvit_small", "fp32")])
def test_hip_vs_reference_fullsize_forward(fs, dev, name, residual):
    """residual: the stream x between the block Linears in bf16 (default, as the reference's autocast run) or
    fp32 (libs/uvit.py UViT.set_residual)."""
    from panopticdiffusionmodels_amd.utils import get_nnet
    cfg, sd = _sd(name, 3, "random")
    net = get_nnet(**cfg)
    net.load_state_dict(sd)
    net = net.to(dev).eval()
    if residual != "bf16":
        net.set_residual(residual)
    inp = {k: v.to(dev) for k, v in fwd_inputs(name).items()}
    with torch.no_grad():
        if cfg["name"] == "uvit_t2i":
            eps, pm = net(inp["x"], inp["t"], inp["context"], mask_token=inp["mask_token"])
            assert rel(pm, fs[f"fwd/{name}/pred_mask"]) < 2e-2
        else:
            eps = net(inp["x"], inp["t"], inp.get("y"))
    assert torch.isfinite(eps).all()
    err = rel(eps, fs[f"fwd/{name}/eps"])
    print(f"{name} residual {residual}: forward rel-L2 vs the reference = {err:.3e}")
    assert err < 2e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize("name,precision", [(n, "bf16") for n in SAMPLE] + [("imagenet512_uvit_huge", "fp8")])
def test_hip_sampler_vs_reference_fullsize(fs, dev, name, precision):
    from panopticdiffusionmodels_amd.sampler import ClassCondSampler, T2ISampler
    from panopticdiffusionmodels_amd.utils import get_nnet
    full = C.get_config(name)
    cfg, sd = _sd(name, 0, "reference")
    np.testing.assert_allclose(_checksum(sd), fs[f"sample/{name}/sd_checksum"], rtol=1e-9)
    net = get_nnet(**cfg)
    net.load_state_dict(sd)
    net = net.to(dev).eval()
    if precision != "bf16":
        net.set_precision(precision)
    inp = {k: v.to(dev) for k, v in sample_inputs(name).items()}
    if cfg["name"] == "uvit_t2i":
        z, pm = T2ISampler(net, cfg_scale=full["cfg_scale"], steps=50).sample(inp["z"], inp["context"],
                                                                               inp["empty_context"], inp["mask_token"])
        assert rel(pm, fs[f"sample/{name}/pred_mask"]) < 2e-2, rel(pm, fs[f"sample/{name}/pred_mask"])
    else:
        s = ClassCondSampler(net, front_end=full["front_end"], cfg_scale=full["cfg_scale"],
                             null_label=cfg["num_classes"] - 1, steps=50, eps=full.get("eps"))
        z = s.sample(inp["z"], inp.get("y"))   # configs[0]: unconditional, cfg_scale 0 (one B-row forward per NFE)
        if cfg_scale_zero(full):
            assert not s.cfg and s.nfe == 50
    assert torch.isfinite(z).all()
    err = rel(z, fs[f"sample/{name}/z"])
    print(f"{name} {precision}: final latent rel-L2 vs the reference = {err:.3e}")
    assert err < TOL_SAMPLE[precision], err

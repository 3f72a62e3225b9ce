"""Parity at the bench's own batch: the kernels bench.py times -- the persistent `gemm8s`
GEMMs (M >= 4096 rows), the persistent `attention_v3` (Dh 64) / `attention_h72` (Dh 72) and, for configs[4], the
MXFP8 GEMMs -- chained through whole forwards and through the two graph-captured sampling lanes, checked against the
REFERENCE's own outputs (tests/golden/fullsize.npz, made by tests/golden/make_fullsize_golden.py with the reference
imported).

The reference samples `mini_batch_size = 50` images per process (configs/imagenet256_uvit_large.py:66,
eval_ldm.py:80-111, eval_ldm_discrete.py:90-107).  The golden fixtures hold 1-2 rows, so the fixture rows are placed
inside a full bench batch (first rows, the first row of the second lane, the last rows) and the rest of the batch is
seeded noise: every row of a U-ViT forward is computed independently of the others (per-row GEMM tiles, per-(image,
head) attention), so a fixture row's result must match the reference whatever surrounds it.  The other rows are
checked against the fp32 oracle (oracle/uvit_ref.py, itself pinned to the reference at <= 1e-5) on a CPU subset.

Tolerances: forward rel-L2 <= 2e-2 (bf16), <= 6e-2 (MXFP8 'fp8'); final 50-NFE latent <= 1e-2
(bf16), <= 3e-2 (MXFP8); panoptic mask <= 2e-2.
"""
import os

import numpy as np
import pytest
import torch

from panopticdiffusionmodels_amd import configs as C
from panopticdiffusionmodels_amd import weights as W

from test_fullsize_golden import _checksum, fwd_inputs, sample_inputs

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOL_FWD = {"bf16": 2e-2, "fp8": 6e-2}
TOL_SAMPLE = {"bf16": 1e-2, "fp8": 3e-2}


def rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.fixture(scope="module")
def fs():
    return np.load(os.path.join(REPO, "tests", "golden", "fullsize.npz"))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _net(name, dev, seed, init, precision="bf16"):
    from panopticdiffusionmodels_amd.utils import get_nnet
    cfg = C.nnet_kwargs(name)
    sd = W.nnet_state_dict(cfg, seed=seed, init=init)
    net = get_nnet(**cfg)
    net.load_state_dict(sd)
    net = net.to(dev).eval()
    if precision != "bf16":
        net.set_precision(precision)
    return net, cfg, sd


def _gemm_policy_is_persistent(rows_per_forward, L):
    """The automatic GEMM choice takes the persistent kernel at >= 4096 rows (csrc/gemm.hip pick_algo); the bench
    batch must land there, or these tests would not cover what the bench times."""
    return rows_per_forward * L >= 4096


# ---------------------------------------------------------------- forward at the bench's rows
FWD_CASES = [("imagenet256_uvit_large", 100, "bf16"), ("imagenet256_uvit_large", 50, "bf16"),
             ("imagenet256_uvit_huge", 100, "bf16"), ("imagenet512_uvit_huge", 100, "fp8"),
             ("imagenet512_uvit_huge", 100, "bf16")]


@pytest.mark.parametrize("name,rows,precision", FWD_CASES)
def test_forward_at_bench_rows_vs_reference(fs, dev, name, rows, precision):
    """One CFG forward of the bench (rows = 2B = 100 for the eager pass, 50 per sampling lane).  The reference's
    B = 2 forward inputs (fwd_inputs, seed 5) sit at rows 0-1 and again at rows-2..rows-1 (the last, ragged GEMM
    row tile); both copies must match the reference's eps, and the batch's other rows the oracle."""
    from oracle import uvit_ref
    net, cfg, sd = _net(name, dev, 3, "random", precision)
    np.testing.assert_allclose(_checksum(sd), fs[f"fwd/{name}/sd_checksum"], rtol=1e-9)
    L = (cfg["img_size"] // cfg["patch_size"]) ** 2 + 2
    assert _gemm_policy_is_persistent(rows, L)
    fx = fwd_inputs(name)
    g = torch.Generator().manual_seed(1000 + rows)
    x = torch.randn(rows, *fx["x"].shape[1:], generator=g)
    t = torch.rand(rows, generator=g) * 998.0 + 1.0
    y = torch.randint(0, cfg["num_classes"], (rows,), generator=g)
    for lo in (0, rows - 2):
        x[lo:lo + 2], t[lo:lo + 2], y[lo:lo + 2] = fx["x"], fx["t"], fx["y"]
    with torch.no_grad():
        eps = net(x.to(dev), t.to(dev), y.to(dev)).float().cpu()
    assert torch.isfinite(eps).all()
    ref = torch.from_numpy(fs[f"fwd/{name}/eps"])
    for lo in (0, rows - 2):
        err = rel(eps[lo:lo + 2], ref)
        print(f"{name} rows {rows} {precision}: fixture rows {lo}-{lo + 1} vs the reference {err:.3e}")
        assert err < TOL_FWD[precision], (lo, err)
    # other rows against the fp32 oracle (a CPU subset: rows straddling the lane / tile boundaries)
    pick = sorted({2, rows // 2 - 1, rows // 2, rows - 3})
    kw = dict(cfg)
    kw.pop("name")
    torch.set_num_threads(min(16, os.cpu_count() or 16))
    with torch.no_grad():
        want = uvit_ref.uvit_forward(sd, kw, x[pick], t[pick], y[pick])
    err = rel(eps[pick], want)
    print(f"{name} rows {rows} {precision}: rows {pick} vs the oracle {err:.3e}")
    assert err < TOL_FWD[precision], err


# ---------------------------------------------------------------- full 50-NFE sampling at the bench's batch
SAMPLE_CASES = [("imagenet256_uvit_large", 50, "bf16"), ("imagenet256_uvit_huge", 50, "bf16"),
                ("imagenet512_uvit_huge", 50, "fp8"), ("cifar10_uvit_small", 4, "bf16")]


@pytest.mark.parametrize("name,B,precision", SAMPLE_CASES)
def test_sampler_at_bench_batch_vs_reference(fs, dev, name, B, precision):
    """bench.py's exact sampling configuration: B images (the config's mini_batch_size) as two graph-captured
    concurrent lanes of B/2, seeded 'reference' init weights (the bench's and the fixture's).  The reference's
    50-NFE sample input sits at rows 0, B/2 (first row of lane 1) and B-1; each of those rows' final latents must
    match the reference's final latent."""
    from panopticdiffusionmodels_amd.sampler import ClassCondSampler
    full = C.get_config(name)
    net, cfg, sd = _net(name, dev, 0, "reference", precision)
    np.testing.assert_allclose(_checksum(sd), fs[f"sample/{name}/sd_checksum"], rtol=1e-9)
    si = sample_inputs(name)
    ref = torch.from_numpy(fs[f"sample/{name}/z"])
    nfix = si["z"].shape[0]                        # 1 (latent configs) or 4 (CIFAR: BASELINE's batch)
    g = torch.Generator().manual_seed(77)
    z = torch.randn(B, *si["z"].shape[1:], generator=g)
    conditional = cfg.get("num_classes", -1) > 0 and "y" in si
    y = torch.randint(0, cfg["num_classes"] - 1, (B,), generator=g) if conditional else None
    slots = [0] if nfix == B else sorted({0, B // 2, B - nfix})
    for lo in slots:
        z[lo:lo + nfix] = si["z"]
        if y is not None:
            y[lo:lo + nfix] = si["y"]
    null = cfg["num_classes"] - 1 if cfg.get("num_classes", -1) > 0 else None
    s = ClassCondSampler(net, front_end=full["front_end"], cfg_scale=full["cfg_scale"], null_label=null, steps=50,
                         eps=full.get("eps"), use_graph=True, lanes=2)
    out = s.sample(z.to(dev), y.to(dev) if y is not None else None)
    torch.cuda.synchronize(dev)
    out = out.float().cpu()
    assert torch.isfinite(out).all()
    for lo in slots:
        err = rel(out[lo:lo + nfix], ref)
        print(f"{name} B={B} lanes=2 {precision}: rows {lo}..{lo + nfix - 1} final latent vs the reference {err:.3e}")
        assert err < TOL_SAMPLE[precision], (lo, err)
    again = s.sample(z.to(dev), y.to(dev) if y is not None else None).float().cpu()   # graph replay
    assert torch.equal(out, again)


def test_t2i_sampler_at_bench_batch_vs_reference(fs, dev):
    """configs[3] as bench.py runs it: B = 32 panoptic co-generation as two graph-captured lanes of 16 (grouped
    image- / mask-stream persistent GEMMs, mask co-update).  The reference's sample input at rows 0, 16 and 31;
    final latent <= 1e-2 and pred_mask <= 2e-2 against the reference's own trajectory."""
    from panopticdiffusionmodels_amd.sampler import T2ISampler
    name, B = "mscoco_uvit_small", 32
    full = C.get_config(name)
    net, cfg, sd = _net(name, dev, 0, "reference")
    np.testing.assert_allclose(_checksum(sd), fs[f"sample/{name}/sd_checksum"], rtol=1e-9)
    si = sample_inputs(name)
    g = torch.Generator().manual_seed(78)
    z = torch.randn(B, *si["z"].shape[1:], generator=g)
    ctx = torch.randn(B, *si["context"].shape[1:], generator=g)
    mt = torch.randn(B, *si["mask_token"].shape[1:], generator=g)
    slots = [0, B // 2, B - 1]
    for lo in slots:
        z[lo], ctx[lo], mt[lo] = si["z"][0], si["context"][0], si["mask_token"][0]
    s = T2ISampler(net, cfg_scale=full["cfg_scale"], steps=50, use_graph=True, lanes=2)
    zo, pm = s.sample(z.to(dev), ctx.to(dev), si["empty_context"].to(dev), mt.to(dev))
    torch.cuda.synchronize(dev)
    zo, pm = zo.float().cpu(), pm.float().cpu()
    assert torch.isfinite(zo).all() and torch.isfinite(pm).all()
    for lo in slots:
        ez = rel(zo[lo:lo + 1], fs[f"sample/{name}/z"])
        em = rel(pm[lo:lo + 1], fs[f"sample/{name}/pred_mask"])
        print(f"{name} B={B} lanes=2: row {lo} latent {ez:.3e} pred_mask {em:.3e}")
        assert ez < 1e-2 and em < 2e-2, (lo, ez, em)

"""U-ViT forward parity on the GPU (HIP path) against the reference's own outputs (golden fixtures) and the
fp32 CPU oracle at the full BASELINE shapes.  Tolerance: bf16 per forward rel-L2 <= 2e-2."""
import numpy as np
import pytest
import torch

from oracle import uvit_ref
from panopticdiffusionmodels_amd import configs as C
from panopticdiffusionmodels_amd import weights as W
from panopticdiffusionmodels_amd.utils import get_nnet

pytestmark = pytest.mark.gpu
TOL_FWD = 2e-2


def rel(a, b):
    a = torch.as_tensor(a).double()
    b = torch.as_tensor(b).double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _net(name, dev, seed=11, init="random"):
    cfg = C.nnet_kwargs(name)
    sd = W.nnet_state_dict(cfg, seed=seed, init=init)
    net = get_nnet(**cfg)
    net.load_state_dict(sd)
    return net.to(dev).eval(), sd, cfg


@pytest.mark.parametrize("name", ["tiny_uvit_cond", "tiny_uvit_h", "tiny_uvit_uncond"])
def test_tiny_forward_vs_reference(golden, dev, name):
    net, sd, cfg = _net(name, dev)
    x = torch.from_numpy(golden[f"{name}/in_x"]).to(dev)
    t = torch.from_numpy(golden[f"{name}/in_t"]).to(dev)
    y = torch.from_numpy(golden[f"{name}/in_y"]).to(dev) if f"{name}/in_y" in golden else None
    with torch.no_grad():
        eps = net(x, t, y).cpu()
    assert rel(eps, golden[f"{name}/eps"]) < TOL_FWD


@pytest.mark.parametrize("name,B", [("imagenet256_uvit_large", 2), ("imagenet256_uvit_huge", 2),
                                    ("imagenet512_uvit_huge", 1), ("cifar10_uvit_small", 3)])
def test_full_forward_vs_oracle(dev, name, B):
    torch.set_num_threads(min(16, torch.get_num_threads()))
    net, sd, cfg = _net(name, dev, seed=3, init="random")
    kw = dict(cfg)
    kw.pop("name")
    g = torch.Generator().manual_seed(1)
    zs = C.get_config(name)["z_shape"]
    x = torch.randn(B, *zs, generator=g)
    t = torch.rand(B, generator=g) * 999
    y = torch.randint(0, 1001, (B,), generator=g) if cfg.get("num_classes", -1) > 0 else None
    with torch.no_grad():
        eps = net(x.to(dev), t.to(dev), y.to(dev) if y is not None else None).cpu()
        ref = uvit_ref.uvit_forward(sd, kw, x, t, y)
    assert torch.isfinite(eps).all()
    assert rel(eps, ref) < TOL_FWD


def test_forward_batch_invariance(dev):
    """Row b of a batched forward equals the single-row forward (no cross-sample leakage)."""
    net, _, _ = _net("tiny_uvit_cond", dev)
    g = torch.Generator().manual_seed(2)
    x = torch.randn(5, 4, 16, 16, generator=g).to(dev)
    t = (torch.rand(5, generator=g) * 999).to(dev)
    y = torch.tensor([0, 3, 10, 7, 1]).to(dev)
    with torch.no_grad():
        full = net(x, t, y)
        one = torch.cat([net(x[i:i + 1], t[i:i + 1], y[i:i + 1]) for i in range(5)])
    assert rel(full.cpu(), one.cpu()) < 1e-6

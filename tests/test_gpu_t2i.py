"""Panoptic t2i (libs/uvit_t2i.py, separate mask stream) on the HIP path vs the reference's own outputs."""
import pytest
import torch

from panopticdiffusionmodels_amd import configs as C
from panopticdiffusionmodels_amd import weights as W
from panopticdiffusionmodels_amd.sampler import T2ISampler
from panopticdiffusionmodels_amd.utils import get_nnet

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.fixture(scope="module")
def net():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cfg = C.nnet_kwargs("tiny_t2i")
    n = get_nnet(**cfg)
    n.load_state_dict(W.nnet_state_dict(cfg, seed=11, init="random"))
    return n.cuda().eval()


def _in(golden, k):
    return torch.from_numpy(golden[f"tiny_t2i/in_{k}"]).cuda()


def test_t2i_forward_with_mask(golden, net):
    eps, pm = net(_in(golden, "x"), _in(golden, "t"), _in(golden, "context"), mask_token=_in(golden, "mask_token"))
    assert rel(eps, golden["tiny_t2i/eps_mask"]) < 2e-2
    assert rel(pm, golden["tiny_t2i/pred_mask"]) < 2e-2


def test_t2i_forward_no_mask(golden, net):
    eps = net(_in(golden, "x"), _in(golden, "t"), _in(golden, "context"))
    assert rel(eps, golden["tiny_t2i/eps_nomask"]) < 2e-2


def test_t2i_forward_ground_truth(golden, net):
    mt = _in(golden, "mask_token")
    eps, y = net(_in(golden, "x"), _in(golden, "t"), _in(golden, "context"), mask_token=mt, use_ground_truth=True)
    assert rel(eps, golden["tiny_t2i/eps_gt"]) < 2e-2
    assert torch.equal(y, mt)


@pytest.mark.parametrize("graph", [False, True])
def test_t2i_sampler_vs_reference(golden, net, graph):
    g = lambda k: torch.from_numpy(golden[f"sample/tiny_t2i/{k}"]).cuda()  # noqa: E731
    s = T2ISampler(net, cfg_scale=C.get_config("tiny_t2i")["cfg_scale"], steps=50, use_graph=graph)
    z, pm = s.sample(g("z_init"), g("context"), g("empty_context"), g("mask_init"))
    assert rel(z, golden["sample/tiny_t2i/z"]) < 1e-2
    assert rel(pm, golden["sample/tiny_t2i/pred_mask"]) < 2e-2

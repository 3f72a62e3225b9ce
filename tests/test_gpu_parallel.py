"""The RCCL branch of the latent gather (parallel.gather_latents -> all_gather_into_tensor, the replacement of
`accelerator.gather` in utils.py:585-588) executed on the device: a world-size-1 `nccl` (= RCCL) group in this
process, CUDA latents.  World size > 1 runs in the driver's multi-GPU bench; the multi-rank ordering / ragged
padding logic is covered by tests/test_parallel_gloo.py."""
import socket

import pytest
import torch
import torch.distributed as dist

from panopticdiffusionmodels_amd import parallel

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def nccl_world1():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    store = dist.TCPStore("127.0.0.1", _free_port(), 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
    try:
        yield dev
    finally:
        dist.destroy_process_group()


def test_gather_latents_rccl_world1(nccl_world1):
    dev = nccl_world1
    assert dist.get_backend() == "nccl"
    z, _ = parallel.sample_inputs(range(5), (4, 32, 32), num_classes=None)
    z = z.to(dev)
    g = parallel.gather_latents(z)
    assert g.is_cuda and g.shape == z.shape
    assert torch.equal(g, z)
    # the bench's timing reduction: all_reduce(MAX) of a float64 on the device
    t = torch.tensor([1.25], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    assert float(t.item()) == 1.25
    dist.barrier()

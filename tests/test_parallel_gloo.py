"""Multi-process (world_size 2, gloo, CPU) checks of the batch-sharded sampling path: shard coverage,
world-size-invariant seeding, and the latent all-gather ordering.  The per-rank 'sampler' here is a CPU
stand-in (the HIP sampler needs a GPU); what is tested is the distribution logic bench.py uses."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from panopticdiffusionmodels_amd import parallel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    idx = parallel.shard(n_total, world, rank)
    z, y = parallel.sample_inputs(idx, (4, 8, 8), num_classes=1000)
    out = torch.tanh(z) * 0.5 + y.view(-1, 1, 1, 1).float() * 1e-3   # stand-in for sample()
    g = parallel.gather_latents(out)
    if rank == 0:
        q.put(g)
    dist.barrier()
    dist.destroy_process_group()


def test_shard_covers_everything():
    for n in (1, 7, 64, 100):
        for w in (1, 2, 3, 8):
            got = [i for r in range(w) for i in parallel.shard(n, w, r)]
            assert got == list(range(n))
            sizes = [len(parallel.shard(n, w, r)) for r in range(w)]
            assert max(sizes) - min(sizes) <= 1


def test_seeding_is_world_size_invariant():
    z_all, y_all = parallel.sample_inputs(range(16), (4, 8, 8), num_classes=1000)
    for w in (2, 4):
        parts = [parallel.sample_inputs(parallel.shard(16, w, r), (4, 8, 8), num_classes=1000) for r in range(w)]
        assert torch.equal(torch.cat([p[0] for p in parts]), z_all)
        assert torch.equal(torch.cat([p[1] for p in parts]), y_all)


@pytest.mark.parametrize("n", [8, 7])   # 7: ragged shards (4 + 3)
def test_gather_world2_gloo(n):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    g = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    z, y = parallel.sample_inputs(range(n), (4, 8, 8), num_classes=1000)
    ref = torch.tanh(z) * 0.5 + y.view(-1, 1, 1, 1).float() * 1e-3
    assert torch.equal(g, ref)

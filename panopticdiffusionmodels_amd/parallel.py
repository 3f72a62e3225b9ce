"""Batch sharding across GPUs: one process per GPU, weights replicated, samples
partitioned by global index, no per-step communication, one all-gather of the final latents.

The reference seeds each rank separately (`set_seed(seed, device_specific=True)`, eval_ldm_discrete.py:30)
so its samples depend on the world size; here every sample's z_T and label are drawn from a generator
seeded by (seed, global index), so a given sample is identical at 1, 2, 4 or 8 GPUs.  The gather replaces
`accelerator.gather` of decoded fp32 images (utils.py:585-588) by an RCCL all-gather of the 16 KiB/image
latents; decoding stays rank-local.
"""
import torch
import torch.distributed as dist


def shard(n_total, world, rank):
    """Contiguous block of global sample indices owned by `rank` (sizes differ by at most one)."""
    base, rem = divmod(n_total, world)
    start = rank * base + min(rank, rem)
    return range(start, start + base + (1 if rank < rem else 0))


def sample_inputs(indices, z_shape, num_classes=None, seed=1234):
    """z_T ~ N(0, 1) and labels ~ U{0..num_classes-1} per global index (CPU generators, deterministic)."""
    zs, ys = [], []
    for i in indices:
        g = torch.Generator().manual_seed(seed * 1_000_003 + int(i))
        zs.append(torch.randn(1, *z_shape, generator=g))
        if num_classes:
            ys.append(torch.randint(0, num_classes, (1,), generator=g))
    z = torch.cat(zs) if zs else torch.empty(0, *z_shape)
    y = torch.cat(ys) if ys else None
    return z, y


def gather_latents(z_local, group=None):
    """All-gather per-rank latent batches -> [sum of rank sizes, ...] in rank order.

    Ranks may hold different counts (shard() gives sizes that differ by one when n_total % world != 0): the
    sizes are exchanged first, every shard is padded to the largest, gathered with one equal-size collective,
    and the padding is trimmed, so the result is the concatenation of the shards in rank order."""
    if not dist.is_available() or not dist.is_initialized():
        return z_local
    world = dist.get_world_size(group)
    z_local = z_local.contiguous()
    n = torch.tensor([z_local.shape[0]], dtype=torch.int64, device=z_local.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    bmax = max(sizes)
    if z_local.shape[0] < bmax:
        pad = z_local.new_zeros((bmax - z_local.shape[0],) + tuple(z_local.shape[1:]))
        z_local = torch.cat([z_local, pad])
    out = torch.empty((world * bmax,) + tuple(z_local.shape[1:]), dtype=z_local.dtype, device=z_local.device)
    if z_local.is_cuda:
        dist.all_gather_into_tensor(out, z_local, group=group)
    else:  # gloo
        parts = list(out.chunk(world))
        dist.all_gather(parts, z_local, group=group)
    if all(s == bmax for s in sizes):
        return out
    return torch.cat([out[r * bmax:r * bmax + sizes[r]] for r in range(world)])

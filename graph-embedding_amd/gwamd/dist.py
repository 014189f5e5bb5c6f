"""Data-parallel sharding over GPUs (one process per GPU, torch.distributed).

The graph is replicated on every rank (RMAT-24 CSR ~8.5 GB of 288 GB HBM).
Units are independent:

* node2vec: global walk index w in [0, num_walks * n); walk w is a pure
  function of (seed, w) (Philox keyed), so a rank computes any contiguous
  block with no communication and the concatenation over ranks is identical
  to a single-GPU run.
* TopSim: query sources; each source's row depends only on (seed, source).

The only exchange step is optional: an all-gather of the emitted walks
(north_star: RCCL all-gather over xGMI), for consumers that need every walk
on every rank.  With backend "nccl" (= RCCL on ROCm) the tensors live in HBM;
the same code runs on "gloo" for CPU tests.
"""
import torch
import torch.distributed as dist


def shard_range(total, world, rank):
    """Contiguous block [begin, begin+count) of `total` units for `rank`
    (strong scaling: blocks differ by at most one unit)."""
    base, rem = divmod(int(total), int(world))
    begin = rank * base + min(rank, rem)
    count = base + (1 if rank < rem else 0)
    return begin, count


def weak_block(step, world, rank, block):
    """First global unit of (step, rank) when every rank processes `block`
    units per step (weak scaling): steps never overlap across ranks."""
    return (int(step) * int(world) + int(rank)) * int(block)


def allgather_rows(local, world, group=None):
    """All-gather row blocks of possibly different lengths (strong-scaling
    shards differ by one row): pads to the longest block, gathers with one
    collective, strips the padding.  Returns the concatenation in rank
    order."""
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes)
    if local.shape[0] < mx:
        pad = torch.full((mx - local.shape[0],) + tuple(local.shape[1:]), -1, dtype=local.dtype,
                         device=local.device)
        local = torch.cat([local, pad])
    out = torch.empty((world * mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if hasattr(dist, "all_gather_into_tensor") and local.device.type == "cuda":
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    else:
        chunks = list(out.chunk(world))
        dist.all_gather(chunks, local.contiguous(), group=group)
    parts = [out[r * mx:r * mx + sizes[r]] for r in range(world)]
    return torch.cat(parts)

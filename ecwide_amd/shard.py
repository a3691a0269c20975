"""Stripe partitioning across GPUs (one process per GPU, no collectives on
the data path).

Stripes are independent: a batch is split into contiguous
stripe ranges, each rank encodes/repairs its own range from its own HBM.
torch.distributed is used only to line ranks up for timing (barrier) and to
take the max of the per-rank times; with the nccl backend that is RCCL, but
no stripe byte ever crosses xGMI.
"""
from __future__ import annotations

import os


def dist_env() -> tuple:
    """(world, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def stripe_shard(total: int, world: int, rank: int) -> tuple:
    """Contiguous share of `total` stripes for `rank` (strong scaling):
    returns (first stripe id, count); the first total % world ranks get one more."""
    if world < 1 or not 0 <= rank < world or total < 0:
        raise ValueError("bad shard request")
    base, extra = divmod(total, world)
    count = base + (1 if rank < extra else 0)
    first = rank * base + min(rank, extra)
    return first, count


def column_shard(block_bytes: int, world: int, rank: int, align: int = 4096) -> tuple:
    """Byte-column share of every block for `rank` (SURVEY §8e fallback when a
    batch has fewer stripes than GPUs): every byte column of a stripe is
    independent, so rank i encodes/repairs columns [offset, offset + length)
    of all blocks. Slices are multiples of `align` (the kernels' 4 KiB column
    tile) except the last; returns (offset, length), length 0 for ranks past
    the end."""
    if world < 1 or not 0 <= rank < world or block_bytes < 0 or align < 1:
        raise ValueError("bad shard request")
    units = -(-block_bytes // align)
    base, extra = divmod(units, world)
    first = rank * base + min(rank, extra)
    count = base + (1 if rank < extra else 0)
    off = min(first * align, block_bytes)
    return off, min((first + count) * align, block_bytes) - off


def weak_shard(per_rank: int, rank: int) -> tuple:
    """Weak scaling: every rank owns `per_rank` stripes with distinct ids."""
    return rank * per_rank, per_rank


def max_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist

    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def host_threads(cap: int = 16) -> int:
    """CPU threads this process may use (the GPU box gives each GPU 16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        n = min(n, int(env))
    return max(1, min(n, cap))

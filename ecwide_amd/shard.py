"""Stripe partitioning across GPUs (one process per GPU, no collectives on
the data path).

Stripes are independent: a batch is split into contiguous
stripe ranges, each rank encodes/repairs its own range from its own HBM.
torch.distributed is used only to line ranks up for timing (barrier) and to
take the max of the per-rank times (bench.py runs those on gloo); no stripe
byte ever crosses xGMI.
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


def hbm_fill_block_mib(free_bytes: int, k: int, parity_num: int, stripes: int, frac: float = 0.97) -> int:
    """Block size (whole MiB) at which `stripes` stripes of k + parity_num
    blocks (+ 4 KiB padding per block) and a one-block-per-stripe repair
    output fit in `frac` of `free_bytes` (BASELINE configs[3])."""
    per_mib = stripes * ((k + parity_num) * ((1 << 20) + 4096) + (1 << 20))
    return int(frac * free_bytes) // per_mib


def plan_rank(stripes_total: int, block_bytes: int, world: int, rank: int, strong: bool,
              per_rank: int = 0, align: int = 4096) -> dict:
    """This rank's share of a batch (no data moves between ranks).

    * weak: `per_rank` stripes of its own (ids rank * per_rank ...);
    * strong: a contiguous range of the `stripes_total` stripes;
    * strong with fewer stripes than ranks: byte columns [col_offset,
      col_offset + block_bytes) of every stripe (column_shard, `align`-aligned).
    Returns {s0, stripes, block_bytes, col_offset, columns}."""
    if not strong:
        s0, n = weak_shard(per_rank, rank)
        return dict(s0=s0, stripes=n, block_bytes=block_bytes, col_offset=0, columns=False)
    if stripes_total < world:
        off, n = column_shard(block_bytes, world, rank, align=align)
        return dict(s0=0, stripes=stripes_total, block_bytes=n, col_offset=off, columns=True)
    s0, n = stripe_shard(stripes_total, world, rank)
    return dict(s0=s0, stripes=n, block_bytes=block_bytes, col_offset=0, columns=False)


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

"""The N>1 path on CPU: world_size-2 gloo ranks split a batch of stripes with
ecwide_amd.shard, each rank encodes its own stripes (oracle on CPU stands in
for the GPU here), and the union of the per-rank results equals the
single-process result — no stripe is lost or duplicated and nothing but
the timing max crosses ranks."""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from ecwide_amd.shard import column_shard, stripe_shard, weak_shard


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, total, q):
    import sys

    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import oracle
    from ecwide_amd.shard import max_over_ranks

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, count = stripe_shard(total, world, rank)
    orc = oracle.Oracle()
    oc = orc.codec("C", 12, 2, 4, 1024)
    out = {}
    for s in range(first, first + count):
        data = [orc.fill(1024, 5, s, j) for j in range(12)]
        par = oc.encode(data)
        out[s] = hashlib.sha256(b"".join(p.tobytes() for p in par)).hexdigest()
    t = max_over_ranks(float(rank + 1))
    dist.barrier()
    q.put((rank, out, t))
    dist.destroy_process_group()


def test_shard_math():
    for total in (0, 1, 7, 256):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                f, c = stripe_shard(total, world, r)
                seen += list(range(f, f + c))
            assert seen == list(range(total))
    assert weak_shard(8, 3) == (24, 8)
    with pytest.raises(ValueError):
        stripe_shard(4, 2, 2)


def test_column_shard_math():
    for B in (0, 1, 4095, 4096, 3 * 4096 + 100, 64 << 20):
        for world in (1, 2, 3, 8):
            cover = []
            for r in range(world):
                off, n = column_shard(B, world, r)
                assert n >= 0 and (n == 0 or off % 4096 == 0)
                if n and off + n < B:
                    assert n % 4096 == 0
                cover += list(range(off, off + n)) if B < 1 << 20 else [off, off + n]
            if B < 1 << 20:
                assert cover == list(range(B))
    assert column_shard(64 << 20, 8, 7) == (56 << 20, 8 << 20)
    with pytest.raises(ValueError):
        column_shard(4096, 2, 2)


def _col_worker(rank, world, port, q):
    import sys

    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B = 3 * 4096 + 100
    off, n = column_shard(B, world, rank)
    orc = oracle.Oracle()
    oc = orc.codec("C", 12, 2, 4, n)
    data = [orc.fill(B, 9, 0, j)[off:off + n].copy() for j in range(12)]
    q.put((rank, off, [p.tobytes() for p in oc.encode(data)]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_column_slices():
    """One stripe, two ranks: each encodes its byte columns; the slices
    concatenate to the single-process encode (SURVEY §8e fallback)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_col_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    import oracle

    orc = oracle.Oracle()
    B = 3 * 4096 + 100
    want = orc.codec("C", 12, 2, 4, B).encode([orc.fill(B, 9, 0, j) for j in range(12)])
    for i, w in enumerate(want):
        assert b"".join(parts[i] for _, _, parts in res) == w.tobytes()


def test_two_rank_gloo_partition():
    world, total = 2, 5
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    merged = {}
    for rank, out, t in res:
        assert t == float(world)  # max over ranks
        assert not set(out) & set(merged)
        merged.update(out)
    assert sorted(merged) == list(range(total))
    import oracle

    orc = oracle.Oracle()
    oc = orc.codec("C", 12, 2, 4, 1024)
    for s in range(total):
        par = oc.encode([orc.fill(1024, 5, s, j) for j in range(12)])
        assert merged[s] == hashlib.sha256(b"".join(p.tobytes() for p in par)).hexdigest()

#!/usr/bin/env python3
"""Host-resident encode + repair with the pinned staging on each NUMA node of
the host in turn (ecw_host_alloc_node), interleaved rounds in one process:
what NUMA-local staging (the bench's host leg) buys over the
other socket's DRAM. One stripe of CL(k, r, m) B-byte blocks per node.

  python tools/host_numa_ab.py [--k 128 --mib 64] [--rounds 3] [--iters 2]
"""
import argparse
import glob
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--r", type=int, default=27)
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=2)
    a = ap.parse_args()
    import numpy as np
    import torch

    import ecwide_amd as E

    nodes = sorted(int(p.rsplit("node", 1)[1]) for p in glob.glob("/sys/devices/system/node/node[0-9]*"))
    dev_node = E._lib.lib.ecw_device_numa_node(0)
    print(f"host NUMA nodes {nodes}; GPU 0 on node {dev_node}", flush=True)
    k, m, r, B = a.k, a.m, a.r, a.mib << 20
    codec = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    nblk = k + codec.parityNum
    slab = E.StripeSlab(codec, stripes=1, block_bytes=B)
    slab.fill_random(seed=103)
    slab.encode()
    want = [p.cpu().numpy() for p in slab.parity(0)]
    stage = {}
    for nd in nodes:
        t0 = time.perf_counter()
        h = E.PinnedHost((nblk + 1) * B, 0, node=nd)
        for j in range(k):
            torch.from_numpy(h.array[j * B:(j + 1) * B]).copy_(slab.block(0, j))
        stage[nd] = h
        print(f"node {nd}: staging on node {h.numa_node} ({time.perf_counter() - t0:.2f} s to allocate, pin, fill)",
              flush=True)
    del slab
    torch.cuda.synchronize()
    nsrc = len(codec.repairSources(0))
    step_b = nblk * B + (nsrc + 1) * B
    res = {nd: ([], []) for nd in nodes}
    for rd in range(a.rounds):
        for nd in (nodes if rd % 2 == 0 else nodes[::-1]):
            hb = stage[nd].array
            v = [hb[i * B:(i + 1) * B] for i in range(nblk + 1)]
            codec.encodeData(v[:k], v[k:nblk])
            t0 = time.perf_counter()
            for _ in range(a.iters):
                codec.encodeData(v[:k], v[k:nblk])
                codec.repairBlock(v[:nblk], 0, v[nblk])
            el = time.perf_counter() - t0
            res[nd][0].append(a.iters * step_b / el / 1e9)
            res[nd][1].append(a.iters * (k + nsrc) * B / el / 1e9)
            if rd == 0:
                ok = np.array_equal(v[nblk], v[0]) and all(np.array_equal(x, y) for x, y in zip(v[k:nblk], want))
                print(f"node {nd}: verified {ok}", flush=True)
    print(f"CL(k={k}, r={r}, m={m}) one stripe of {a.mib} MiB blocks in pinned host memory, encodeData + repair of D0, "
          f"median of {a.rounds} interleaved rounds x {a.iters}")
    for nd in nodes:
        tag = "local" if nd == dev_node else "remote"
        print(f"  staging on node {nd} ({tag}): {statistics.median(res[nd][0]):6.2f} GB/s, H2D "
              f"{statistics.median(res[nd][1]):6.2f} GB/s  rounds {[round(x, 1) for x in res[nd][0]]}", flush=True)


if __name__ == "__main__":
    main()

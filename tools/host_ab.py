#!/usr/bin/env python3
"""Host-resident encode + repair through two builds of libecwide.so on the same
pinned, NUMA-local host blocks, interleaved rounds in one process (the bench's
host leg): for host-pipeline changes (tools/variants.py builds,
e.g. -DECW_HOST_IN_STREAMS=1). Every build's parities and rebuilt block are
checked against the device-resident path's.

  python tools/host_ab.py build/variants/in1.so [--k 128 --mib 64] [--rounds 4] [--iters 2]
"""
import argparse
import os
import statistics
import sys
import time
from ctypes import byref, c_void_p

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+", help="other builds, timed beside ecwide_amd/libecwide.so")
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--r", type=int, default=27)
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=2)
    a = ap.parse_args()
    import numpy as np
    import torch

    import ecwide_amd as E
    from ecwide_amd import _lib

    k, m, r, B = a.k, a.m, a.r, a.mib << 20
    codec = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    np_ = codec.parityNum
    nblk = k + np_
    slab = E.StripeSlab(codec, stripes=1, block_bytes=B)
    slab.fill_random(seed=103)
    slab.encode()
    want = [p.cpu().numpy() for p in slab.parity(0)]
    h = E.PinnedHost((nblk + 1) * B, 0)
    for j in range(k):
        torch.from_numpy(h.array[j * B:(j + 1) * B]).copy_(slab.block(0, j))
    del slab
    torch.cuda.synchronize()
    print(f"pinned staging on NUMA node {h.numa_node} (GPU's node {_lib.lib.ecw_device_numa_node(0)})", flush=True)
    base = h.array.ctypes.data
    addr = [base + i * B for i in range(nblk + 1)]
    blocks = (c_void_p * (nblk + 1))(*addr)
    data = (c_void_p * k)(*addr[:k])
    par = (c_void_p * np_)(*addr[k:nblk])
    out = c_void_p(addr[nblk])
    builds = [("product", _lib.lib, codec._h)]
    for path in a.libs:
        L = _lib.load(path, strict=False)
        sch = _lib.ecw_scheme()
        assert L.ecw_scheme_init(byref(sch), b"C", k, m, r, B) == 0
        hh = c_void_p()
        assert L.ecw_codec_create(byref(sch), 1, 0, 0, 0, byref(hh)) == 0
        builds.append((os.path.basename(path).rsplit(".", 1)[0], L, hh))
    nsrc = len(codec.repairSources(0))
    step_b = nblk * B + (nsrc + 1) * B
    res = {n: [] for n, _, _ in builds}
    for rd in range(a.rounds):
        for name, L, hh in (builds if rd % 2 == 0 else builds[::-1]):
            run = lambda: (L.ecw_encode(hh, data, par, B), L.ecw_repair(hh, blocks, 0, out, B))
            assert run() == (0, 0), name
            t0 = time.perf_counter()
            for _ in range(a.iters):
                assert run() == (0, 0), name
            res[name].append(a.iters * step_b / (time.perf_counter() - t0) / 1e9)
            if rd < 2:
                v = h.array
                ok = np.array_equal(v[nblk * B:(nblk + 1) * B], v[:B]) and all(
                    np.array_equal(v[(k + i) * B:(k + i + 1) * B], w) for i, w in enumerate(want))
                assert ok, f"{name}: host results differ"
    print(f"CL(k={k}, r={r}, m={m}) one stripe of {a.mib} MiB blocks in pinned host memory, encode + repair of D0, "
          f"GB/s median of {a.rounds} interleaved rounds x {a.iters} (every build verified)")
    for name, v in res.items():
        print(f"  {name:10s} {statistics.median(v):7.2f} GB/s  rounds {[round(x, 1) for x in v]}", flush=True)


if __name__ == "__main__":
    main()

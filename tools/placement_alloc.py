#!/usr/bin/env python3
"""Does the allocation kind change the placement spread? Split-layout slabs
(bench shape, 4 stripes) allocated with hipExtMallocWithFlags: default
(hipDeviceMallocDefault) and physically contiguous (hipDeviceMallocContiguous),
NSLABS of each, encoded in interleaved rounds in one process.

  python tools/placement_alloc.py [--slabs 3] [--rounds 4]
  python tools/placement_alloc.py --offsets 0,4096,65536,1048576 --slabs 2
      (each slab encoded at several start offsets inside its allocation)
"""
import argparse
import ctypes
import os
import statistics
import sys
from ctypes import c_int, c_size_t, c_uint, c_void_p

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--r", type=int, default=27)
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--stripes", type=int, default=4)
    ap.add_argument("--slabs", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--offsets", default="0", help="slab start offsets (bytes) inside each allocation")
    a = ap.parse_args()
    import torch

    import ecwide_amd as E
    from ecwide_amd import _lib

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(c_void_p), c_size_t, c_uint]
    hip.hipFree.argtypes = [c_void_p]
    L = _lib.load()
    B, S = a.mib << 20, a.stripes
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(a.k, a.m, a.r, B), 1, False)
    k, np_ = c.encodeDataNum, c.parityNum
    bs = (B + 4096 + 255) // 256 * 256
    offs = [int(x) for x in a.offsets.split(",")]
    size = S * (k + np_) * bs + max(offs)
    st = c_void_p(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    slabs, allocs = [], []
    for kind, flag in (("default", 0), ("contiguous", 4)):
        for i in range(a.slabs):
            p = c_void_p()
            rc = hip.hipExtMallocWithFlags(ctypes.byref(p), size, flag)
            if rc != 0:
                print(f"{kind} #{i}: hipExtMallocWithFlags({size >> 30} GiB, {flag}) failed: {rc}")
                continue
            for o in offs:
                assert L.ecw_fill_random_pieces_dev(0, c_void_p(p.value + o), bs, k * bs, S, k, B, B, 0, 0, 103 + i,
                                                    0, 0, st) == 0
                slabs.append((f"{kind} #{i} +{o}", p.value + o))
            allocs.append(p.value)
    torch.cuda.synchronize()
    nbytes = S * (k + np_) * B

    def enc(base):
        rc = L.ecw_encode_batch_split_dev(c._h, c_void_p(base), bs, k * bs, c_void_p(base + S * k * bs), bs,
                                          np_ * bs, S, B, st)
        assert rc == 0, rc

    for _, base in slabs:
        enc(base)
    torch.cuda.synchronize()
    res = {n: [] for n, _ in slabs}
    for rd in range(a.rounds):
        for name, base in slabs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                enc(base)
            e1.record()
            torch.cuda.synchronize()
            res[name].append(3 * nbytes / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    print(f"CL(k={a.k},r={a.r},m={a.m}) B={a.mib} MiB x{S} stripes, split layout: encode GB/s median (min..max)")
    for name, base in slabs:
        xs = res[name]
        print(f"  {name:24s} {statistics.median(xs):7.1f} ({min(xs):6.1f}..{max(xs):6.1f}) base 0x{base:x}",
              flush=True)
    for base in allocs:
        hip.hipFree(c_void_p(base))


if __name__ == "__main__":
    main()

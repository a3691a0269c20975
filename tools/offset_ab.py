#!/usr/bin/env python3
"""Slab start offset inside ONE allocation (StripeSlab base_offset), A/B in
interleaved rounds: the slab is allocated once with room for the largest
offset, then re-based and re-filled per candidate, so physical placement is
the same for all of them. Repeated over --allocs allocations.

  python tools/offset_ab.py [--layout tiled] [--offsets 0,4096,8192] [--allocs 3]
"""
import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--r", type=int, default=27)
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--stripes", type=int, default=4)
    ap.add_argument("--layout", default="tiled")
    ap.add_argument("--offsets", default="0,4096,8192,2101248")
    ap.add_argument("--allocs", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch

    import ecwide_amd as E

    B = a.mib << 20
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(a.k, a.m, a.r, B), 1, False)
    offs = [int(x) for x in a.offsets.split(",")]
    slabs = [E.StripeSlab(c, stripes=a.stripes, block_bytes=B, layout=a.layout, base_offset=max(offs))
             for _ in range(a.allocs)]
    out = torch.empty(a.stripes * B, dtype=torch.uint8, device="cuda")
    enc_b, rep_b = slabs[0].encode_bytes(), slabs[0].repair_bytes(0)
    res = {(i, o): ([], []) for i in range(a.allocs) for o in offs}
    for rd in range(a.rounds):
        for i, sl in enumerate(slabs):
            for o in offs[rd % len(offs):] + offs[:rd % len(offs)]:
                sl.off, sl.base = o, sl.buf.data_ptr() + o
                sl.fill_random(seed=103)
                sl.encode()
                sl.repair(0, out)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ev[0].record()
                for _ in range(3):
                    sl.encode()
                ev[1].record()
                for _ in range(3):
                    sl.repair(0, out)
                ev[2].record()
                torch.cuda.synchronize()
                res[(i, o)][0].append(3 * enc_b / (ev[0].elapsed_time(ev[1]) * 1e-3) / 1e9)
                res[(i, o)][1].append(3 * rep_b / (ev[1].elapsed_time(ev[2]) * 1e-3) / 1e9)
    print(f"{a.layout} slab CL(k={a.k},r={a.r},m={a.m}) B={a.mib} MiB x{a.stripes}: GB/s median over {a.rounds} rounds")
    for i in range(a.allocs):
        line = "  ".join(f"+{o}: enc {statistics.median(res[(i, o)][0]):6.0f} rep {statistics.median(res[(i, o)][1]):6.0f}"
                         for o in offs)
        print(f"  alloc {i} (0x{slabs[i].buf.data_ptr():x}): {line}", flush=True)


if __name__ == "__main__":
    main()

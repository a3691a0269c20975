#!/usr/bin/env python3
"""Where do per-block pointers lose rate? Interleaved A/B in ONE process of
the bench encode (CL(128, 27, 3), 64 MiB blocks) over the same number of
stripes in several block placements:

  split4k   StripeSlab split layout, block stride B + 4 KiB (bench other_layout)
  split0    the same with block stride exactly B
  sep       every block its own torch.empty(B) (bench pointer leg)
  seppad    every block its own torch.empty(B + pad), first B bytes used
  carved    pointer tables into one allocation, block stride B + pad

  python tools/ptr_placement.py [--stripes 4] [--rounds 5] [--variants ...]
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
    ap.add_argument("--pad", type=int, default=4096)
    ap.add_argument("--variants", default="split4k,split0,sep,seppad,carved")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=4)
    a = ap.parse_args()
    import torch

    import ecwide_amd as E

    B, S = a.mib << 20, a.stripes
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(a.k, a.m, a.r, B), 1, False)
    k, np_ = c.encodeDataNum, c.parityNum
    gen = torch.Generator(device="cuda").manual_seed(7)
    keep = []

    def rand_(t):
        t.random_(0, 256, generator=gen)

    def blocks_sep(size):
        d = [[torch.empty(size, dtype=torch.uint8, device="cuda") for _ in range(k)] for _ in range(S)]
        p = [[torch.empty(size, dtype=torch.uint8, device="cuda") for _ in range(np_)] for _ in range(S)]
        for row in d:
            for t in row:
                rand_(t)
        return [[t[:B] for t in row] for row in d], [[t[:B] for t in row] for row in p]

    def blocks_carved(stride):
        dbuf = torch.empty(S * k * stride, dtype=torch.uint8, device="cuda")
        pbuf = torch.empty(S * np_ * stride, dtype=torch.uint8, device="cuda")
        rand_(dbuf)
        keep.extend([dbuf, pbuf])
        d = [[dbuf[(s * k + j) * stride:][:B] for j in range(k)] for s in range(S)]
        p = [[pbuf[(s * np_ + i) * stride:][:B] for i in range(np_)] for s in range(S)]
        return d, p

    runs = {}
    for v in a.variants.split(","):
        if v in ("split4k", "split0"):
            sl = E.StripeSlab(c, stripes=S, block_bytes=B, layout="split", pad=a.pad if v == "split4k" else 0)
            sl.fill_random(seed=103)
            keep.append(sl)
            runs[v] = sl.encode
            continue
        if v == "sep":
            d, p = blocks_sep(B)
        elif v == "seppad":
            d, p = blocks_sep(B + a.pad)
        elif v == "carved":
            d, p = blocks_carved(B + a.pad)
        else:
            raise SystemExit(f"unknown variant {v}")
        bb = E.BlockBatch(c, d, p)
        keep.append((d, p, bb))
        runs[v] = bb.encode
    torch.cuda.synchronize()
    nbytes = S * (k + np_) * B
    res = {v: [] for v in runs}
    names = list(runs)
    for rd in range(a.rounds):
        order = names[rd % len(names):] + names[:rd % len(names)]
        for v in order:
            runs[v]()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                runs[v]()
            e1.record()
            torch.cuda.synchronize()
            res[v].append(nbytes * a.iters / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    print(f"CL(k={a.k},r={a.r},m={a.m}) B={a.mib} MiB x{S} stripes, pad {a.pad}: encode GB/s median "
          f"(min..max) over {a.rounds} interleaved rounds")
    for v, xs in res.items():
        print(f"  {v:8s} {statistics.median(xs):7.1f} ({min(xs):6.1f}..{max(xs):6.1f})  frac "
              f"{statistics.median(xs) / 8000:.3f}", flush=True)


if __name__ == "__main__":
    main()

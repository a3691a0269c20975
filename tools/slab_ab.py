#!/usr/bin/env python3
"""Bench-step A/B of StripeSlab layouts in ONE process: every layout's slab
allocated side by side, rounds interleaved (layout order rotated each round),
encode and D0-repair timed with events per round. The bench's own workload
(CL(128, 27, 3), 64 MiB blocks, 8 stripes) by default.

  python tools/slab_ab.py [--layouts tiled,split] [--rounds 6] [--iters 5]
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
    ap.add_argument("--stripes", type=int, default=8)
    ap.add_argument("--layouts", default="tiled,split")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    import torch

    import ecwide_amd as E

    B = a.mib << 20
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(a.k, a.m, a.r, B), 1, False)
    slabs = {}
    for name in a.layouts.split(","):
        sl = E.StripeSlab(c, stripes=a.stripes, block_bytes=B, layout=name)
        sl.fill_random(seed=103)
        slabs[name] = (sl, torch.empty(a.stripes * B, dtype=torch.uint8, device="cuda"))
    enc_b = slabs[next(iter(slabs))][0].encode_bytes()
    rep_b = slabs[next(iter(slabs))][0].repair_bytes(0)
    res = {n: ([], [], []) for n in slabs}
    names = list(slabs)
    for rd in range(a.rounds):
        order = names[rd % len(names):] + names[:rd % len(names)]
        for name in order:
            sl, out = slabs[name]
            sl.encode()
            sl.repair(0, out)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record()
            for _ in range(a.iters):
                sl.encode()
            ev[1].record()
            for _ in range(a.iters):
                sl.repair(0, out)
            ev[2].record()
            torch.cuda.synchronize()
            e_ms, r_ms = ev[0].elapsed_time(ev[1]) / a.iters, ev[1].elapsed_time(ev[2]) / a.iters
            res[name][0].append(enc_b / e_ms / 1e6)
            res[name][1].append(rep_b / r_ms / 1e6)
            res[name][2].append((enc_b + rep_b) / (e_ms + r_ms) / 1e6)
    print(f"CL(k={a.k},r={a.r},m={a.m}) B={a.mib} MiB x{a.stripes}: GB/s median (min..max) over {a.rounds} "
          f"interleaved rounds")
    for name, (e, r, st) in res.items():
        f = lambda v: f"{statistics.median(v):7.1f} ({min(v):6.1f}..{max(v):6.1f})"
        print(f"  {name:8s} encode {f(e)}  repair {f(r)}  step {f(st)}", flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Does one huge slab run slower than the same stripes in several smaller
allocations? Encode + repair of S stripes (8 MiB blocks, tiled) as one
StripeSlab and as S/C slabs of C stripes, same process, alternating phases.

  python tools/slab_split.py [--stripes 256 --chunk 32 --rounds 2]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=256)
    ap.add_argument("--chunk", type=int, default=32)
    ap.add_argument("--mib", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    import torch

    import ecwide_amd as E
    B = a.mib << 20
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(128, 3, 27, B), 1, False)

    def timed(slabs):
        outs = [torch.empty(sl.stripes * B, dtype=torch.uint8, device="cuda") for sl in slabs]
        for i, sl in enumerate(slabs):
            sl.fill_random(seed=5, s0=i * sl.stripes)
            sl.encode()
            sl.repair(0, outs[i])
        torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        for _ in range(a.iters):
            for sl in slabs:
                sl.encode()
        e[1].record()
        for _ in range(a.iters):
            for i, sl in enumerate(slabs):
                sl.repair(0, outs[i])
        e[2].record()
        torch.cuda.synchronize()
        eb = sum(sl.encode_bytes() for sl in slabs) * a.iters
        rb = sum(sl.repair_bytes(0) for sl in slabs) * a.iters
        te, tr = e[0].elapsed_time(e[1]) * 1e-3, e[1].elapsed_time(e[2]) * 1e-3
        return eb / te / 1e9, rb / tr / 1e9, (eb + rb) / (te + tr) / 1e9

    for rnd in range(a.rounds):
        for name, n, per in (("one slab", 1, a.stripes), (f"{a.stripes // a.chunk} slabs", a.stripes // a.chunk, a.chunk)):
            slabs = [E.StripeSlab(c, stripes=per, block_bytes=B, layout="tiled", chunk=8192) for _ in range(n)]
            enc, rep, step = timed(slabs)
            print(f"round {rnd} {name:10s} x {per:3d} stripes: encode {enc:7.1f}  repair {rep:7.1f}  step {step:7.1f} GB/s",
                  flush=True)
            del slabs
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

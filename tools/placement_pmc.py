#!/usr/bin/env python3
"""Physical-placement study: several identical split slabs (bench shape, fewer
stripes) in one process; each is encoded in turn, round after round, and its
rate printed. Run plain for the rates, and under `rocprofv3 --pmc ...` to get
per-dispatch counters: the encode dispatches come in the order printed
("order"), so `--summarize <counter_collection.csv>` groups them per slab.

  python tools/placement_pmc.py [--slabs 4] [--stripes 4] [--rounds 3]
  python tools/placement_pmc.py --summarize gpurun_out/pmc/..._counter_collection.csv --slabs 4 --rounds 3
"""
import argparse
import csv
import os
import statistics
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def summarize(path, slabs, rounds):
    # per dispatch: counter values (one row per counter per dispatch)
    disp = defaultdict(dict)
    names = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            kn = row.get("Kernel_Name", "")
            if "encode_kernel" not in kn:
                continue
            d = int(row["Dispatch_Id"])
            names[d] = kn
            disp[d][row["Counter_Name"]] = disp[d].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    ids = sorted(disp)
    if not ids or len(ids) % (slabs * (rounds + 1)):
        raise SystemExit(f"{len(ids)} encode dispatches, not a multiple of {slabs} x ({rounds} + 1)")
    per = len(ids) // (slabs * (rounds + 1))
    ids = ids[slabs * per:]  # the warm-up encodes
    agg = defaultdict(lambda: defaultdict(float))
    for n, d in enumerate(ids):
        slab = (n // per) % slabs
        for c, v in disp[d].items():
            agg[slab][c] += v / rounds
    counters = sorted({c for s in agg.values() for c in s})
    print("per-slab mean per encode over", rounds, "rounds,", per, "dispatches each")
    print("slab " + " ".join(f"{c:>34s}" for c in counters))
    for s in sorted(agg):
        print(f"{s:4d} " + " ".join(f"{agg[s][c]:34.4g}" for c in counters))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--r", type=int, default=27)
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--stripes", type=int, default=4)
    ap.add_argument("--slabs", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--layout", default="split")
    ap.add_argument("--summarize", default=None)
    ap.add_argument("--extra", action="store_true", help="also time repair and a 4 GiB copy per slab")
    a = ap.parse_args()
    if a.summarize:
        return summarize(a.summarize, a.slabs, a.rounds)
    import torch

    import ecwide_amd as E

    B = a.mib << 20
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(a.k, a.m, a.r, B), 1, False)
    slabs = []
    for i in range(a.slabs):
        sl = E.StripeSlab(c, stripes=a.stripes, block_bytes=B, layout=a.layout)
        sl.fill_random(seed=103 + i)
        slabs.append(sl)
    for sl in slabs:  # warm-up: tables, tickets
        sl.encode()
    torch.cuda.synchronize()
    nbytes = slabs[0].encode_bytes()
    rbytes = slabs[0].repair_bytes(0)
    cbytes = min(4 << 30, slabs[0].buf.numel())
    out = torch.empty(max(a.stripes * B, cbytes), dtype=torch.uint8, device="cuda")
    res = [([], [], []) for _ in slabs]

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e-3

    for rd in range(a.rounds):
        for i, sl in enumerate(slabs):
            res[i][0].append(nbytes / timed(sl.encode) / 1e9)
        if a.extra:
            for i, sl in enumerate(slabs):
                res[i][1].append(rbytes / timed(lambda: sl.repair(0, out)) / 1e9)
                # read 4 GiB of the slab, write them to `out` (both counted)
                res[i][2].append(2 * cbytes / timed(lambda: out[:cbytes].copy_(sl.buf[:cbytes])) / 1e9)
    print(f"order: {a.slabs} warm-up encodes, then {a.rounds} rounds of slabs 0..{a.slabs - 1}")
    f = lambda xs: f"{statistics.median(xs):7.1f} ({min(xs):6.1f}..{max(xs):6.1f})" if xs else "-"
    for i, (e, r, cp) in enumerate(res):
        print(f"slab {i}: encode {f(e)} repair {f(r)} copy {f(cp)} GB/s base 0x{slabs[i].buf.data_ptr():x}",
              flush=True)


if __name__ == "__main__":
    main()

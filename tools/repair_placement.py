#!/usr/bin/env python3
"""Placement robustness of the tiled slab's CL repair.

Several identical tiled slabs (the bench's headline layout: 8 KiB column
pieces, CL(128, 27, 3), 64 MiB blocks) and one split slab (whole blocks: the
reference layout, as a same-process yardstick) are allocated side by side in
ONE process; where each allocation lands physically sets its rate (DESIGN.md
§5). Every XOR schedule (ecw_set_schedule: K column tiles per workgroup read
diagonally, group order, write window) is timed on every slab in interleaved
rounds, and a schedule is judged by its WORST slab, not its median: the bench
line gets one allocation, and a schedule that is fast on a good placement but
slow on a bad one is what the driver's box sees.

  python tools/repair_placement.py [--slabs 5] [--stripes 4] [--rounds 4] [--scheds auto 1,0 2,0,11,64 ...]
  rocprofv3 --pmc ... -- python3 tools/repair_placement.py --pmc-reps 3 ...   (fixed dispatch order)
  python tools/repair_placement.py --summarize <counter_collection.csv> [same --slabs/--scheds/--pmc-reps]
  python tools/repair_placement.py --scheds auto --enc-libs build/variants/ring3.so ...   (encode builds A/B)

Schedules are "K,ORDER[,LOG2P,W]" (ecwide_amd.parse_schedule; no window unless
given) or "auto" (the library's own choice). --enc-libs times every slab's
encode through other builds of the library too (tools/variants.py: compile-time
tile changes), on the same slabs in the same rounds, after checking that each
build writes the same parity bytes as the package's own.
"""
import argparse
import csv
import os
import statistics
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SCHEDS = ["auto", "1,0", "2,0", "4,0", "1,0,11,64", "2,0,11,64", "4,0,11,64", "2,0,10,32", "4,0,10,32", "2,1,11,64"]


def legs(a):
    """(slab index, schedule) in the order the PMC mode dispatches them."""
    names = [f"T{i}" for i in range(a.slabs)] + (["S"] if a.split else [])
    return [(n, sc) for n in names for sc in a.scheds]


def run(a):
    import torch

    import ecwide_amd as E

    k, m, r, B, S = a.k, a.m, a.r, a.mib << 20, a.stripes
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    slabs = {}
    order = [f"T{i}" for i in range(a.slabs)]
    if a.split:
        order.insert(min(a.split_at, len(order)), "S")
    for n in order:  # allocated in this order, side by side
        sl = E.StripeSlab(c, stripes=S, block_bytes=B, layout="split" if n == "S" else "tiled")
        sl.fill_random(seed=a.seed)
        slabs[n] = sl
    out = torch.empty(S * B, dtype=torch.uint8, device="cuda")
    for n, sl in slabs.items():
        sl.encode()
    torch.cuda.synchronize()
    print("allocation order " + " ".join(f"{n}@0x{slabs[n].buf.data_ptr():x}" for n in order), flush=True)
    elibs = []  # (name, encode fn per slab) for each extra build of the library
    if a.enc_libs:
        from ctypes import byref, c_void_p

        from ecwide_amd import _lib
        st = c_void_p(torch.cuda.current_stream().cuda_stream)
        for path in a.enc_libs:
            L = _lib.load(path, strict=False)
            sch = _lib.ecw_scheme()
            assert L.ecw_scheme_init(byref(sch), b"C", k, m, r, B) == 0
            h = c_void_p()
            assert L.ecw_codec_create(byref(sch), 1, 0, 0, 0, byref(h)) == 0

            def enc(sl, L=L, h=h):
                n_, len_ = (sl.units, sl.chunk) if sl.layout == "tiled" else (sl.stripes, sl.len)
                assert L.ecw_encode_batch_split_dev(h, *sl._split_args(), n_, len_, st) == 0
            elibs.append((os.path.basename(path).rsplit(".", 1)[0], enc))
        np_ = c.parityNum
        for n, sl in slabs.items():  # same parity bytes as the package's build, every slab
            want = [sl.block(s, k + i).clone() for s in (0, S - 1) for i in range(np_)]
            for name, enc in elibs:
                sl.buf[sl.off + sl.parity_offset:].zero_()  # the parity region ends the slab's buffer
                enc(sl)
                torch.cuda.synchronize()
                got = [sl.block(s, k + i) for s in (0, S - 1) for i in range(np_)]
                if not all(torch.equal(x, y) for x, y in zip(got, want)):
                    raise SystemExit(f"slab {n}: build {name} writes other parity bytes")
        print(f"every slab's parity identical under {len(elibs)} other build(s)", flush=True)
    rbytes = slabs[order[0]].repair_bytes(0)
    ebytes = slabs[order[0]].encode_bytes()
    names = list(slabs)

    def timed(fn, iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e-3 / iters

    def set_sched(sc):
        E.set_schedule(**E.parse_schedule(xor=None if sc == "auto" else sc))

    # every (slab, schedule) once, checked against D0
    for n in names:
        for sc in a.scheds:
            set_sched(sc)
            out.fill_(0)
            slabs[n].repair(0, out)
            torch.cuda.synchronize()
            for s in (0, S - 1):
                if not torch.equal(out[s * B:(s + 1) * B], slabs[n].block(s, 0)):
                    raise SystemExit(f"slab {n} schedule {sc}: repair != D0 (stripe {s})")
    print(f"every (slab, schedule) repair == D0 ({len(names)} slabs x {len(a.scheds)} schedules)", flush=True)
    if a.pmc_reps:
        # fixed order for the counter passes: legs() order, pmc_reps dispatches each
        for n, sc in legs(a):
            set_sched(sc)
            for _ in range(a.pmc_reps):
                slabs[n].repair(0, out)
            torch.cuda.synchronize()
        E.set_schedule()
        for n in names:  # then each slab's encode (its placement's rate for the streaming mix)
            for _ in range(a.pmc_reps):
                slabs[n].encode()
        torch.cuda.synchronize()
        print("pmc order done", flush=True)
        return
    rep = defaultdict(list)
    enc = defaultdict(list)
    encs = defaultdict(list)  # (slab, encode schedule) -> GB/s
    combos = [(n, sc) for n in names for sc in a.scheds]
    ecombos = [(n, w) for n in names for w in a.enc_scheds] + [(n, "lib:" + nm) for n in names for nm, _ in elibs]
    efn = dict(elibs)
    for rd in range(a.rounds):
        rot = combos[(rd * 7) % len(combos):] + combos[:(rd * 7) % len(combos)]
        for n, sc in rot:
            set_sched(sc)
            rep[(n, sc)].append(rbytes / timed(lambda: slabs[n].repair(0, out), a.iters) / 1e9)
        E.set_schedule()
        for n in names:
            enc[n].append(ebytes / timed(slabs[n].encode, 2) / 1e9)
        erot = ecombos[(rd * 5) % max(1, len(ecombos)):] + ecombos[:(rd * 5) % max(1, len(ecombos))]
        for n, w in erot:  # the encode under each write-window / tile-order setting
            if w.startswith("lib:"):
                E.set_schedule()
                encs[(n, w)].append(ebytes / timed(lambda: efn[w[4:]](slabs[n]), 2) / 1e9)
                continue
            base, _, rflag = w.partition("+")
            E.set_schedule(**E.parse_schedule(window=base, remap="1" if rflag == "r" else None))
            encs[(n, w)].append(ebytes / timed(slabs[n].encode, 2) / 1e9)
        E.set_schedule()
        print(f"round {rd + 1}/{a.rounds} done", flush=True)
    E.set_schedule()
    med = {key: statistics.median(v) for key, v in rep.items()}
    print(f"\nCL(k={k}, r={r}, m={m}) B={a.mib} MiB x {S} stripes per slab; D0 repair GB/s, median of {a.rounds} "
          f"interleaved rounds x {a.iters} launches; T* = tiled slabs (8 KiB pieces), S = split slab")
    print("slab  encode  " + " ".join(f"{sc:>11s}" for sc in a.scheds))
    for n in names:
        print(f"{n:4s} {statistics.median(enc[n]):7.1f} " + " ".join(f"{med[(n, sc)]:11.1f}" for sc in a.scheds))
    tiled = [n for n in names if n.startswith("T")]
    print("\nper schedule over the tiled slabs: worst / median / best (GB/s), worst vs the split slab's default")
    split_auto = med.get(("S", "auto"))
    rank = []
    for sc in a.scheds:
        v = sorted(med[(n, sc)] for n in tiled)
        rel = f"  worst/split_auto {v[0] / split_auto:.4f}" if split_auto else ""
        print(f"  {sc:11s} {v[0]:7.1f} {statistics.median(v):7.1f} {v[-1]:7.1f}{rel}")
        rank.append((v[0], sc))
    best = max(rank)
    print(f"best by worst tiled slab: {best[1]} ({best[0]:.1f} GB/s)")
    if split_auto:
        sv = [med[("S", sc)] for sc in a.scheds]
        print("split slab: " + " ".join(f"{sc}={x:.1f}" for sc, x in zip(a.scheds, sv)))
    ecols = a.enc_scheds + ["lib:" + nm for nm, _ in elibs]
    if ecols:
        emed = {key: statistics.median(v) for key, v in encs.items()}
        print(f"\nencode GB/s per slab under each encode schedule (window: auto | off | on | LOG2P,W; +r = per-XCD "
              f"tile order), median of {a.rounds} rounds x 2 encodes")
        print("slab " + " ".join(f"{w:>10s}" for w in ecols))
        for n in names:
            print(f"{n:4s} " + " ".join(f"{emed[(n, w)]:10.1f}" for w in ecols))
        print("per encode schedule over the tiled slabs: worst / median / best")
        erank = []
        for w in ecols:
            v = sorted(emed[(n, w)] for n in tiled)
            print(f"  {w:10s} {v[0]:7.1f} {statistics.median(v):7.1f} {v[-1]:7.1f}")
            erank.append((v[0], w))
        print(f"best encode schedule by worst tiled slab: {max(erank)[1]} ({max(erank)[0]:.1f} GB/s)")


def _csv_rows(path):
    with open(path) as f:
        yield from csv.DictReader(f)


def summarize(a):
    """Counters (and, with a kernel trace of the same run, durations) per
    (slab, schedule); per schedule the slowest and fastest tiled slab side by
    side -- what the worst placement pays for."""
    per = defaultdict(lambda: defaultdict(float))
    dur = {}
    for path in a.summarize:
        for row in _csv_rows(path):
            name = row.get("Kernel_Name", "")
            if "xor_kernel_fixed" not in name:
                continue
            d = int(row["Dispatch_Id"])
            if "Counter_Name" in row:
                per[d][row["Counter_Name"]] += float(row["Counter_Value"])
            elif "Start_Timestamp" in row:
                dur[d] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6  # ms
    ids = sorted(per or dur)
    L = legs(a)
    ids = ids[len(L):]  # the correctness pass dispatches every leg once first
    if len(ids) != len(L) * a.pmc_reps:
        print(f"warning: {len(ids)} timed xor dispatches, expected {len(L) * a.pmc_reps}")
    B, S = a.mib << 20, a.stripes
    alg = S * (a.r + 1) * B
    res = {}
    for i, (n, sc) in enumerate(L):
        grp = ids[i * a.pmc_reps:(i + 1) * a.pmc_reps]
        if not grp:
            break
        cs = sorted({c for d in grp for c in per[d]})
        avg = {c: sum(per[d][c] for d in grp) / len(grp) for c in cs}
        ms = sum(dur[d] for d in grp if d in dur) / max(1, sum(1 for d in grp if d in dur)) if dur else None
        res[(n, sc)] = (avg, ms)
    def line(n, sc):
        avg, ms = res[(n, sc)]
        extra = f" {ms:.4f} ms = {alg / (ms * 1e-3) / 1e9:.1f} GB/s" if ms else ""
        if avg.get("TCC_EA0_RDREQ_sum") and "TCC_EA0_RDREQ_LEVEL_sum" in avg:
            extra += f" | read level/req {avg['TCC_EA0_RDREQ_LEVEL_sum'] / avg['TCC_EA0_RDREQ_sum']:.1f}"
        if avg.get("TCC_EA0_WRREQ_sum") and "TCC_EA0_WRREQ_LEVEL_sum" in avg:
            extra += f" | write level/req {avg['TCC_EA0_WRREQ_LEVEL_sum'] / avg['TCC_EA0_WRREQ_sum']:.1f}"
        if "FETCH_SIZE" in avg:
            extra += f" | read/alg {avg['FETCH_SIZE'] * 1024 * 2 / (S * a.r * B):.5f}"
        if "WRITE_SIZE" in avg:
            extra += f" | write/alg {avg['WRITE_SIZE'] * 1024 / (S * B):.5f}"
        return f"{n:3s} {sc:11s}{extra} | " + " ".join(f"{c}={v:.4g}" for c, v in avg.items())
    for n, sc in L:
        if (n, sc) in res:
            print(line(n, sc))
    if dur:
        print("per schedule: slowest / fastest tiled slab (this run's own durations)")
        for sc in a.scheds:
            tl = [(res[(n, sc)][1], n) for n, s2 in L if s2 == sc and n.startswith("T") and (n, sc) in res]
            if tl:
                print("  slowest " + line(max(tl)[1], sc))
                print("  fastest " + line(min(tl)[1], sc))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--r", type=int, default=27)
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--stripes", type=int, default=4)
    ap.add_argument("--slabs", type=int, default=5)
    ap.add_argument("--split", type=int, default=1, help="1: also a split slab (the same-process yardstick)")
    ap.add_argument("--split-at", type=int, default=2, help="its position in the allocation order")
    ap.add_argument("--scheds", nargs="+", default=SCHEDS)
    ap.add_argument("--enc-scheds", nargs="*", default=[],
                    help="also time each slab's encode under these write-window settings (auto | off | on | "
                         "LOG2P,W, '+r' = per-XCD tile order)")
    ap.add_argument("--enc-libs", nargs="*", default=[],
                    help="also time each slab's encode through these builds of libecwide.so (tools/variants.py)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--seed", type=int, default=103)
    ap.add_argument("--pmc-reps", type=int, default=0)
    ap.add_argument("--summarize", nargs="*")
    a = ap.parse_args()
    summarize(a) if a.summarize else run(a)

#!/usr/bin/env python3
"""Counter evidence for the XOR schedules: one process,
the bench's pointer-leg placement (every 64 MiB block its own torch.empty) and
the split slab, CL(128, 27, 3) D0 repair, each schedule run `--reps` times in
a fixed order, so the xor_kernel_fixed dispatches of a rocprofv3 run come in
the order printed:

  rocprofv3 --kernel-trace --stats ... -- python3 tools/repair_pmc.py
  rocprofv3 --pmc FETCH_SIZE ... -- python3 tools/repair_pmc.py
  python tools/repair_pmc.py --summarize <counter_collection.csv> [...]

--summarize averages every counter over each schedule's dispatches and adds
bytes per dispatch against the algorithmic (n + 1) * B * stripes.
"""
import argparse
import csv
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

LEGS = [("sep", "1,0"), ("sep", "4,0"), ("sep", "auto"), ("split", "1,0"), ("split", "4,0"), ("split", "auto")]
# then the encode of each placement (write window: the library's choice), `reps` encodes of 2 launches each
ENC_LEGS = ["sep", "split", "tiled"]
ENC_LAUNCHES = 2


def run(a):
    import torch

    import ecwide_amd as E

    k, m, r, B, S = 128, 3, 27, 64 << 20, a.stripes
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    np_ = c.parityNum
    gen = torch.Generator(device="cuda").manual_seed(3)
    data = [[torch.empty(B, dtype=torch.uint8, device="cuda") for _ in range(k)] for _ in range(S)]
    par = [[torch.empty(B, dtype=torch.uint8, device="cuda") for _ in range(np_)] for _ in range(S)]
    for row in data:
        for t in row:
            t.random_(0, 256, generator=gen)
    batch = E.BlockBatch(c, data, par)
    split = E.StripeSlab(c, stripes=S, block_bytes=B, layout="split")
    split.fill_random(seed=5)
    out = torch.empty(S * B, dtype=torch.uint8, device="cuda")
    outs = [out[s * B:(s + 1) * B] for s in range(S)]
    batch.encode()
    split.encode()
    torch.cuda.synchronize()
    rep = {"sep": lambda: batch.repair(0, outs), "split": lambda: split.repair(0, out)}
    d0 = {"sep": lambda: data[0][0], "split": lambda: split.block(0, 0)}
    ok = True
    for place, sched in LEGS:
        E.set_schedule(**E.parse_schedule(xor=sched))
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record()
        for _ in range(a.reps):
            rep[place]()
        e[1].record()
        torch.cuda.synchronize()
        ms = e[0].elapsed_time(e[1]) / a.reps
        print(f"{place:6s} sched {sched:5s} {a.reps} dispatches, {ms:.4f} ms each, "
              f"{S * (r + 1) * B / (ms * 1e-3) / 1e9:.1f} GB/s", flush=True)
        ok = ok and torch.equal(out[:B], d0[place]())  # (both placements repair into `out`)
    print(f"repairs == D0: {ok}")
    E.set_schedule()
    tiled = E.StripeSlab(c, stripes=S, block_bytes=B, layout="tiled")
    tiled.fill_random(seed=5)
    assert tiled.encode_launches() == ENC_LAUNCHES and split.encode_launches() == ENC_LAUNCHES
    enc = {"sep": batch.encode, "split": split.encode, "tiled": tiled.encode}
    for place in ENC_LEGS:
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record()
        for _ in range(a.reps):
            enc[place]()
        e[1].record()
        torch.cuda.synchronize()
        ms = e[0].elapsed_time(e[1]) / a.reps
        print(f"{place:6s} encode {a.reps} x {ENC_LAUNCHES} dispatches, {ms:.4f} ms per encode, "
              f"{S * (k + np_) * B / (ms * 1e-3) / 1e9:.1f} GB/s", flush=True)


def summarize(a):
    per = defaultdict(lambda: defaultdict(float))  # dispatch id -> counter -> value
    eper = defaultdict(lambda: defaultdict(float))
    names = {}
    for path in a.summarize:
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "")
                tgt = per if "xor_kernel_fixed" in name else eper if "encode_kernel_asm" in name else None
                if tgt is None:
                    continue
                d = int(row["Dispatch_Id"])
                tgt[d][row["Counter_Name"]] += float(row["Counter_Value"])
                names[d] = name
    summarize_encode(a, eper)
    ids = sorted(per)
    if len(ids) != len(LEGS) * a.reps:
        print(f"warning: {len(ids)} xor dispatches, expected {len(LEGS) * a.reps}")
    B, S = 64 << 20, a.stripes
    alg = S * 28 * B
    for i, (place, sched) in enumerate(LEGS):
        grp = ids[i * a.reps:(i + 1) * a.reps]
        if not grp:
            break
        counters = sorted({c for d in grp for c in per[d]})
        avg = {c: sum(per[d][c] for d in grp) / len(grp) for c in counters}
        extra = ""
        if "FETCH_SIZE" in avg:
            extra += f" read/alg {avg['FETCH_SIZE'] * 1024 * 2 / (S * 27 * B):.5f}"
        if "WRITE_SIZE" in avg:
            extra += f" write/alg {avg['WRITE_SIZE'] * 1024 / (S * B):.5f}"
        if "TCC_EA0_RDREQ_LEVEL_sum" in avg and avg.get("TCC_EA0_RDREQ_sum"):
            extra += f" read level/req {avg['TCC_EA0_RDREQ_LEVEL_sum'] / avg['TCC_EA0_RDREQ_sum']:.1f}"
        kern = names[grp[0]].split("(")[0][-60:]
        print(f"{place:6s} sched {sched:5s} [{kern}] " + " ".join(f"{c}={v:.4g}" for c, v in avg.items()) + extra
              + f" (algorithmic {alg / 1e9:.3f} GB/dispatch)")


def summarize_encode(a, eper):
    ids = sorted(eper)
    n = a.reps * ENC_LAUNCHES
    # the encodes before the timed legs (one per placement) come first: take the last len(ENC_LEGS) * n
    ids = ids[-len(ENC_LEGS) * n:]
    B, S, k, np_ = 64 << 20, a.stripes, 128, 8
    for i, place in enumerate(ENC_LEGS):
        grp = ids[i * n:(i + 1) * n]
        if not grp:
            break
        counters = sorted({c for d in grp for c in eper[d]})
        avg = {c: sum(eper[d][c] for d in grp) / len(grp) for c in counters}
        extra = ""
        if "FETCH_SIZE" in avg:
            extra += f" read/alg {avg['FETCH_SIZE'] * 1024 * 2 / (S * k * B / ENC_LAUNCHES):.5f}"
        if "WRITE_SIZE" in avg:
            extra += f" write/alg {avg['WRITE_SIZE'] * 1024 / (S * np_ * B / ENC_LAUNCHES):.5f}"
        if "TCC_EA0_RDREQ_LEVEL_sum" in avg and avg.get("TCC_EA0_RDREQ_sum"):
            extra += f" read level/req {avg['TCC_EA0_RDREQ_LEVEL_sum'] / avg['TCC_EA0_RDREQ_sum']:.1f}"
        print(f"{place:6s} encode (per launch) " + " ".join(f"{c}={v:.4g}" for c, v in avg.items()) + extra)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--summarize", nargs="*")
    a = ap.parse_args()
    summarize(a) if a.summarize else run(a)

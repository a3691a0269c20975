#!/usr/bin/env python3
"""CL repair (XOR of the r survivors of D0) over separately allocated blocks:
where does it lose against the slabs, and which XOR schedule wins it back?
One process, one libecwide.so build, every (placement, schedule) pair timed in
interleaved rounds (placement differs per allocation).

Placements (S stripes of CL(k, r, m), B-byte blocks):
  tiled     StripeSlab tiled layout (8 KiB pieces; the bench's headline layout)
  split     whole blocks at stride B + 4 KiB, parity blocks in a region of their own
  blocks    whole blocks at stride B + 4 KiB, [D.., G.., L..] per stripe (the block slab)
  sep       every block its own torch.empty(B) (the bench's pointer leg)
  carved0   pointer tables into one allocation, block stride exactly B
  carved4k  the same at block stride B + 4 KiB
Schedules ("K,ORDER[,LOG2P,W]", set with ecw_set_schedule; ecw_xor.hpp launch_xor_range):
  K tiles per workgroup read diagonally, ORDER 1 = column-major groups,
  LOG2P,W = write window; "auto" = the library's choice; a "+r" suffix (also on
  --enc-windows settings) adds the per-XCD tile order (xcd_remap = 1).

  python tools/repair_ab.py [--lib build/variants/X.so] [--stripes 4] [--scheds 1,0 2,0 4,0 ...]
"""
import argparse
import ctypes
import os
import statistics
import sys
from ctypes import byref, c_void_p

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(REPO, "ecwide_amd", "libecwide.so"))
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--r", type=int, default=27)
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--stripes", type=int, default=4)
    ap.add_argument("--chunk", type=int, default=8192, help="column piece of the tiled placement")
    ap.add_argument("--placements", default="tiled,split,sep,carved0,carved4k")
    ap.add_argument("--scheds", nargs="+", default=["1,0", "2,0", "4,0", "1,1", "4,1", "1,0,11,64", "4,0,11,64"])
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--encode", action="store_true", help="also time the encode of every placement")
    ap.add_argument("--enc-windows", nargs="*", default=[],
                    help="with --encode: encode write-window settings to time the encode under "
                         "(off | on | LOG2P,W; auto = the library's choice)")
    a = ap.parse_args()
    import torch

    from ecwide_amd import _lib
    from ecwide_amd.codec import apply_schedule, parse_schedule

    L = _lib.load(a.lib, strict=False)
    k, m, r, S = a.k, a.m, a.r, a.stripes
    B = a.mib << 20
    g = -(-k // r)
    np_ = m + g
    sch = _lib.ecw_scheme()
    assert L.ecw_scheme_init(byref(sch), b"C", k, m, r, B) == 0
    h = c_void_p()
    assert L.ecw_codec_create(byref(sch), 1, 0, 0, 0, byref(h)) == 0
    idx = (ctypes.c_int * 256)()
    nsrc = L.ecw_repair_sources(h, 0, idx, 256)
    srcs = list(idx[:nsrc])
    stream = c_void_p(torch.cuda.current_stream().cuda_stream)
    gen = torch.Generator(device="cuda").manual_seed(11)
    keep = []
    out = torch.empty(S * B, dtype=torch.uint8, device="cuda")
    outs = [out[s * B:(s + 1) * B] for s in range(S)]
    otab = torch.tensor([o.data_ptr() for o in outs], dtype=torch.int64, device="cuda")

    def tables(blocks):  # blocks[s][b], b in [D.., G.., L..]
        dtab = torch.tensor([blocks[s][j].data_ptr() for s in range(S) for j in range(k)], dtype=torch.int64,
                            device="cuda")
        ptab = torch.tensor([blocks[s][k + i].data_ptr() for s in range(S) for i in range(np_)],
                            dtype=torch.int64, device="cuda")
        stab = torch.tensor([blocks[s][i].data_ptr() for s in range(S) for i in srcs], dtype=torch.int64,
                            device="cuda")
        keep.append((blocks, dtab, ptab, stab))
        enc = lambda: L.ecw_encode_ptrs_dev(h, S, c_void_p(dtab.data_ptr()), c_void_p(ptab.data_ptr()), B, stream)
        rep = lambda: L.ecw_xor_reduce_ptrs_dev(0, S, nsrc, c_void_p(stab.data_ptr()), c_void_p(otab.data_ptr()),
                                                B, stream)
        return enc, rep, [(lambda s=s: blocks[s][0]) for s in range(S)]

    legs = {}
    for p in a.placements.split(","):
        if p in ("tiled", "split"):
            if p == "tiled":
                ch = a.chunk
                units = S * (B // ch)
                dbuf = torch.empty(units * k * ch, dtype=torch.uint8, device="cuda")
                pbuf = torch.empty(units * np_ * ch, dtype=torch.uint8, device="cuda")
                args = (c_void_p(dbuf.data_ptr()), ch, k * ch, c_void_p(pbuf.data_ptr()), ch, np_ * ch)
                n_units, ulen = units, ch
                d0 = [(lambda s=s, buf=dbuf, ch=ch: buf.view(S, B // ch, k, ch)[s, :, 0, :].reshape(-1)) for s in range(S)]
            else:
                bs = B + 4096
                dbuf = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
                pbuf = torch.empty(S * np_ * bs, dtype=torch.uint8, device="cuda")
                args = (c_void_p(dbuf.data_ptr()), bs, k * bs, c_void_p(pbuf.data_ptr()), bs, np_ * bs)
                n_units, ulen = S, B
                d0 = [(lambda s=s, buf=dbuf, bs=bs: buf[s * k * bs:s * k * bs + B]) for s in range(S)]
            dbuf.random_(0, 256, generator=gen)
            keep.append((dbuf, pbuf))
            enc = (lambda args=args, n=n_units, ln=ulen:
                   L.ecw_encode_batch_split_dev(h, *args, n, ln, stream))
            rep = (lambda args=args, n=n_units, ln=ulen:
                   L.ecw_repair_batch_split_dev(h, *args, n, 0, c_void_p(out.data_ptr()), ln, ln, stream))
            legs[p] = (enc, rep, d0)
            continue
        if p == "blocks":  # the block slab: [D.., G.., L..] per stripe at block stride B + 4 KiB
            bs = B + 4096
            big = torch.empty(S * (k + np_) * bs, dtype=torch.uint8, device="cuda")
            big.random_(0, 256, generator=gen)
            keep.append(big)
            enc = (lambda big=big, bs=bs:
                   L.ecw_encode_batch_dev(h, c_void_p(big.data_ptr()), bs, (k + np_) * bs, S, B, stream))
            rep = (lambda big=big, bs=bs:
                   L.ecw_repair_batch_dev(h, c_void_p(big.data_ptr()), bs, (k + np_) * bs, S, 0,
                                          c_void_p(out.data_ptr()), B, B, stream))
            d0 = [(lambda s=s, big=big, bs=bs: big[s * (k + np_) * bs:][:B]) for s in range(S)]
            legs[p] = (enc, rep, d0)
            continue
        if p == "sep":
            blocks = [[torch.empty(B, dtype=torch.uint8, device="cuda") for _ in range(k + np_)] for _ in range(S)]
            for row in blocks:
                for t in row[:k]:
                    t.random_(0, 256, generator=gen)
        elif p in ("carved0", "carved4k"):
            bs = B + (4096 if p == "carved4k" else 0)
            big = torch.empty(S * (k + np_) * bs, dtype=torch.uint8, device="cuda")
            big.random_(0, 256, generator=gen)
            keep.append(big)
            blocks = [[big[(s * (k + np_) + b) * bs:][:B] for b in range(k + np_)] for s in range(S)]
        else:
            raise SystemExit(f"unknown placement {p}")
        legs[p] = tables(blocks)
        # where the blocks start (virtual addresses; the physical pages are the driver's)
        pa = [blocks[s][b].data_ptr() for s in range(S) for b in srcs]
        print(f"# {p}: source starts mod 2 MiB {sorted({x % (2 << 20) for x in pa})[:4]}, "
              f"mod 64 MiB distinct {len({x % (64 << 20) for x in pa})}, first {hex(pa[0])}", flush=True)
    # every placement: encode once (L0 needed by the repair), check the repair
    for p, (enc, rep, d0) in legs.items():
        assert enc() == 0, p
        assert rep() == 0, p
        torch.cuda.synchronize()
        ok = all(torch.equal(out[s * B:(s + 1) * B], d0[s]()) for s in range(S))
        print(f"# {p}: repair == D0: {ok}", flush=True)
    rep_bytes = S * (nsrc + 1) * B
    enc_bytes = S * (k + np_) * B
    res, encw = {}, {}
    combos = [(p, sc) for p in legs for sc in a.scheds]
    for rd in range(a.rounds):
        order = combos[rd % len(combos):] + combos[:rd % len(combos)]
        for p, sc in order:
            enc, rep, d0 = legs[p]
            base, _, rflag = sc.partition("+")  # "+r": the per-XCD tile order
            apply_schedule(L, **parse_schedule(xor=base, remap="1" if rflag == "r" else None))
            assert rep() == 0
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            for _ in range(a.iters):
                rep()
            e[1].record()
            if a.encode and sc == a.scheds[0]:
                for _ in range(a.iters):
                    enc()
            e[2].record()
            torch.cuda.synchronize()
            rr = res.setdefault((p, sc), ([], []))
            rr[0].append(rep_bytes * a.iters / (e[0].elapsed_time(e[1]) * 1e-3) / 1e9)
            if a.encode and sc == a.scheds[0]:
                rr[1].append(enc_bytes * a.iters / (e[1].elapsed_time(e[2]) * 1e-3) / 1e9)
                for wv in a.enc_windows:  # the encode under other write-window settings, same round
                    wbase, _, rflag = wv.partition("+")
                    apply_schedule(L, **parse_schedule(window=wbase, remap="1" if rflag == "r" else None))
                    f = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                    enc()
                    f[0].record()
                    for _ in range(a.iters):
                        enc()
                    f[1].record()
                    torch.cuda.synchronize()
                    encw.setdefault((p, wv), []).append(enc_bytes * a.iters / (f[0].elapsed_time(f[1]) * 1e-3) / 1e9)
                apply_schedule(L)
            if rd == 0:
                ok = all(torch.equal(out[s * B:(s + 1) * B], d0[s]()) for s in range(S))
                if not ok:
                    print(f"  !! {p} sched {sc}: repair != D0", flush=True)
    apply_schedule(L)
    print(f"CL(k={k},r={r},m={m}) B={a.mib} MiB x{S} stripes, repair of D0 ({nsrc} sources): GB/s median "
          f"(min..max) over {a.rounds} interleaved rounds; lib {os.path.basename(a.lib)}")
    for (p, sc), (rp, en) in res.items():
        enc = f"   encode {statistics.median(en):7.1f}" if en else ""
        print(f"  {p:9s} sched {sc:11s} repair {statistics.median(rp):7.1f} ({min(rp):6.1f}..{max(rp):6.1f}) "
              f"frac {statistics.median(rp) / 8000:.3f}{enc}", flush=True)
    for (p, wv), en in encw.items():
        print(f"  {p:9s} encode, ECW_WRITE_WINDOW={wv:8s} {statistics.median(en):7.1f} ({min(en):6.1f}..{max(en):6.1f}) "
              f"frac {statistics.median(en) / 8000:.3f}", flush=True)


if __name__ == "__main__":
    main()

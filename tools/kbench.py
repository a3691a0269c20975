#!/usr/bin/env python3
"""Interleaved A/B timing of libecwide.so variants on one GPU (one process,
same data, rounds interleaved: cdna_hip_programming.md §5.4 rule 24).

  python tools/kbench.py [--k 128 --m 3 --r 27 --mib 64 --stripes 4 --rounds 5] build/variants/*.so

A lib given as PATH@VALUE runs with the encode write window VALUE (off | on |
LOG2P,W; ecw_set_schedule) set around its calls, so one build can be
A/B-ed against itself: ecwide_amd/libecwide.so@off ecwide_amd/libecwide.so@on.
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
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--r", type=int, default=27)
    ap.add_argument("--mib", type=float, default=64)
    ap.add_argument("--stripes", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--code", default="C", help="C (CL, locals) or R (RS, globals only)")
    ap.add_argument("--pad", type=int, default=4096, help="block stride = B + pad (rounded to 256)")
    ap.add_argument("--literal", action="store_true", help="ECWide-C literal local mode (zero L blocks)")
    ap.add_argument("--ptr", action="store_true",
                    help="encode each stripe with ecw_encode_dev and its blocks in reverse order "
                         "(pointer mode, not one stride apart)")
    ap.add_argument("--chunk", type=int, default=0,
                    help="chunk-interleaved layout: each stripe stored as B/CHUNK column chunks, "
                         "the k+m+g blocks' chunks adjacent (timed as B/CHUNK mini-stripes)")
    ap.add_argument("--split", action="store_true",
                    help="with --chunk: data chunks in one region, parities in another "
                         "(ecw_encode_batch_split_dev; encode only)")
    ap.add_argument("--tables", action="store_true",
                    help="pointer tables over separately allocated blocks (ecw_encode_ptrs_dev, the "
                         "bench's pointer leg; encode only)")
    a = ap.parse_args()
    assert not (a.tables and (a.check or a.split or a.ptr or a.chunk)), "--tables runs alone"
    import torch

    from ecwide_amd import _lib
    from ecwide_amd.codec import apply_schedule, parse_schedule

    k, m, r = a.k, a.m, a.r
    B = int(a.mib * (1 << 20))
    S = a.stripes
    if a.chunk:
        assert B % a.chunk == 0
        S, B = S * (B // a.chunk), a.chunk
    g = -(-k // r) if a.code == "C" else 0
    nblk = k + m + g
    bstride = (B + a.pad + 255) // 256 * 256
    sstride = nblk * bstride
    buf = torch.empty(S * sstride, dtype=torch.uint8, device="cuda")
    out = torch.empty(S * B, dtype=torch.uint8, device="cuda")
    stream = c_void_p(torch.cuda.current_stream().cuda_stream)
    libs = []
    envs = {}
    for spec in a.libs:
        path, _, env = spec.partition("@")
        L = _lib.load(path, strict=False)
        sch = _lib.ecw_scheme()
        assert L.ecw_scheme_init(byref(sch), a.code.encode(), k, m, r, B) == 0
        h = c_void_p()
        assert L.ecw_codec_create(byref(sch), 1, 0, 1 if a.literal else 0, 0, byref(h)) == 0
        name = os.path.basename(path) + (f"@{env}" if env else "")
        envs[name] = env
        libs.append((name, L, h))
    L0 = libs[0][1]
    if a.split:
        assert a.chunk and a.pad == 0, "--split needs --chunk and --pad 0"
        del buf
        buf = torch.empty(S * k * B, dtype=torch.uint8, device="cuda")
        pbuf = torch.empty(S * (m + g) * B, dtype=torch.uint8, device="cuda")
        bstride, sstride = B, k * B
    assert L0.ecw_fill_random_dev(0, c_void_p(buf.data_ptr()), bstride, sstride, S, k, B, 1, 0, 0, stream) == 0
    if a.tables:
        del buf
        blocks = [torch.empty(B, dtype=torch.uint8, device="cuda") for _ in range(S * nblk)]
        for t in blocks[:S * k]:
            t.random_(0, 256)
        dtab = torch.tensor([blocks[s_ * nblk + j].data_ptr() for s_ in range(S) for j in range(k)],
                            dtype=torch.int64, device="cuda")
        ptab = torch.tensor([blocks[s_ * nblk + k + i].data_ptr() for s_ in range(S) for i in range(m + g)],
                            dtype=torch.int64, device="cuda")
        buf = blocks[0]
        idx = (ctypes.c_int * 256)()
        # RS codes have no local groups: no repair sources, the repair leg is skipped
        nsrc = L0.ecw_repair_sources(libs[0][2], 0, idx, 256) if a.code == "C" else 0
        stab = torch.tensor([blocks[s_ * nblk + idx[i]].data_ptr() for s_ in range(S) for i in range(nsrc)],
                            dtype=torch.int64, device="cuda")
        outs = [torch.empty(B, dtype=torch.uint8, device="cuda") for _ in range(S)]
        otab = torch.tensor([o.data_ptr() for o in outs], dtype=torch.int64, device="cuda")
    enc_bytes = S * nblk * B
    rep_bytes = S * (r + 1) * B  # --tables: nsrc = r sources + 1 output as well
    ref = None
    if a.check:
        assert libs[0][1].ecw_encode_batch_dev(libs[0][2], c_void_p(buf.data_ptr()), bstride, sstride, S, B, stream) == 0
        torch.cuda.synchronize()
        ref = torch.stack([buf[s_ * sstride + k * bstride:s_ * sstride + nblk * bstride] for s_ in range(S)]).clone()
    if a.ptr:
        base = buf.data_ptr()
        dptrs = [(c_void_p * k)(*[base + s_ * sstride + (k - 1 - j) * bstride for j in range(k)]) for s_ in range(S)]
        pptrs = [(c_void_p * (m + g))(*[base + s_ * sstride + (nblk - 1 - i) * bstride for i in range(m + g)])
                 for s_ in range(S)]
    res = {n: ([], []) for n, _, _ in libs}
    for rd in range(a.rounds):
        for name, L, h in libs:
            if hasattr(L, "ecw_set_schedule"):  # (builds before round 5 read ECW_WRITE_WINDOW per launch)
                apply_schedule(L, **parse_schedule(window=envs[name] or None))
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            for it in range(a.iters + 1):
                if it == 1:
                    e[0].record()
                if a.tables:
                    st = L.ecw_encode_ptrs_dev(h, S, c_void_p(dtab.data_ptr()), c_void_p(ptab.data_ptr()), B, stream)
                    assert st == 0, (name, st)
                elif a.split:
                    st = L.ecw_encode_batch_split_dev(h, c_void_p(buf.data_ptr()), B, k * B,
                                                      c_void_p(pbuf.data_ptr()), B, (m + g) * B, S, B, stream)
                    assert st == 0, (name, st)
                elif a.ptr:
                    for s_ in range(S):
                        st = L.ecw_encode_dev(h, dptrs[s_], pptrs[s_], B, stream)
                        assert st == 0, (name, st)
                else:
                    st = L.ecw_encode_batch_dev(h, c_void_p(buf.data_ptr()), bstride, sstride, S, B, stream)
                    assert st == 0, (name, st)
            e[1].record()
            rep_iters = a.iters if a.code == "C" and not a.literal and not a.split and not (a.tables and nsrc <= 0) else 0  # literal L: no repair
            for it in range(rep_iters):
                if a.tables:
                    st = L.ecw_xor_reduce_ptrs_dev(0, S, nsrc, c_void_p(stab.data_ptr()), c_void_p(otab.data_ptr()),
                                                   B, stream)
                    assert st == 0, (name, st)
                    continue
                st = L.ecw_repair_batch_dev(h, c_void_p(buf.data_ptr()), bstride, sstride, S, 0,
                                            c_void_p(out.data_ptr()), B, B, stream)
                assert st == 0, (name, st)
            e[2].record()
            torch.cuda.synchronize()
            res[name][0].append(enc_bytes * a.iters / (e[0].elapsed_time(e[1]) * 1e-3) / 1e9)
            if rep_iters:
                res[name][1].append(rep_bytes * rep_iters / (max(e[1].elapsed_time(e[2]), 1e-6) * 1e-3) / 1e9)
            if ref is not None and "ablate" not in name:  # every parity block of every stripe (pads included)
                got = torch.stack([buf[s_ * sstride + k * bstride:s_ * sstride + nblk * bstride] for s_ in range(S)])
                if not torch.equal(got, ref):
                    print(f"  !! {name}: parity differs from {libs[0][0]}")
    print(f"{a.code}(k={k},r={r},m={m}) B={B} x{S} stripes pad={a.pad}; GB/s median (min..max) over {a.rounds} rounds")
    for name, (en, rp) in res.items():
        rep = f"repair {statistics.median(rp):8.1f} ({min(rp):7.1f}..{max(rp):7.1f})" if rp else "repair  (not run)"
        print(f"{name:28s} encode {statistics.median(en):8.1f} ({min(en):7.1f}..{max(en):7.1f})   {rep}", flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Slab layouts compared on the SAME physical memory: one allocation, every
variant carved out of it in turn, rounds interleaved. (Separate processes
land on different physical pages, which moves the rate by up to 4 % by
itself -- DESIGN.md section 5.)

  python tools/layout_ab.py [--k 128 --m 3 --r 27 --mib 64 --stripes 8 --rounds 3]
"""
import argparse
import os
import statistics
import sys
from ctypes import byref, c_void_p

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--r", type=int, default=27)
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--stripes", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--variants", default="blocks:4096,tiled:8192:0,tiled:8192:4096,tiled:8192:256,tiled:4096:0")
    ap.add_argument("--libs", default="", help="comma-separated libecwide.so builds to compare (default: the in-tree one)")
    a = ap.parse_args()
    import torch

    from ecwide_amd import _lib

    libs = [(os.path.basename(p), _lib.load(p, strict=False)) for p in a.libs.split(",") if p] or [("", _lib.lib)]
    L = libs[0][1]
    k, m, r, S = a.k, a.m, a.r, a.stripes
    B = a.mib << 20
    g = -(-k // r)
    np_ = m + g
    sch = _lib.ecw_scheme()
    assert L.ecw_scheme_init(byref(sch), b"C", k, m, r, B) == 0
    handles = []
    for _, Lx in libs:
        hx = c_void_p()
        assert Lx.ecw_codec_create(byref(sch), 1, 0, 0, 0, byref(hx)) == 0
        handles.append(hx)
    stream = c_void_p(torch.cuda.current_stream().cuda_stream)
    variants = []
    need = 0
    for spec in a.variants.split(","):
        p = spec.split(":")
        if p[0] == "blocks":
            pad = int(p[1])
            bs = (B + pad + 255) // 256 * 256
            variants.append(("blocks pad=%d" % pad, "blocks", bs, S * (k + np_) * bs, None))
            need = max(need, S * (k + np_) * bs)
        else:
            ch, up = int(p[1]), int(p[2])
            units = S * (B // ch)
            dst, pst = k * ch + up, np_ * ch + up
            poff = (units * dst + 4095) // 4096 * 4096
            variants.append(("tiled %dK unit_pad=%d" % (ch >> 10, up), "tiled", (ch, units, dst, pst, poff),
                             poff + units * pst, None))
            need = max(need, poff + units * pst)
    buf = torch.empty(need, dtype=torch.uint8, device="cuda")
    out = torch.empty(S * B, dtype=torch.uint8, device="cuda")
    base = buf.data_ptr()
    enc_bytes, rep_bytes = S * (k + np_) * B, S * (r + 1) * B
    res = {}

    def run(v, what, L, h):
        name, kind, geo, _, _ = v
        if kind == "blocks":
            bs = geo
            if what == "fill":
                return L.ecw_fill_random_dev(0, c_void_p(base), bs, (k + np_) * bs, S, k, B, 1, 0, 0, stream)
            if what == "enc":
                return L.ecw_encode_batch_dev(h, c_void_p(base), bs, (k + np_) * bs, S, B, stream)
            return L.ecw_repair_batch_dev(h, c_void_p(base), bs, (k + np_) * bs, S, 0, c_void_p(out.data_ptr()),
                                          B, B, stream)
        ch, units, dst, pst, poff = geo
        if what == "fill":
            return L.ecw_fill_random_dev(0, c_void_p(base), ch, dst, units, k, ch, 1, 0, 0, stream)
        if what == "enc":
            return L.ecw_encode_batch_split_dev(h, c_void_p(base), ch, dst, c_void_p(base + poff), ch, pst, units,
                                                ch, stream)
        return L.ecw_repair_batch_split_dev(h, c_void_p(base), ch, dst, c_void_p(base + poff), ch, pst, units, 0,
                                            c_void_p(out.data_ptr()), ch, ch, stream)

    for _ in range(a.rounds):
        for v in variants:
            for (lname, Lx), hx in zip(libs, handles):
                key = (v[0] + " " + lname).strip()
                res.setdefault(key, ([], []))
                assert run(v, "fill", Lx, hx) == 0
                assert run(v, "enc", Lx, hx) == 0 and run(v, "rep", Lx, hx) == 0
                e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                e[0].record()
                for _ in range(a.iters):
                    assert run(v, "enc", Lx, hx) == 0
                e[1].record()
                for _ in range(a.iters):
                    assert run(v, "rep", Lx, hx) == 0
                e[2].record()
                torch.cuda.synchronize()
                res[key][0].append(enc_bytes * a.iters / (e[0].elapsed_time(e[1]) * 1e-3) / 1e9)
                res[key][1].append(rep_bytes * a.iters / (e[1].elapsed_time(e[2]) * 1e-3) / 1e9)
    print(f"CL(k={k},r={r},m={m}) B={a.mib} MiB x{S} stripes, one allocation; GB/s median over {a.rounds} rounds")
    for name, (en, rp) in res.items():
        ee, rr = statistics.median(en), statistics.median(rp)
        step = (enc_bytes + rep_bytes) / (enc_bytes / ee + rep_bytes / rr)
        print(f"{name:40s} encode {ee:8.1f}  repair {rr:8.1f}  step {step:8.1f}", flush=True)


if __name__ == "__main__":
    main()

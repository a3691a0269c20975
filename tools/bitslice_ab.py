#!/usr/bin/env python3
"""Prototype A/B (tools/ only): the bit-sliced encode tile (tools/csrc/bitslice.hip)
against the product's encode on the bench's tiled geometry (8 KiB units,
ecw_encode_batch_split_dev), same buffers, rounds interleaved. The prototype's
parities are first compared byte for byte with the product's (which the GPU
suite pins to the oracle).

  python tools/bitslice_ab.py [--k 128 --m 3 --r 27 --stripes 8 --mib 64] build/bitslice.so [more.so ...]
"""
import argparse
import ctypes
import os
import statistics
import sys
from ctypes import byref, c_int, c_void_p

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("protos", nargs="+")
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--r", type=int, default=27)
    ap.add_argument("--code", default="C")
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--stripes", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=4)
    a = ap.parse_args()
    import torch

    from ecwide_amd import _lib

    k, m, r = a.k, a.m, a.r
    g = -(-k // r) if a.code == "C" else 0
    P = 8192
    S = a.stripes * (a.mib << 20) // P
    L = _lib.load()
    sch = _lib.ecw_scheme()
    assert L.ecw_scheme_init(byref(sch), a.code.encode(), k, m, r, P) == 0
    h = c_void_p()
    assert L.ecw_codec_create(byref(sch), 1, 0, 0, 0, byref(h)) == 0
    mat = (ctypes.c_uint8 * (m * k))()
    assert L.ecw_codec_encode_matrix(h, mat, m * k) == 0
    # 4 words per source: byte (i & 3) of word 4j + (i >> 2) = matrix[i][j]
    coef = [sum(mat[i * k + j] << (8 * (i & 3)) for i in range(m) if i >> 2 == w) for j in range(k) for w in range(4)]
    coef_t = torch.tensor(coef, dtype=torch.int64).to(torch.int32).cuda()
    data = torch.empty(S * k * P, dtype=torch.uint8, device="cuda")
    par = torch.empty(S * (m + g) * P, dtype=torch.uint8, device="cuda")
    stream = c_void_p(torch.cuda.current_stream().cuda_stream)
    assert L.ecw_fill_random_dev(0, c_void_p(data.data_ptr()), P, k * P, S, k, P, 1, 0, 0, stream) == 0

    def prod():
        st = L.ecw_encode_batch_split_dev(h, c_void_p(data.data_ptr()), P, k * P, c_void_p(par.data_ptr()), P,
                                          (m + g) * P, S, P, stream)
        assert st == 0, st

    protos = []
    for path in a.protos:
        lib = ctypes.CDLL(os.path.abspath(path))
        f = lib.bs_encode_split
        f.argtypes = [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]

        def run(f=f):
            st = f(c_void_p(data.data_ptr()), c_void_p(par.data_ptr()), c_void_p(coef_t.data_ptr()), k, m, r, g, S,
                   stream)
            assert st == 0, st

        protos.append((os.path.basename(path), run))
    prod()
    torch.cuda.synchronize()
    ref = par.clone()
    for name, run in protos:
        par.zero_()
        run()
        torch.cuda.synchronize()
        same = torch.equal(par, ref)
        print(f"{name}: parities {'==' if same else '!='} product", flush=True)
        if not same and "abl" not in name:
            bad = (par != ref).nonzero()
            print("  first differing byte", int(bad[0]), "of", par.numel(), "count", bad.numel())
            return 1
    del ref
    nbytes = S * (k + m + g) * P
    res = {n: [] for n in ["product"] + [n for n, _ in protos]}
    for _ in range(a.rounds):
        for name, run in [("product", prod)] + protos:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            run()
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(nbytes * a.iters / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    print(f"{a.code}(k={k},r={r},m={m}) {a.stripes} x {a.mib} MiB as {S} units of 8 KiB; encode GB/s median (min..max)")
    for name, v in res.items():
        print(f"  {name:24s} {statistics.median(v):8.1f} ({min(v):7.1f}..{max(v):7.1f})", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

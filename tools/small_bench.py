#!/usr/bin/env python3
"""ECWide-H-sized calls (4 KiB blocks, host memory): per-call ecw_encode vs one
batched ecw_encode_stripes, stripes/s and GB/s of (k + m) * 4 KiB per stripe.
Shape: g_encode's Cauchy (GK=11 data, 3 global parities; ECWide-H/proxy/
encode.cpp:145-175, common.hpp:21-32)."""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=2000)
    ap.add_argument("--k", type=int, default=11)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--len", type=int, default=4096)
    ap.add_argument("--threads", type=int, default=4, help="concurrent ISA-L-shim callers (ECWide-H: 4)")
    a = ap.parse_args()
    import ecwide_amd as E
    from ecwide_amd._lib import lib

    k, m, ln, S = a.k, a.m, a.len, a.stripes
    c = E.NativeCodec.getRsCodec(E.CodingScheme.getRsScheme(k, m, ln))
    rng = np.random.default_rng(1)
    data = [[rng.integers(0, 256, ln, dtype=np.uint8) for _ in range(k)] for _ in range(S)]
    par = [[np.zeros(ln, np.uint8) for _ in range(m)] for _ in range(S)]
    dptr = (ctypes.c_void_p * (S * k))(*[d.ctypes.data for row in data for d in row])
    pptr = (ctypes.c_void_p * (S * m))(*[x.ctypes.data for row in par for x in row])
    assert lib.ecw_encode_stripes(c._h, S, dptr, pptr, ln) == 0  # warm-up (allocations)
    t = time.perf_counter()
    assert lib.ecw_encode_stripes(c._h, S, dptr, pptr, ln) == 0
    tb = time.perf_counter() - t
    n1 = min(S, 200)
    t = time.perf_counter()
    for s in range(n1):
        c.encodeData(data[s], par[s])
    t1 = (time.perf_counter() - t) / n1
    by = (k + m) * ln
    # ISA-L shim (libecw_isal.so) from several threads: group-commit batching
    import threading
    shim = ctypes.CDLL(os.path.join(REPO, "ecwide_amd", "libecw_isal.so"))
    u8p = ctypes.POINTER(ctypes.c_uint8)
    full = np.zeros((k + m) * k, np.uint8)
    shim.gf_gen_cauchy1_matrix(full.ctypes.data_as(u8p), k + m, k)
    tbl = np.zeros(32 * k * m, np.uint8)
    shim.ec_init_tables(k, m, full[k * k:].copy().ctypes.data_as(u8p), tbl.ctypes.data_as(u8p))
    per_t = S // a.threads
    arrs = [((u8p * k)(*[d.ctypes.data_as(u8p) for d in data[s]]), (u8p * m)(*[x.ctypes.data_as(u8p) for x in par[s]]))
            for s in range(S)]

    def run(t):
        for s in range(t * per_t, (t + 1) * per_t):
            shim.ec_encode_data(ln, k, m, tbl.ctypes.data_as(u8p), arrs[s][0], arrs[s][1])

    th = [threading.Thread(target=run, args=(t,)) for t in range(a.threads)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    ts = time.perf_counter() - t0
    n_s = per_t * a.threads
    print(f"ISA-L shim, {a.threads} threads: {n_s / ts:,.0f} stripes/s ({n_s * by / ts / 1e9:.2f} GB/s)")
    print(f"k={k} m={m} len={ln}: batched {S} stripes {tb * 1e3:.2f} ms = {S / tb:,.0f} stripes/s "
          f"({S * by / tb / 1e9:.2f} GB/s); per call {t1 * 1e6:.1f} us = {1 / t1:,.0f} stripes/s "
          f"({by / t1 / 1e9:.3f} GB/s)")


if __name__ == "__main__":
    main()

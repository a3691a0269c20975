#!/usr/bin/env python3
"""Per-call latency of synchronous small encodes (the request service) through
one libecwide.so build, e.g. the phase-traced variant:

  python tools/variants.py svctrace=-DECW_SVC_TRACE=1
  python tools/svc_latency.py build/variants/svctrace.so     # phase means printed at exit

ECWide-H's g_encode shape: ecw_encode on a k=11, m=3 Cauchy matrix codec, 4 KiB."""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import numpy as np

    from ecwide_amd import _lib

    L = _lib.load(sys.argv[1] if len(sys.argv) > 1 else _lib.LIB_PATH, strict=False)
    k, m, ln, n = 11, 3, int(os.environ.get("LEN", 4096)), int(os.environ.get("CALLS", 5000))
    mat = np.array([[1 if i == j else 0 for j in range(k)] for i in range(k)], np.uint8)
    rows = np.zeros((m, k), np.uint8)
    for i in range(m):  # Cauchy rows 1 / ((k + i) ^ j), the g_encode matrix
        for j in range(k):
            x, inv = (k + i) ^ j, 1
            for _ in range(254):  # x^254 = x^-1 in GF(2^8), poly 0x11D
                a, b, p = inv, x, 0
                while b:
                    if b & 1:
                        p ^= a
                    a = ((a << 1) ^ 0x11D) if a & 0x80 else (a << 1)
                    b >>= 1
                inv = p
            rows[i, j] = inv
    del mat
    h = ctypes.c_void_p()
    assert L.ecw_matrix_codec_create(rows.ctypes.data_as(_lib._u8p), k, m, 0, ctypes.byref(h)) == 0
    d = [np.random.default_rng(j).integers(0, 256, ln, dtype=np.uint8) for j in range(k)]
    p = [np.zeros(ln, np.uint8) for _ in range(m)]
    dp = (ctypes.c_void_p * k)(*[x.ctypes.data for x in d])
    pp = (ctypes.c_void_p * m)(*[x.ctypes.data for x in p])
    for _ in range(100):
        assert L.ecw_encode(h, dp, pp, ln) == 0
    nt = int(os.environ.get("THREADS", 1))
    name = os.path.basename(sys.argv[1]) if len(sys.argv) > 1 else "libecwide.so"
    if nt == 1:
        t = time.perf_counter()
        for _ in range(n):
            L.ecw_encode(h, dp, pp, ln)
        el = time.perf_counter() - t
        print(f"{name}: {el / n * 1e6:.2f} us per synchronous k={k} m={m} {ln} B call "
              f"({(k + m) * ln * n / el / 1e9:.2f} GB/s)", flush=True)
        return
    import threading

    def worker():  # each thread its own buffers; ctypes drops the GIL in the call
        d2 = [x.copy() for x in d]
        p2 = [np.zeros(ln, np.uint8) for _ in range(m)]
        a = (ctypes.c_void_p * k)(*[x.ctypes.data for x in d2])
        b = (ctypes.c_void_p * m)(*[x.ctypes.data for x in p2])
        for _ in range(n):
            L.ecw_encode(h, a, b, ln)

    th = [threading.Thread(target=worker) for _ in range(nt)]
    t = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    el = time.perf_counter() - t
    print(f"{name}: {nt} threads x {n} synchronous k={k} m={m} {ln} B calls: "
          f"{(k + m) * ln * n * nt / el / 1e9:.2f} GB/s", flush=True)


if __name__ == "__main__":
    main()

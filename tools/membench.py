#!/usr/bin/env python3
"""HBM ceilings for the stripe access pattern on this GPU.

Measures (GB/s of bytes read + written):
  * torch copy of a large buffer (the float4-copy style ceiling);
  * the XOR-reduce kernel over n rows (n = 1 .. 128) of B bytes with a
    given block stride — how the rate falls with the number of concurrent
    row streams, and whether padding the stride matters.
"""
import argparse
import os
import sys
from ctypes import c_void_p

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def timeit(fn, iters=5):
    import torch

    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--rows", type=int, default=128)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--pads", default="0,4096,73728,1060864")
    ap.add_argument("--ns", default="1,2,4,8,16,27,64,128")
    ap.add_argument("--no-copy", action="store_true")
    a = ap.parse_args()
    import torch

    from ecwide_amd import _lib

    L = _lib.load(a.lib) if a.lib else _lib.lib
    B = a.mib << 20
    stream = c_void_p(torch.cuda.current_stream().cuda_stream)
    big = torch.empty(8 << 30, dtype=torch.uint8, device="cuda")
    dst = torch.empty(8 << 30, dtype=torch.uint8, device="cuda")
    if not a.no_copy:
        t = timeit(lambda: dst.copy_(big))
        print(f"torch copy 8 GiB: {2 * big.numel() / t / 1e9:8.1f} GB/s")
    del dst
    out = torch.empty(B, dtype=torch.uint8, device="cuda")
    for pad in [int(x) for x in a.pads.split(",")]:
        stride = B + pad
        nrows = min(a.rows, (big.numel() - B) // stride + 1)
        base = big.data_ptr()
        line = f"stride B+{pad:>8}: "
        for n in [int(x) for x in a.ns.split(",")]:
            if n > nrows:
                break
            arr = (c_void_p * n)(*[base + i * stride for i in range(n)])

            def run():
                assert L.ecw_xor_reduce_dev(0, arr, n, c_void_p(out.data_ptr()), B, stream) == 0

            t = timeit(run)
            line += f" n={n}:{(n + 1) * B / t / 1e9:7.0f}"
        print(line, flush=True)


if __name__ == "__main__":
    main()

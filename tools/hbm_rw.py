#!/usr/bin/env python3
"""HBM rate for read-only, write-only and copy streams (torch ops, 8 GiB),
to price writes against reads on this GPU."""
import torch


def t(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e-3


n = 8 << 30
x = torch.empty(n, dtype=torch.uint8, device="cuda")
y = torch.empty(n, dtype=torch.uint8, device="cuda")
x.random_()
xi = x.view(torch.int32)
out = torch.empty(1, dtype=torch.int64, device="cuda")
print(f"write-only fill_ : {n / t(lambda: y.fill_(7)) / 1e9:8.1f} GB/s")
print(f"copy (r+w)       : {2 * n / t(lambda: y.copy_(x)) / 1e9:8.1f} GB/s")
print(f"read-only amax   : {n / t(lambda: torch.amax(xi)) / 1e9:8.1f} GB/s")

#!/usr/bin/env python3
"""Raw pinned host <-> HBM copy rates on this box (hipMemcpyAsync through torch):
one stream vs two / four streams issuing slices of the same total, per slice
size -- what the host-resident pipeline's H2D could reach if its copies were
spread over more than one copy queue.

  python tools/h2d_probe.py [--total-mib 2048]
"""
import argparse
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total-mib", type=int, default=2048)
    a = ap.parse_args()
    n = a.total_mib << 20
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    h.random_(0, 256)
    streams = [torch.cuda.Stream() for _ in range(4)]
    for slice_mib in (8, 32, 128):
        sl = slice_mib << 20
        for ns in (1, 2, 4):
            for direction in ("h2d", "d2h", "both"):
                best = 0.0
                for rep in range(3):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for i, o in enumerate(range(0, n, sl)):
                        st = streams[i % ns]
                        with torch.cuda.stream(st):
                            if direction in ("h2d", "both"):
                                d[o:o + sl].copy_(h[o:o + sl], non_blocking=True)
                            if direction in ("d2h", "both"):
                                h2[o:o + sl].copy_(d[o:o + sl], non_blocking=True)
                    torch.cuda.synchronize()
                    dt = time.perf_counter() - t0
                    moved = n * (2 if direction == "both" else 1)
                    best = max(best, moved / dt / 1e9)
                print(f"slice {slice_mib:4d} MiB  streams {ns}  {direction:5s} {best:7.2f} GB/s", flush=True)


if __name__ == "__main__":
    main()

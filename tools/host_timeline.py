#!/usr/bin/env python3
"""One host-resident encodeData + repair of D0 (pinned, NUMA-local; the bench's
host leg) repeated a few times with wall-clock marks, for a
`rocprofv3 --kernel-trace --memory-copy-trace` timeline of the pipeline: where the
time between the copies goes.

  rocprofv3 --kernel-trace --memory-copy-trace -d OUT -o run -- python3 tools/host_timeline.py
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch

    import ecwide_amd as E

    k, m, r, B = 128, 3, 27, 64 << 20
    codec = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    nblk = k + codec.parityNum
    h = E.PinnedHost((nblk + 1) * B, 0)
    v = [h.array[i * B:(i + 1) * B] for i in range(nblk + 1)]
    for j in range(k):
        v[j][:] = (j * 37) & 0xFF
    codec.encodeData(v[:k], v[k:nblk])
    codec.repairBlock(v[:nblk], 0, v[nblk])
    torch.cuda.synchronize()
    for it in range(3):
        t0 = time.perf_counter()
        codec.encodeData(v[:k], v[k:nblk])
        t1 = time.perf_counter()
        codec.repairBlock(v[:nblk], 0, v[nblk])
        t2 = time.perf_counter()
        print(f"iter {it}: encode {1e3 * (t1 - t0):.2f} ms ({nblk * B / (t1 - t0) / 1e9:.1f} GB/s), "
              f"repair {1e3 * (t2 - t1):.2f} ms ({28 * B / (t2 - t1) / 1e9:.1f} GB/s)", flush=True)


if __name__ == "__main__":
    main()

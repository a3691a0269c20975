#!/usr/bin/env python3
"""Which side of the block layout costs the encode its rate: the read layout
(k data rows B apart) or the write layout (m + g parity rows B apart)?

The product's split-layout encode (ecw_encode_batch_split_dev: data and
parities with strides of their own) runs the same CL(128, 27, 3) encode with
every combination of data layout (block rows / tiled 8 KiB pieces) and parity
layout (parity rows inside the block slab / separate parity blocks / compact
per column piece), all carved from ONE allocation and timed in interleaved
rounds (same physical memory). Per-stripe variants make one call per stripe
(each an 8 KiB-piece batch of 16,384 tiles).

  python tools/rw_layout.py [--stripes 8 --mib 64 --rounds 3]
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
    ap.add_argument("--pad", type=int, default=4096)
    ap.add_argument("--ptr-stripes", type=int, default=4, help="stripes of separately allocated blocks (0 = skip)")
    ap.add_argument("--alloc-stripes", type=int, default=4,
                    help="stripes of separately allocated blocks behind pointer tables (0 = skip)")
    ap.add_argument("--offsets", default="", help="comma-separated shifts of the parity region (bytes, 256-multiples)")
    a = ap.parse_args()
    import torch

    from ecwide_amd import _lib

    L = _lib.lib
    k, m, r, S = a.k, a.m, a.r, a.stripes
    B = a.mib << 20
    g = -(-k // r)
    np_ = m + g
    sch = _lib.ecw_scheme()
    assert L.ecw_scheme_init(byref(sch), b"C", k, m, r, B) == 0
    h = c_void_p()
    assert L.ecw_codec_create(byref(sch), 1, 0, 0, 0, byref(h)) == 0
    bs = (B + a.pad + 255) // 256 * 256
    ss = (k + np_) * bs
    slab_bytes = S * ss
    sep_bytes = S * np_ * bs + (64 << 20)  # + room for the --offsets shifts
    buf = torch.empty(slab_bytes + sep_bytes, dtype=torch.uint8, device="cuda")
    base = buf.data_ptr()
    sep = base + slab_bytes
    stream = c_void_p(torch.cuda.current_stream().cuda_stream)
    assert L.ecw_fill_random_dev(0, c_void_p(base), 0, 0, 1, 1, slab_bytes + sep_bytes, 5, 0, 0, stream) == 0
    ch = 8192
    pieces = B // ch
    tiled_par = (S * pieces * k * ch + 4095) // 4096 * 4096

    def split(d, dbs, dss, p, pbs, pss, n, ln):
        st = L.ecw_encode_batch_split_dev(h, c_void_p(d), dbs, dss, c_void_p(p), pbs, pss, n, ln, stream)
        assert st == 0, st

    # pointer mode on separately allocated blocks (caching-allocator placement)
    ptr_sets = []
    if a.ptr_stripes:
        blocks_t = [[torch.empty(B, dtype=torch.uint8, device="cuda") for _ in range(k + np_)]
                    for _ in range(a.ptr_stripes)]
        for bl in blocks_t:
            for t in bl[:k]:
                assert L.ecw_fill_random_dev(0, c_void_p(t.data_ptr()), 0, 0, 1, 1, B, 6, 0, 0, stream) == 0
            ptr_sets.append(((c_void_p * k)(*[t.data_ptr() for t in bl[:k]]),
                             (c_void_p * np_)(*[t.data_ptr() for t in bl[k:]])))

    def ptr_mode():
        for d, p in ptr_sets:
            assert L.ecw_encode_dev(h, d, p, B, stream) == 0

    def tables(dptrs, pptrs):
        """one ecw_encode_ptrs_dev launch over device pointer tables"""
        dt = torch.tensor(dptrs, dtype=torch.int64, device="cuda")
        pt = torch.tensor(pptrs, dtype=torch.int64, device="cuda")
        n = len(dptrs) // k

        def run(dt=dt, pt=pt, n=n):
            assert L.ecw_encode_ptrs_dev(h, n, c_void_p(dt.data_ptr()), c_void_p(pt.data_ptr()), B, stream) == 0
        return run

    # the "parity region after data" blocks, addressed through pointer tables
    P = base + S * k * bs
    tab_split = tables([base + s * k * bs + j * bs for s in range(S) for j in range(k)],
                       [P + s * np_ * bs + i * bs for s in range(S) for i in range(np_)])
    # separately allocated blocks (data of all stripes first, then parities), B or B + pad bytes each
    sep_tabs = {}
    for extra in (0, a.pad):
        if not a.alloc_stripes:
            break
        ts = [torch.empty(B + extra, dtype=torch.uint8, device="cuda") for _ in range(a.alloc_stripes * (k + np_))]
        for t in ts[:a.alloc_stripes * k]:
            assert L.ecw_fill_random_dev(0, c_void_p(t.data_ptr()), 0, 0, 1, 1, B, 7, 0, 0, stream) == 0
        sep_tabs[extra] = (ts, tables([t.data_ptr() for t in ts[:a.alloc_stripes * k]],
                                      [t.data_ptr() for t in ts[a.alloc_stripes * k:]]))

    variants = {
        # data rows B + pad apart, parities inside the slab (ecw_encode_batch_dev)
        "blocks / parity in slab": lambda: split(base, bs, ss, base + k * bs, bs, ss, S, B),
        # data rows as the block slab, parity blocks in a region of their own (pointer mode with
        # separately allocated parity buffers)
        "blocks / separate parity blocks": lambda: split(base, bs, ss, sep, bs, np_ * bs, S, B),
        # data blocks of all stripes, then the parity blocks of all stripes right after them
        "blocks / parity region after data": lambda: split(base, bs, k * bs, base + S * k * bs, bs, np_ * bs, S, B),
        # data rows as the block slab, parities compact per 8 KiB column piece
        "blocks / compact parity pieces": lambda: [
            split(base + s * ss, bs, ch, sep + s * pieces * np_ * ch, ch, np_ * ch, pieces, ch) for s in range(S)],
        # tiled data (a piece's k rows contiguous), parities as separate blocks
        "tiled / separate parity blocks": lambda: [
            split(base + s * pieces * k * ch, ch, k * ch, sep + s * np_ * bs, bs, ch, pieces, ch) for s in range(S)],
        # the tiled slab (bench layout)
        "tiled / compact parity pieces": lambda: split(base, ch, k * ch, base + tiled_par, ch, np_ * ch, S * pieces, ch),
    }
    if ptr_sets:
        variants[f"pointer mode, separate allocations (x{len(ptr_sets)})"] = ptr_mode
    variants["pointer tables over parity-region layout"] = tab_split
    for extra, (_, run) in sep_tabs.items():
        variants[f"pointer tables, separate allocations of B+{extra} (x{a.alloc_stripes})"] = run
    for x in (int(v) for v in a.offsets.split(",") if v):
        # parity region right after the data region, shifted by x bytes
        variants[f"blocks / parity region after data +{x}"] = (
            lambda x=x: split(base, bs, k * bs, base + S * k * bs + x, bs, np_ * bs, S, B))
    res = {n: [] for n in variants}
    for _ in range(a.rounds):
        for name, run in variants.items():
            run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            nst = len(ptr_sets) if name.startswith("pointer mode") else (a.alloc_stripes if "separate alloc" in name
                                                                           else S)
            nbytes = nst * (k + np_) * B
            res[name].append(nbytes * a.iters / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    print(f"CL(k={k},r={r},m={m}) B={B >> 20} MiB x{S} stripes, block pad {a.pad}: encode GB/s median (min..max), "
          f"{a.rounds} interleaved rounds on one allocation")
    for name, v in res.items():
        print(f"  {name:34s} {statistics.median(v):8.1f} ({min(v):7.1f}..{max(v):7.1f})", flush=True)


if __name__ == "__main__":
    main()

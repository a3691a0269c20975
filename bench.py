#!/usr/bin/env python3
"""Device-resident encode + single-block-repair GB/s on wide CL stripes.

One step = encode every stripe of an HBM-resident slab (k data blocks ->
m Cauchy global + g XOR local parities, one kernel launch) and repair data
block D0 of every stripe from its r surviving group members (one launch).
Algorithmic bytes per stripe: encode (k+m+g)*B, repair (r+1)*B (inputs +
outputs, ISA-L's perf_print convention). GB = 1e9.

Multi-GPU (launched by torch.distributed.run): each rank owns its own slab
of `--stripes` stripes (distinct stripe ids), no data moves between GPUs;
torch.distributed is used only for the barrier and the max-over-ranks time.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--layout", choices=["blocks", "tiled"], default="tiled",
                    help="slab layout in HBM (ecwide_amd/slab.py): tiled (default; each --chunk-kib column piece "
                         "of the k data blocks contiguous, parities apart) or whole blocks at a padded stride")
    ap.add_argument("--other-layout-steps", type=int, default=5,
                    help="N=1: also time this many steps on the other layout and report them in the line (0 = off)")
    ap.add_argument("--chunk-kib", type=int, default=8, help="column piece of the tiled layout")
    ap.add_argument("--unit-pad", type=int, default=0, help="tiled layout: padding after each piece run (bytes)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--r", type=int, default=27)
    ap.add_argument("--block-mib", type=float, default=64.0)
    ap.add_argument("--stripes", type=int, default=8, help="stripes per GPU")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline leg (0 = skip)")
    ap.add_argument("--cpu-sample-mib", type=float, default=4.0)
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    ap.add_argument("--verify", action="store_true", help="check one stripe against the oracle after timing")
    ap.add_argument("--hbm-fill", action="store_true",
                    help="BASELINE configs[3]: 256 stripes per GPU, block size = the largest whole MiB "
                         "that fits the GPU's free HBM")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling (BASELINE configs[4]): --stripes (or the --hbm-fill batch) is the "
                         "TOTAL, split by stripe across the ranks")
    ap.add_argument("--pageable", action="store_true",
                    help="with --host-resident: ordinary pageable host blocks instead of pinned ones")
    ap.add_argument("--host-resident", action="store_true",
                    help="measure the PCIe-inclusive rate (pinned host blocks) instead")
    return ap.parse_args()


def dist_setup(args):
    import torch

    from ecwide_amd.shard import dist_env

    world, rank, local = dist_env()
    # one process per GPU; on a box with fewer GPUs than ranks (a rehearsal of
    # the N>1 path) ranks share devices and the timing collective runs on gloo
    ndev = max(1, torch.cuda.device_count())
    dev = local % ndev
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist

        if ndev >= world:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev}"))
        else:
            dist.init_process_group("gloo")
    return world, rank, dev


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def max_over_ranks(world, x: float) -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist

    on_gpu = dist.get_backend() == "nccl"
    t = torch.tensor([x], dtype=torch.float64, device="cuda" if on_gpu else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cpu_baseline(args, k, m, r):
    """The reference's CPU path restated (oracle, test infrastructure): ECWide-C
    encodeData = ec_encode_data with the AVX2 4-bit-split dot products
    (global rows) + one pass per local group, then decodeData of D0 (XOR of
    the r survivors), timed on a bounded column sample of the same stripe."""
    import ctypes

    import numpy as np

    import oracle

    orc = oracle.Oracle()
    B = int(args.cpu_sample_mib * (1 << 20))
    oc = orc.codec("C", k, m, r, B)
    data = [orc.fill(B, args.seed, 0, j) for j in range(k)]
    par = [np.zeros(B, np.uint8) for _ in range(oc.parity_num)]
    u8p = ctypes.POINTER(ctypes.c_uint8)
    dp = (u8p * k)(*[d.ctypes.data_as(u8p) for d in data])
    pp = (u8p * len(par))(*[p.ctypes.data_as(u8p) for p in par])
    g = oc.group_num
    per_stripe = (k + m + g + r + 1) * B

    ones = orc.init_tables(r, 1, np.ones(r, np.uint8))

    def run(threads):
        oc.encode_into(dp, pp, B, literal=False, threads=threads)
        # decodeData: ec_encode_data with the all-ones table (NativeCodec.cc:248)
        return orc.encode_data(ones, data[1:r] + [par[m]], 1, avx2=True)[0]

    from ecwide_amd.shard import host_threads

    t1 = host_threads()
    res = {}
    for threads in sorted({1, t1}):
        run(threads)  # warm
        n, t0 = 0, time.perf_counter()
        while True:
            rep = run(threads)
            n += 1
            el = time.perf_counter() - t0
            if el > args.cpu_seconds / 2 or n >= 50:
                break
        assert np.array_equal(rep, data[0])
        res[threads] = n * per_stripe / el / 1e9
    return {
        "value": round(res[1], 3),
        "unit": "GB/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"1 stripe CL(k={k},r={r},m={m}) column sample B={B >> 20} MiB: ECWide-C encodeData flow "
                   f"(AVX2 nibble-pshufb dot products, global + per-group passes) + XOR repair of D0; "
                   f"single thread = ECWide-C's one ComputeWorker thread"),
        "value_all_cores": round(res[t1], 3),
        "cores_all": t1,
        "host_cpu": platform.processor() or platform.machine(),
        "avx2": orc.have_avx2(),
    }


def host_resident(args):
    """PCIe-inclusive rate: blocks live in pinned host memory; ecw_encode /
    ecw_repair pipeline them through HBM with hipMemcpyAsync in and out.
    Reported separately, never as the bench `value`."""
    import numpy as np
    import torch

    import ecwide_amd as E

    torch.cuda.set_device(0)
    k, m, r = args.k, args.m, args.r
    B = int(args.block_mib * (1 << 20))
    codec = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    nblk = k + codec.parityNum
    hb = torch.empty(nblk * B, dtype=torch.uint8, pin_memory=not args.pageable)
    slab = E.StripeSlab(codec, stripes=1, block_bytes=B)
    slab.fill_random(seed=args.seed)
    for j in range(k):
        hb[j * B:(j + 1) * B].copy_(slab.block(0, j))
    del slab
    torch.cuda.synchronize()
    views = [hb[i * B:(i + 1) * B].numpy() for i in range(nblk)]
    out = torch.empty(B, dtype=torch.uint8, pin_memory=not args.pageable).numpy()
    enc_b = nblk * B
    rep_b = (len(codec.repairSources(0)) + 1) * B
    codec.encodeData(views[:k], views[k:])
    codec.repairBlock(views, 0, out)
    it = max(1, args.steps // 4)
    t0 = time.perf_counter()
    for _ in range(it):
        codec.encodeData(views[:k], views[k:])
    t1 = time.perf_counter()
    for _ in range(it):
        codec.repairBlock(views, 0, out)
    t2 = time.perf_counter()
    assert np.array_equal(out, views[0])
    line = {
        "metric": ("host-resident encode + single-block-repair GB/s "
                   + ("(pageable host blocks, e.g. Java direct ByteBuffers)" if args.pageable
                      else "(pinned host blocks, hipMemcpyAsync in/out)")),
        "value": round(it * (enc_b + rep_b) / (t2 - t0) / 1e9, 2),
        "unit": "GB/s", "n_gpus": 1, "iters": it,
        "encode_GBps": round(it * enc_b / (t1 - t0) / 1e9, 2),
        "repair_GBps": round(it * rep_b / (t2 - t1) / 1e9, 2),
        "pcie_bytes_per_encode": (k + codec.parityNum) * B,
        "config": {"k": k, "r": r, "m": m, "block_bytes": B, "stripes": 1,
                   "pipeline": "8 MiB column slices, 3 HBM slots, H2D/kernel/D2H on 3 streams"},
    }
    print(json.dumps(line), flush=True)


def main():
    args = parse()
    import torch

    if args.host_resident:
        host_resident(args)
        return
    world, rank, local = dist_setup(args)
    import ecwide_amd as E

    k, m, r = args.k, args.m, args.r
    S = args.stripes
    if args.hbm_fill:
        S = 256
        free = torch.cuda.mem_get_info(local)[0]
        g0 = -(-k // r)
        # slab: S * (k+m+g) blocks of B + 4 KiB pad, plus the S-block repair output
        per_mib = S * ((k + m + g0) * ((1 << 20) + 4096) + (1 << 20))
        args.block_mib = float(int(0.97 * free) // per_mib)
        assert args.block_mib >= 1, f"{free} B free: too small for {S} stripes"
    B = int(args.block_mib * (1 << 20))
    from ecwide_amd.shard import column_shard, stripe_shard, weak_shard

    S_total = S if args.strong else S * world
    B_full = B
    columns = args.strong and S_total < world
    if columns:
        # fewer stripes than GPUs (SURVEY §8e fallback): every rank takes its
        # byte columns of every stripe instead
        s0 = 0
        B = column_shard(B_full, world, rank, align=(args.chunk_kib << 10) if args.layout == "tiled" else 4096)[1]
        assert B > 0, "more GPUs than 4 KiB column tiles"
    else:
        # each rank owns distinct stripe ids; no data exchange between ranks
        s0, S = stripe_shard(S_total, world, rank) if args.strong else weak_shard(S, rank)
    scheme = E.CodingScheme.getClScheme(k, m, r, B)
    codec = E.NativeCodec.getClCodec(scheme, 1, False, device=local)
    slab = E.StripeSlab(codec, stripes=S, block_bytes=B, device=local, layout=args.layout,
                        chunk=args.chunk_kib << 10, unit_pad=args.unit_pad)
    out = torch.empty(S * B, dtype=torch.uint8, device=f"cuda:{local}")
    slab.fill_random(seed=args.seed, s0=s0)
    torch.cuda.synchronize()
    enc_bytes = slab.encode_bytes()
    rep_bytes = slab.repair_bytes(0)
    step_bytes = enc_bytes + rep_bytes

    def step(evs=None):
        if evs is not None:
            evs[0].record()
        slab.encode()
        if evs is not None:
            evs[1].record()
        slab.repair(0, out)
        if evs is not None:
            evs[2].record()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # timed region: exactly K steps
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier(world)
    el = time.perf_counter() - t0
    el_max = max_over_ranks(world, el)

    # per-kernel durations with events on the launch stream (separate pass,
    # same work, so the timed region carries no event overhead)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    for i in range(args.steps):
        step(evs[i])
    torch.cuda.synchronize()
    enc_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    rep_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps

    ok = None
    if args.verify and rank == 0 and not columns:
        import numpy as np

        import oracle

        orc = oracle.Oracle()
        if args.layout == "tiled":
            # every (stripe, piece) unit is an independent stripe of `chunk` bytes
            ch = slab.chunk
            oc = orc.codec("C", k, m, r, ch)
            par0 = [p.cpu().numpy() for p in slab.parity(0)]
            ok = True
            for piece in (0, slab.pieces - 1):
                want = oc.encode([orc.fill(ch, args.seed, piece, j) for j in range(k)])
                ok = ok and all(np.array_equal(p[piece * ch:(piece + 1) * ch], w) for p, w in zip(par0, want))
        else:
            oc = orc.codec("C", k, m, r, B)
            data = [orc.fill(B, args.seed, 0, j) for j in range(k)]
            want = oc.encode(data, threads=min(os.cpu_count() or 1, 32))
            ok = all(np.array_equal(p.cpu().numpy(), w) for p, w in zip(slab.parity(0), want))
        ok = ok and torch.equal(out[:B], slab.block(0, 0))

    if rank != 0:
        if world > 1:
            import torch.distributed as dist

            dist.destroy_process_group()
        return

    # every stripe costs the same bytes; in column mode each stripe's bytes are
    # spread over the ranks in proportion to their column slices
    total_bytes = step_bytes * B_full // B // S * S_total * args.steps
    value = total_bytes / el_max / 1e9
    achieved = enc_bytes / (enc_ms * 1e-3) / 1e9
    launches = slab.encode_launches()  # one encode() = `launches` equal kernel launches
    traffic = None
    if os.path.exists(args.pmc):
        try:
            pmc = json.load(open(args.pmc))
            key = f"k{k}_r{r}_m{m}_B{B}_S{S}" + (f"_tiled{args.chunk_kib}k" if args.layout == "tiled" else "")
            ratio = pmc.get(key, {}).get("traffic_over_algorithmic")
            traffic = ratio * enc_bytes / launches if ratio else None  # PMC bytes of one launch
        except Exception:
            traffic = None
    g = codec.groupNum
    line = {
        "metric": "device-resident encode + single-block-repair GB/s, wide stripe (shards in HBM)",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (counter PRNG, uniform random bytes, generated in HBM)",
        "config": {
            "workload": (f"CL(k={k}, r={r}, m={m}, g={g}) B={B >> 20} MiB, {S} stripes/GPU: batched encode + "
                         f"repair of D0") + (f" [strong: {S_total} stripes in total]" if args.strong else "")
            + (f" [column-sliced: {B} of {B_full} B per block on this rank]" if columns else "") + (" [configs[3]: 256 stripes filling HBM, "
                                             f"{slab.buf.numel() / 2**30:.1f} GiB slab]" if args.hbm_fill else ""),
            "k": k, "r": r, "m": m, "g": g, "block_bytes": B_full, "block_bytes_per_gpu": B, "stripes_per_gpu": S, "stripes_total": S_total,
            "parallelism": f"stripe-partitioned x{world} (no collectives on the data path)",
            "layout": ("blocks (each block contiguous, block stride B + 4 KiB)" if args.layout == "blocks" else
                       f"tiled ({args.chunk_kib} KiB column pieces: the k data pieces contiguous, "
                       f"parities in their own region)"),
            "encode_bytes_per_step_per_gpu": enc_bytes,
            "repair_bytes_per_step_per_gpu": rep_bytes,
        },
        "encode_GBps": round(enc_bytes / (enc_ms * 1e-3) / 1e9, 2),
        "repair_GBps": round(rep_bytes / (rep_ms * 1e-3) / 1e9, 2),
        "roofline": {
            "bound": "hbm",
            "kernel": "encode_kernel_asm (ecwide_amd/csrc/ecw_kernels.hip + ecw_encode_asm.hpp)",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            # PMC-measured HBM bytes of one launch over this run's launch time
            "traffic_GBps": round(traffic * launches / (enc_ms * 1e-3) / 1e9, 2) if traffic else None,
            # per kernel launch (rocprof's unit); one encode() of the slab = `launches` launches
            "launch_ms": round(enc_ms / launches, 4),
            "algorithmic_bytes_per_launch": enc_bytes // launches,
            "launches_per_encode": launches,
            "encode_call_ms": round(enc_ms, 4),
            "repair_launch_ms": round(rep_ms, 4),
            "repair_frac": round(rep_bytes / (rep_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        },
        "cpu_baseline": None,
    }
    if ok is not None:
        line["verified"] = bool(ok)
    if world == 1 and args.other_layout_steps > 0 and not args.hbm_fill:
        # the same workload on the other slab layout, for comparison (not `value`)
        other = "blocks" if args.layout == "tiled" else "tiled"
        del slab
        torch.cuda.empty_cache()
        slab2 = E.StripeSlab(codec, stripes=S, block_bytes=B, device=local, layout=other,
                             chunk=args.chunk_kib << 10, unit_pad=args.unit_pad)
        slab2.fill_random(seed=args.seed, s0=s0)
        n2 = args.other_layout_steps
        for _ in range(2):
            slab2.encode()
            slab2.repair(0, out)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n2):
            slab2.encode()
            slab2.repair(0, out)
        torch.cuda.synchronize()
        el2 = time.perf_counter() - t0
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record()
        for _ in range(n2):
            slab2.encode()
        ev[1].record()
        for _ in range(n2):
            slab2.repair(0, out)
        ev[2].record()
        torch.cuda.synchronize()
        line["other_layout"] = {
            "layout": other, "steps": n2,
            "value": round(step_bytes * n2 / el2 / 1e9, 2),
            "encode_GBps": round(enc_bytes * n2 / (ev[0].elapsed_time(ev[1]) * 1e-3) / 1e9, 2),
            "repair_GBps": round(rep_bytes * n2 / (ev[1].elapsed_time(ev[2]) * 1e-3) / 1e9, 2),
        }
        del slab2
        torch.cuda.empty_cache()
    if world == 1 and args.cpu_seconds > 0:
        line["cpu_baseline"] = cpu_baseline(args, k, m, r)
    print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()

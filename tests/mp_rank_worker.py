"""One rank of the 2-rank GPU test (tests/test_gpu_multirank.py), started by
torch.distributed.run: the product's StripeSlab encode + D0 repair on this
rank's share (ecwide_amd.shard.plan_rank) of a batch, written to
<out>/rank<r>.npz for the parent to merge. Each rank also checks its own
share against the oracle (8 KiB column windows at the first and last piece of
its column slice, first and last stripe; every D0 repair against the
generator's bytes) and writes that verdict into the .npz, so two ranks that
computed the same wrong bytes still fail. Ranks may share one GPU (gloo)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    outdir, mode = sys.argv[1], sys.argv[2]
    import torch
    import torch.distributed as dist

    import ecwide_amd as E
    from ecwide_amd.shard import dist_env, plan_rank

    world, rank, local = dist_env()
    torch.cuda.set_device(local % torch.cuda.device_count())
    dist.init_process_group("gloo")
    k, m, r, B, chunk, seed = 32, 3, 11, 4 * 8192, 8192, 61
    total = 5 if mode == "stripes" else 1
    sh = plan_rank(total, B, world, rank, strong=True, align=chunk)
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, sh["block_bytes"]), 1, False)
    slab = E.StripeSlab(c, stripes=sh["stripes"], block_bytes=sh["block_bytes"], layout="tiled", chunk=chunk)
    slab.fill_random(seed=seed, s0=sh["s0"], col_offset=sh["col_offset"])
    slab.encode()
    out = torch.empty(sh["stripes"] * sh["block_bytes"], dtype=torch.uint8, device="cuda")
    slab.repair(0, out)
    torch.cuda.synchronize()
    res = {"s0": sh["s0"], "col_offset": sh["col_offset"], "stripes": sh["stripes"]}
    for s in range(sh["stripes"]):
        res[f"par{s}"] = np.stack([p.cpu().numpy() for p in slab.parity(s)])
        res[f"rep{s}"] = out[s * sh["block_bytes"]:(s + 1) * sh["block_bytes"]].cpu().numpy()
    res.update(oracle_verdict(res, sh, k, m, r, chunk, seed))
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


def oracle_verdict(res, sh, k, m, r, W, seed) -> dict:
    """This rank's share against the oracle (ECWide-C encodeData restated,
    NativeCodec.cc:137-219): windows of W bytes at the first and last piece of
    the column slice of the first and last stripe; D0 repairs against the
    generator's own bytes of block 0."""
    import oracle

    orc = oracle.Oracle()
    oc = orc.codec("C", k, m, r, W)
    n, off0, s0 = sh["block_bytes"], sh["col_offset"], sh["s0"]
    windows, bad = 0, []
    for s in sorted({0, sh["stripes"] - 1}):
        for off in sorted({0, n - W}):
            want = oc.encode([orc.fill(W, seed, s0 + s, j, off0 + off) for j in range(k)])
            for i, w in enumerate(want):
                if not np.array_equal(res[f"par{s}"][i][off:off + W], w):
                    bad.append(f"stripe {s0 + s} parity {i} column {off0 + off}")
            windows += 1
    repairs = 0
    for s in range(sh["stripes"]):
        if not np.array_equal(res[f"rep{s}"], orc.fill(n, seed, s0 + s, 0, off0)):
            bad.append(f"stripe {s0 + s} D0 repair")
        repairs += 1
    return {"oracle_windows": windows, "oracle_repairs": repairs, "oracle_ok": not bad,
            "oracle_failed": "; ".join(bad)}


if __name__ == "__main__":
    main()

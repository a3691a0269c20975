"""One rank of the 2-rank GPU test (tests/test_gpu_multirank.py), started by
torch.distributed.run: the product's StripeSlab encode + D0 repair on this
rank's share (ecwide_amd.shard.plan_rank) of a batch, written to
<out>/rank<r>.npz for the parent to merge. Ranks may share one GPU (gloo)."""
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
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""The N>1 path with the product on the GPU: two torch.distributed.run ranks
(sharing the box's GPU, gloo) each encode and repair their share of a batch
with StripeSlab (tests/mp_rank_worker.py); each rank's share matches the
oracle (its own verdict), and the union of their outputs equals the oracle's
encode of the whole batch and the single-process GPU encode, for stripe
sharding and for the byte-column fallback."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("mode", ["stripes", "columns"])
def test_two_ranks_union_equals_single_process(tmp_path, mode):
    import torch

    import ecwide_amd as E

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(HERE, "mp_rank_worker.py"),
           str(tmp_path), mode]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    k, m, r, B, chunk, seed = 32, 3, 11, 4 * 8192, 8192, 61
    total = 5 if mode == "stripes" else 1
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    slab = E.StripeSlab(c, stripes=total, block_bytes=B, layout="tiled", chunk=chunk)
    slab.fill_random(seed=seed)
    slab.encode()
    torch.cuda.synchronize()
    want = {s: np.stack([p.cpu().numpy() for p in slab.parity(s)]) for s in range(total)}
    import oracle

    orc = oracle.Oracle()
    oc = orc.codec("C", k, m, r, B)  # ECWide-C encodeData restated (NativeCodec.cc:137-219)
    want_orc = {s: np.stack(oc.encode([orc.fill(B, seed, s, j) for j in range(k)])) for s in range(total)}
    for s in range(total):
        assert np.array_equal(want[s], want_orc[s]), ("single-process GPU encode vs oracle", mode, s)
    d0 = {s: slab.block(s, 0).cpu().numpy() for s in range(total)}
    got_par = {s: np.zeros_like(want[s]) for s in range(total)}
    got_rep = {s: np.zeros(B, np.uint8) for s in range(total)}
    covered = {s: np.zeros(B, bool) for s in range(total)}
    for rank in range(2):
        z = np.load(tmp_path / f"rank{rank}.npz")
        s0, off, n = int(z["s0"]), int(z["col_offset"]), int(z["stripes"])
        # the rank's own check of its share against the oracle
        assert bool(z["oracle_ok"]), (mode, rank, str(z["oracle_failed"]))
        assert int(z["oracle_windows"]) >= 1 and int(z["oracle_repairs"]) == n, (mode, rank)
        for i in range(n):
            par, rep = z[f"par{i}"], z[f"rep{i}"]
            w = rep.size
            assert not covered[s0 + i][off:off + w].any(), "a column or stripe owned twice"
            covered[s0 + i][off:off + w] = True
            got_par[s0 + i][:, off:off + w] = par
            got_rep[s0 + i][off:off + w] = rep
    for s in range(total):
        assert covered[s].all(), (mode, s)
        assert np.array_equal(got_par[s], want_orc[s]), (mode, s)
        assert np.array_equal(got_par[s], want[s]), (mode, s)
        assert np.array_equal(got_rep[s], d0[s]), (mode, s)


def test_bench_two_ranks_survive_an_injected_failure():
    """bench.py's fail-safe N > 1 path with the product on the GPU (both ranks on
    the box's one GPU): rank 1 raises in the middle of the configs1 leg, after
    its second collective; every rank leaves that leg at the same collective,
    the line keeps the main leg (verified against the oracle) and every other
    leg, and names the failing rank."""
    import json

    REPO = os.path.dirname(HERE)
    env = {x: v for x, v in os.environ.items() if x not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--block-mib", "4", "--stripes", "2", "--configs4-steps", "0", "--shape-steps", "1",
           "--other-layout-steps", "0", "--host-iters", "1", "--cpu-seconds", "0",
           "--inject-fail", "rank=1,leg=configs1,at=2", "--collective-timeout", "60"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["value"] > 0 and line["verified"] and line["n_gpus"] == 2
    c1 = line["configs1"]
    assert c1["rank"] == 1 and c1["failed_ranks"] == [1] and "before collective 2" in c1["error"]
    assert line["configs0_shape"]["verified"] and line["host_resident"]["verified"]
    assert line["chunk_generator"]["verified"]
    assert line["legs_not_measured"] == ["configs1"]

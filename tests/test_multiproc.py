"""The N>1 path on CPU: world_size-2 gloo ranks split a batch of stripes with
ecwide_amd.shard, each rank encodes its own stripes (oracle on CPU stands in
for the GPU here), and the union of the per-rank results equals the
single-process result — no stripe is lost or duplicated and nothing but
the timing max crosses ranks."""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from ecwide_amd.shard import column_shard, stripe_shard, weak_shard


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, total, q):
    import sys

    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import oracle
    from ecwide_amd.shard import max_over_ranks

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, count = stripe_shard(total, world, rank)
    orc = oracle.Oracle()
    oc = orc.codec("C", 12, 2, 4, 1024)
    out = {}
    for s in range(first, first + count):
        data = [orc.fill(1024, 5, s, j) for j in range(12)]
        par = oc.encode(data)
        out[s] = hashlib.sha256(b"".join(p.tobytes() for p in par)).hexdigest()
    t = max_over_ranks(float(rank + 1))
    dist.barrier()
    q.put((rank, out, t))
    dist.destroy_process_group()


def test_shard_math():
    for total in (0, 1, 7, 256):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                f, c = stripe_shard(total, world, r)
                seen += list(range(f, f + c))
            assert seen == list(range(total))
    assert weak_shard(8, 3) == (24, 8)
    with pytest.raises(ValueError):
        stripe_shard(4, 2, 2)


def test_column_shard_math():
    for B in (0, 1, 4095, 4096, 3 * 4096 + 100, 64 << 20):
        for world in (1, 2, 3, 8):
            cover = []
            for r in range(world):
                off, n = column_shard(B, world, r)
                assert n >= 0 and (n == 0 or off % 4096 == 0)
                if n and off + n < B:
                    assert n % 4096 == 0
                cover += list(range(off, off + n)) if B < 1 << 20 else [off, off + n]
            if B < 1 << 20:
                assert cover == list(range(B))
    assert column_shard(64 << 20, 8, 7) == (56 << 20, 8 << 20)
    with pytest.raises(ValueError):
        column_shard(4096, 2, 2)


def _col_worker(rank, world, port, q):
    import sys

    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B = 3 * 4096 + 100
    off, n = column_shard(B, world, rank)
    orc = oracle.Oracle()
    oc = orc.codec("C", 12, 2, 4, n)
    data = [orc.fill(B, 9, 0, j)[off:off + n].copy() for j in range(12)]
    q.put((rank, off, [p.tobytes() for p in oc.encode(data)]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_column_slices():
    """One stripe, two ranks: each encodes its byte columns; the slices
    concatenate to the single-process encode (SURVEY §8e fallback)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_col_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    import oracle

    orc = oracle.Oracle()
    B = 3 * 4096 + 100
    want = orc.codec("C", 12, 2, 4, B).encode([orc.fill(B, 9, 0, j) for j in range(12)])
    for i, w in enumerate(want):
        assert b"".join(parts[i] for _, _, parts in res) == w.tobytes()


def test_two_rank_gloo_partition():
    world, total = 2, 5
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    merged = {}
    for rank, out, t in res:
        assert t == float(world)  # max over ranks
        assert not set(out) & set(merged)
        merged.update(out)
    assert sorted(merged) == list(range(total))
    import oracle

    orc = oracle.Oracle()
    oc = orc.codec("C", 12, 2, 4, 1024)
    for s in range(total):
        par = oc.encode([orc.fill(1024, 5, s, j) for j in range(12)])
        assert merged[s] == hashlib.sha256(b"".join(p.tobytes() for p in par)).hexdigest()


# ---- bench.py's own rank orchestration (no GPU: --dry-run) -------------------
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env=None):
    import json
    import subprocess
    import sys

    e = {x: v for x, v in os.environ.items() if x not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, env=e)
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) <= 1, p.stdout[-2000:]  # rank 0 prints exactly one JSON line, whatever happened
    return p, (json.loads(lines[0]) if lines else None)


def test_bench_gpus2_launches_two_ranks_weak_default_and_configs4_leg():
    """`bench.py --gpus 2` (no torch.distributed.run around it) starts 2 ranks
    itself. Its main leg is the N=1 workload on EVERY rank (8 stripes of 64 MiB
    per GPU, weak scaling; distinct stripe ids per rank); the configs[4] leg
    splits the 256-stripe HBM-filling batch (B sized so the whole batch fits
    one GPU, the same B on every rank) by stripe; the reported time is the
    max over ranks."""
    p, line = _bench("--gpus", "2", "--dry-run", "--dry-run-free-gib", "287")
    assert p.returncode == 0, p.stderr[-2000:]
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and not line["hbm_fill"]
    assert line["stripes_total"] == 16 and line["block_bytes"] == 64 << 20
    assert [(x["s0"], x["stripes"]) for x in line["shares"]] == [(0, 8), (8, 8)]
    c4 = line["configs4"]
    assert c4["stripes_total"] == 256 and c4["block_bytes"] == 8 << 20
    assert [(x["s0"], x["stripes"]) for x in c4["shares"]] == [(0, 128), (128, 128)]
    assert line["el_max"] == max(line["rank_seconds"]) and len(line["rank_seconds"]) == 2


def test_bench_config_same_at_every_n():
    """SCALE's N=1 point is BENCH: the N=1 and N>1 lines carry the same
    `config` apart from stripes_total (n_gpus is top-level)."""
    lines = {}
    for n in (1, 2, 4, 8):
        p, line = _bench("--gpus", str(n), "--dry-run")
        assert p.returncode == 0, p.stderr[-2000:]
        lines[n] = line
    base = dict(lines[1]["config"])
    assert base["stripes_total"] == 8 and base["stripes_per_gpu"] == 8 and base["k"] == 128
    assert base["block_bytes"] == 64 << 20 and "per GPU" in base["workload"]
    for n in (2, 4, 8):
        c = dict(lines[n]["config"])
        assert c.pop("stripes_total") == 8 * n
        assert c == {x: v for x, v in base.items() if x != "stripes_total"}
        assert lines[n]["n_gpus"] == n and lines[n]["scaling"] == "weak"
        assert [x["s0"] for x in lines[n]["shares"]] == [8 * r for r in range(n)]
        c4 = lines[n]["configs4"]  # the 256-stripe batch, split by stripe at every N
        assert c4["stripes_total"] == 256 and sum(x["stripes"] for x in c4["shares"]) == 256


def test_bench_dry_run_n8_per_rank_fields():
    """the driver's first 8-GPU run. Every per-rank field
    has 8 entries, the configs[4] split gives each GPU 32 of the 256 stripes,
    and the k=32 shape legs keep their per-GPU stripe counts (weak)."""
    p, line = _bench("--gpus", "8", "--dry-run")
    assert p.returncode == 0, p.stderr[-2000:]
    assert line["n_gpus"] == 8 and len(line["rank_ms_per_step"]) == 8
    assert len(line["roofline"]["rank_launch_ms"]) == 8
    c4 = line["configs4"]
    assert c4["stripes_per_gpu"] == 32 and len(c4["rank_ms_per_step"]) == 8
    assert [x["stripes"] for x in c4["shares"]] == [32] * 8
    assert line["configs1"]["stripes_per_gpu"] == 32 and line["configs1"]["stripes_total"] == 256
    assert line["configs1"]["block_bytes"] == 16 << 20
    assert line["configs0_shape"]["stripes_per_gpu"] == 8 and line["configs0_shape"]["block_bytes"] == 64 << 20
    assert len(line["configs0_shape"]["rank_ms_per_step"]) == 8
    # the host-resident leg runs on every rank, its own pinned stripe each
    h = line["host_resident"]
    for key in ("rank_GBps", "rank_h2d_GBps", "rank_numa_node", "rank_gpu_numa_node"):
        assert len(h[key]) == 8, key


def test_bench_dry_run_strong_and_column_modes():
    p, line = _bench("--gpus", "2", "--dry-run", "--strong", "--stripes", "6")
    assert p.returncode == 0, p.stderr[-2000:]
    assert line["scaling"] == "strong" and line["stripes_total"] == 6
    assert [(x["s0"], x["stripes"]) for x in line["shares"]] == [(0, 3), (3, 3)]
    # fewer stripes than ranks: byte columns of every stripe, aligned to the tiled piece
    p, line = _bench("--gpus", "3", "--dry-run", "--strong", "--stripes", "1")
    assert p.returncode == 0, p.stderr[-2000:]
    sh = line["shares"]
    assert sh[0]["col_offset"] == 0 and all(x["col_offset"] % 8192 == 0 for x in sh)
    assert sum(x["block_bytes"] for x in sh) == 64 << 20
    for a, b in zip(sh, sh[1:]):
        assert a["col_offset"] + a["block_bytes"] == b["col_offset"]
    # --hbm-fill: the configs[3] batch is the main leg, split by stripe
    p, line = _bench("--gpus", "2", "--dry-run", "--hbm-fill")
    assert p.returncode == 0, p.stderr[-2000:]
    assert line["hbm_fill"] and line["scaling"] == "strong" and line["stripes_total"] == 256
    assert line.get("configs4") is None


def test_bench_rejects_world_size_mismatch():
    p, _ = _bench("--gpus", "2", "--dry-run", env={"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=3" in p.stderr


def test_plan_rank_and_hbm_fill_sizing():
    from ecwide_amd.shard import hbm_fill_block_mib, plan_rank

    # 288 GiB HBM, k=128 + 8 parities, 256 stripes: 8 MiB blocks (272 GiB slab)
    assert hbm_fill_block_mib(287 << 30, 128, 8, 256) == 8
    assert hbm_fill_block_mib(1 << 30, 128, 8, 256) == 0
    for world in (1, 2, 4, 8):
        got = [plan_rank(256, 8 << 20, world, r, strong=True) for r in range(world)]
        assert sum(g["stripes"] for g in got) == 256 and all(not g["columns"] for g in got)
        assert [g["s0"] for g in got] == [256 // world * r for r in range(world)]
    w = plan_rank(8, 1 << 26, 4, 3, strong=False, per_rank=8)
    assert (w["s0"], w["stripes"]) == (24, 8)


# ---- the fail-safe N>1 path: one JSON line whatever a rank does
def _main_intact(line, n):
    assert line["n_gpus"] == n and line["stripes_total"] == 8 * n and len(line["rank_seconds"]) == n
    assert [x["s0"] for x in line["shares"]] == [8 * r for r in range(n)]


@pytest.mark.parametrize("n,rank", [(8, 3), (2, 1)])
def test_bench_injected_failure_in_host_leg(n, rank):
    """A rank raising in the host-resident leg: every rank leaves that leg at
    the same collective, the line carries host_resident.error with the rank,
    the main leg and the other legs are intact, nobody hangs, rc 0."""
    p, line = _bench("--gpus", str(n), "--dry-run", "--dry-run-fail", f"rank={rank},leg=host")
    assert p.returncode == 0, p.stderr[-2000:]
    _main_intact(line, n)
    h = line["host_resident"]
    assert h["rank"] == rank and h["failed_ranks"] == [rank] and "InjectedFailure" in h["error"]
    assert line["legs_not_measured"] == ["host_resident"]
    assert len(line["configs4"]["shares"]) == n and line["configs1"]["stripes_per_gpu"] == 32
    assert line["chunk_generator"] == {"dry_run": True}  # rank 0's own leg after it still ran


@pytest.mark.parametrize("n,rank,leg,at", [(8, 5, "configs4", 2), (2, 0, "configs1", 1), (2, 1, "main", 3)])
def test_bench_injected_failure_mid_leg(n, rank, leg, at):
    """The failing rank has passed some of the leg's collectives (at = the
    collective it fails before) while the others wait in the next one: its
    fail-sync stands in for that collective; the next leg runs normally."""
    p, line = _bench("--gpus", str(n), "--dry-run", "--dry-run-fail", f"rank={rank},leg={leg},at={at}")
    err = line["main_error"] if leg == "main" else line[leg]
    assert err["rank"] == rank and f"before collective {at}" in err["error"]
    assert line["legs_not_measured"] == [leg]
    if leg == "main":
        assert p.returncode == 1 and line["value"] is None  # no headline: a failed run
        assert line["configs4"]["stripes_total"] == 256
    else:
        assert p.returncode == 0, p.stderr[-2000:]
        _main_intact(line, n)
        assert "stripes_total" in line["configs0_shape"] and "rank_GBps" in line["host_resident"]


def test_bench_hung_rank_times_out_and_line_survives():
    """A rank hanging inside a leg (as inside a GPU call): the others' leg
    collective times out (--collective-timeout), they skip the later
    collective legs, rank 0 prints the line; the hung rank exits soon after
    the line is out (not at its deadline), so the launcher returns."""
    import time

    t0 = time.time()
    p, line = _bench("--gpus", "2", "--dry-run", "--dry-run-fail", "rank=1,leg=configs1,at=1,mode=hang",
                     "--collective-timeout", "4", "--deadline-s", "200")
    assert time.time() - t0 < 60
    assert p.returncode == 0, p.stderr[-2000:]
    _main_intact(line, 2)
    assert "collective failed in leg configs1" in line["configs1"]["error"]
    for leg in ("configs0_shape", "host_resident"):
        assert "no collectives after an earlier failure" in line[leg]["skipped"]
    assert line["legs_not_measured"] == ["configs1", "configs0_shape", "host_resident"]
    assert "configs4" in line and "error" not in line["configs4"]
    assert "after rank 0 printed the line: exiting" in p.stderr


def test_bench_hung_rank0_prints_from_watchdog():
    """Rank 0 itself stuck in a leg: the other rank's collective times out and
    leaves an abort marker; rank 0's watchdog prints the line it has (the
    main leg) --collective-timeout + 30 s later, well before the deadline."""
    import time

    t0 = time.time()
    p, line = _bench("--gpus", "2", "--dry-run", "--dry-run-fail", "rank=0,leg=configs0_shape,at=1,mode=hang",
                     "--collective-timeout", "4", "--deadline-s", "200")
    assert time.time() - t0 < 90
    assert p.returncode == 0, p.stderr[-2000:]
    _main_intact(line, 2)
    assert "rank 0 stuck in leg configs0_shape" in line["error"]
    assert "configs0_shape" in line["legs_not_measured"] and "stripes_per_gpu" in line["configs1"]


def test_bench_rank_exit_still_prints_line():
    """A rank dying (segfault-like exit): torch.distributed.run SIGTERMs the
    others; rank 0's watchdog prints what it has, naming the leg it was in."""
    p, line = _bench("--gpus", "2", "--dry-run", "--dry-run-fail", "rank=1,leg=configs4,at=1,mode=exit",
                     "--collective-timeout", "20")
    assert line is not None, p.stderr[-2000:]
    _main_intact(line, 2)
    assert "SIGTERM" in line["error"] and ("in leg configs4" in line["error"] or "(between legs)" in line["error"])
    # every leg after the cut is listed, the one in flight included
    assert {"configs4", "configs1", "configs0_shape", "host_resident", "chunk_generator"} <= set(
        line["legs_not_measured"])


def test_bench_time_budget_drops_optional_legs():
    """--budget-s: a leg starts only if elapsed (max over ranks) + its
    estimate fits; the decision is the same on every rank."""
    p, line = _bench("--gpus", "2", "--dry-run", "--budget-s", "30")
    assert p.returncode == 0, p.stderr[-2000:]
    _main_intact(line, 2)
    assert "time budget" in line["configs4"]["skipped"]  # 40 s estimate
    assert "stripes_per_gpu" in line["configs1"]         # 12 s estimate fits
    assert "configs4" in line["legs_not_measured"]


def test_bench_n8_estimate_within_budget():
    """The driver's 8-GPU run: every leg's estimate plus startup fits the
    default budget, which sits below the hard deadline."""
    p, line = _bench("--gpus", "8", "--dry-run")
    assert p.returncode == 0, p.stderr[-2000:]
    b = line["budget"]
    assert b["estimated_total_s"] < b["budget_s"] < b["deadline_s"] <= 540
    assert set(b["estimate_s"]) == {"configs4", "configs1", "configs0_shape", "host_resident", "chunk_generator"}
    assert line["legs_not_measured"] == []


def test_bench_launches_on_one_port_do_not_share_markers():
    """The driver runs N = 1, 2, 4, 8 back to back, possibly on one master
    port: a later launch must not read an earlier launch's "printed" marker
    (its ranks would take it as rank 0 having printed and exit)."""
    import json
    import subprocess
    import sys
    import time

    port = _free_port()
    e = {x: v for x, v in os.environ.items() if x not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", f"--master-port={port}", os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run",
           "--dry-run-slow", "20"]  # a run of several seconds: the watchdog polls every second
    lines = []
    for i in range(2):
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=e)
        assert p.returncode == 0, p.stderr[-2000:]
        lines.append(json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][0]))
        if i == 0:
            time.sleep(17)  # older than Line.GRACE_AFTER_PRINT_S
    assert lines[1]["legs_not_measured"] == [] and "rank_GBps" in lines[1]["host_resident"]


def test_bench_sigterm_at_n1_prints_the_line():
    """A launcher's SIGTERM (or a driver's own time limit) in the middle of a
    run: the watchdog prints the line it has, with the leg it was in, once."""
    import json
    import signal
    import subprocess
    import sys
    import time

    e = {x: v for x, v in os.environ.items() if x not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.Popen([sys.executable, os.path.join(REPO, "bench.py"), "--dry-run", "--dry-run-slow", "200"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=e)
    time.sleep(15)  # the stand-in main leg takes 10 s at this scale, configs4 4 s more
    p.send_signal(signal.SIGTERM)
    out, err = p.communicate(timeout=60)
    lines = [x for x in out.splitlines() if x.startswith("{")]
    assert len(lines) == 1, (out[-2000:], err[-2000:])
    line = json.loads(lines[0])
    assert line["error"].startswith("terminated (SIGTERM) in leg") and line["n_gpus"] == 1
    assert line["dry_run"] and "in leg main" not in line["error"]  # the main leg finished before the signal
    assert p.returncode == 0  # the main leg (a dry run here) is in the line


def test_bench_sigterm_inside_main_leg_fails_the_run():
    """Cut off inside the main leg: one line that still names the metric, no
    value, exit code 1."""
    import json
    import signal
    import subprocess
    import sys
    import time

    e = {x: v for x, v in os.environ.items() if x not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.Popen([sys.executable, os.path.join(REPO, "bench.py"), "--dry-run", "--dry-run-slow", "400"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=e)
    time.sleep(8)
    p.send_signal(signal.SIGTERM)
    out, err = p.communicate(timeout=60)
    lines = [x for x in out.splitlines() if x.startswith("{")]
    assert len(lines) == 1, (out[-2000:], err[-2000:])
    line = json.loads(lines[0])
    assert line["metric"] and line["value"] is None and "in leg main" in line["error"]
    assert line["legs_not_measured"][0] == "main" and p.returncode == 1

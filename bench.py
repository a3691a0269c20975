#!/usr/bin/env python3
"""Device-resident encode + single-block-repair GB/s on wide CL stripes.

One step = encode every stripe of an HBM-resident slab (k data blocks ->
m Cauchy global + g XOR local parities, one kernel launch) and repair data
block D0 of every stripe from its r surviving group members (one launch).
Algorithmic bytes per stripe: encode (k+m+g)*B, repair (r+1)*B (inputs +
outputs, ISA-L's perf_print convention). GB = 1e9.

Workloads (BASELINE.json configs):
  * `value`, at every N — the metric's point, configs[2]'s shape: CL(k=128,
    r=27, m=3), 64 MiB blocks, 8 stripes PER GPU ("scaling": "weak"), so
    the N=1 line (= BENCH) and every N>1 line of the 1/2/4/8 curve measure
    the same per-GPU workload; stripe 0 is the stripe the committed
    full-size digests pin (seed 103, tests/golden/manifest.json).
  * `configs4`, a second timed leg in the same line: the configs[3] batch
    (256 stripes, block size sized so the whole batch fills ONE GPU's HBM,
    the same B at every N) split by stripe over the N GPUs ("strong"; at
    N=1 it is configs[3] itself).
  * `other_layout` (N=1): the same workload in the reference's block
    layouts (split slab, pointer tables over separately allocated blocks),
    interleaved round by round with the tiled slab in one process.
  * `host_resident` (rank 0): the PCIe-inclusive rate (pinned host blocks,
    hipMemcpyAsync in and out) and the ChunkGenerator replay timed around
    encodeChunks as ChunkGenerator.java:126-131 times it.
  `--hbm-fill` makes configs[3] the main leg, `--strong` splits --stripes.

Multi-GPU: `python bench.py --gpus N` starts N rank processes itself
(torch.distributed.run in a child process, before any GPU call in this one)
unless it already runs under torch.distributed.run. One process per GPU; each
rank owns its stripes in its own HBM, no data moves between GPUs;
torch.distributed (gloo: there is no data exchange to put on RCCL) only lines
ranks up (barrier) and takes the max of the per-rank times.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

T_START = time.time()  # the process's start: the time budget and the hard deadline count from here

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md
HBM_FILL_STRIPES = 256  # BASELINE configs[3]
DEFAULT_SEED = 103      # = manifest "cfg3_full": the bench's stripe 0 is the digest-pinned stripe


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without a torch.distributed.run environment bench.py launches them")
    ap.add_argument("--layout", choices=["blocks", "split", "tiled"], default="tiled",
                    help="slab layout in HBM (ecwide_amd/slab.py): tiled (default; each --chunk-kib column piece "
                         "of the k data blocks contiguous, parities apart), split (whole blocks, parity blocks in "
                         "a region of their own) or blocks (whole blocks, [D.., G.., L..] per stripe)")
    ap.add_argument("--other-layout-steps", type=int, default=2,
                    help="N=1: encode + repair steps per layout and round in the whole-block legs (split slab, "
                         "pointer tables), interleaved with the tiled slab (0 = off)")
    ap.add_argument("--other-layout-rounds", type=int, default=4, help="rounds of the interleaved layout legs")
    ap.add_argument("--configs4-steps", type=int, default=5,
                    help="timed steps of the configs[3]/[4] HBM-filling leg reported as `configs4` (0 = off)")
    ap.add_argument("--shape-steps", type=int, default=5,
                    help="timed steps of each other single-GPU BASELINE shape (configs1, configs0_shape; 0 = off)")
    ap.add_argument("--host-iters", type=int, default=2,
                    help="rank 0: encodes + repairs of the PCIe-inclusive host-resident leg (0 = off)")
    ap.add_argument("--chunk-kib", type=int, default=None,
                    help="column piece of the tiled layout (default: ecwide_amd.slab.default_chunk(k), 8 KiB at "
                         "k=128, 16 KiB at k<=32)")
    ap.add_argument("--unit-pad", type=int, default=0, help="tiled layout: padding after each piece run (bytes)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--r", type=int, default=27)
    ap.add_argument("--block-mib", type=float, default=None, help="block size (default 64; --hbm-fill: from free HBM)")
    ap.add_argument("--stripes", type=int, default=None, help="stripes per GPU (weak) or in total (--strong); default 8")
    ap.add_argument("--seed", type=int, default=DEFAULT_SEED)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline leg (0 = skip)")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    ap.add_argument("--no-verify", dest="verify", action="store_false",
                    help="skip the parity check after timing (default: every rank checks sampled column pieces "
                         "of its first/middle/last stripe against the oracle and every stripe's D0 repair; at the "
                         "default shape stripe 0 is also checked against the committed full-size digests)")
    ap.add_argument("--verify", dest="verify", action="store_true")
    ap.add_argument("--hbm-fill", action="store_true",
                    help="main leg = BASELINE configs[3]: 256 stripes, block size = the largest whole MiB at which "
                         "the batch fits one GPU's free HBM (split by stripe over the ranks at N>1)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: --stripes is the TOTAL, split by stripe (default: per GPU)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: plan every rank's share and run the rank orchestration and timing reduction "
                         "only (CPU test of the N>1 path; --dry-run-free-gib stands in for free HBM)")
    ap.add_argument("--dry-run-free-gib", type=float, default=287.0)
    ap.add_argument("--dry-run-slow", type=float, default=1.0,
                    help="--dry-run: scale the stand-in legs' sleeps (a longer run for the orchestration tests)")
    ap.add_argument("--inject-fail", "--dry-run-fail", dest="inject_fail", default=None,
                    help="rank=R,leg=NAME[,at=I][,mode=raise|hang|exit]: make rank R fail in leg NAME (at its start, "
                         "or just before the leg's I-th collective) -- the test of the fail-safe N>1 path")
    ap.add_argument("--budget-s", type=float, default=450.0,
                    help="time budget: an optional leg starts only if the elapsed time (max over ranks, from "
                         "process start) plus its estimate fits (leg_estimates)")
    ap.add_argument("--deadline-s", type=float, default=540.0,
                    help="hard deadline after process start: rank 0 prints the line with what it has, every rank "
                         "exits (a rank stuck in a GPU call included)")
    ap.add_argument("--collective-timeout", type=float, default=120.0,
                    help="seconds a leg collective waits for the other ranks before the group counts as broken")
    ap.add_argument("--profile-csv", default=os.path.join(REPO, "profiles", "r06fin_bench_kernel_stats.csv"),
                    help="committed rocprofv3 --stats kernel summary of this workload on this kernel build: the "
                         "line's roofline.profile_frac / profile_repair_frac are recomputed from it")
    ap.add_argument("--pageable", action="store_true",
                    help="with --host-resident: ordinary pageable host blocks instead of pinned ones")
    ap.add_argument("--host-resident", action="store_true",
                    help="measure the PCIe-inclusive rate (pinned host blocks) instead")
    ap.add_argument("--small-calls", action="store_true",
                    help="measure ECWide-H's synchronous one-chunk ec_encode_data calls (k=11, m=3) instead")
    ap.add_argument("--small-len", type=int, default=4096)
    ap.add_argument("--small-calls-n", type=int, default=5000, help="calls per thread")
    return ap.parse_args(argv)


# ---- rank orchestration ------------------------------------------------------
def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv: list) -> int:
    """Start n ranks of this script under torch.distributed.run in a child
    process (never exec: this process has not touched the GPU and stays the
    parent) and return its exit code; rank 0 prints the JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


class LegAborted(Exception):
    """Another rank failed in the current leg: every rank leaves it at the same
    collective (the one the failing rank's fail-sync matched)."""


class GroupBroken(Exception):
    """A collective timed out or lost a peer (a rank hung or died): no further
    collective can run in this process."""


class InjectedFailure(RuntimeError):
    """--inject-fail: a deliberate failure on one rank (CPU tests of the N>1
    path and the one-GPU rehearsal)."""


def parse_inject(spec: str | None) -> dict | None:
    """`rank=R,leg=NAME[,at=I][,mode=raise|hang|exit]`: rank R fails in leg NAME
    at its start (at=0) or just before the leg's I-th collective."""
    if not spec:
        return None
    kv = dict(x.split("=", 1) for x in spec.split(",") if x)
    leg = {"host": "host_resident", "chunkgen": "chunk_generator", "cpu": "cpu_baseline"}.get(kv["leg"], kv["leg"])
    mode = kv.get("mode", "raise")
    if mode not in ("raise", "hang", "exit") or leg not in LEG_NAMES:
        raise SystemExit(f"bench.py: bad --inject-fail {spec!r} (legs: {', '.join(LEG_NAMES)})")
    return {"rank": int(kv["rank"]), "leg": leg, "at": int(kv.get("at", 0)), "mode": mode}


class Dist:
    """World/rank/device of this process and the bench's one collective.

    Every barrier, max, min and gather is `_sync`: ONE all-reduce (sum) of a
    fixed-shape vector [failures, x of rank 0 .. N-1] on a gloo group with a
    short timeout. Because every collective has the same shape, a rank that
    fails inside a leg makes a single fail-sync that stands in for whichever
    collective the other ranks wait in; they see failures > 0 there and leave
    the leg together (LegAborted), so an exception on one rank never strands
    the others in a barrier. A rank that hangs or dies turns into a timeout /
    closed connection on the others (GroupBroken): they skip every later leg
    and rank 0 still prints the line (run_leg, Line)."""

    def __init__(self, args):
        from ecwide_amd.shard import dist_env

        self.world, self.rank, self.local = dist_env()
        if self.world != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={self.world}")
        self.dry = args.dry_run
        self.inject = parse_inject(args.inject_fail)
        self.budget = args.budget_s
        self.leg, self.leg_sync, self.broken = None, 0, None
        self.leg_seconds = {}
        self.dev, self.ndev, self.backend, self.pg = None, 0, None, None
        self.run_tag = None
        if not self.dry:
            import torch

            self.ndev = torch.cuda.device_count()
            if self.ndev < 1:
                raise SystemExit("bench.py: no GPU visible (use --dry-run for the CPU rehearsal)")
            # one process per GPU; on a box with fewer GPUs than ranks (a
            # rehearsal of the N>1 path) ranks share devices over gloo
            self.dev = self.local % self.ndev
            torch.cuda.set_device(self.dev)
        self.distinct = self.dry or self.ndev >= self.world  # refined below from the ranks' PCI ids
        if self.world > 1:
            import datetime

            import torch
            import torch.distributed as dist

            # no stripe byte moves between ranks: the only collectives are the
            # barriers around the timed regions and a few scalars (max time, min
            # block size, verification), so they run on gloo over loopback --
            # the same on one GPU or eight, and no RCCL communicator is set up.
            # The rendezvous may wait for a slow first `import torch` on a fresh
            # box; the legs' collectives get a group with a short timeout.
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=max(600.0, args.collective_timeout)))
            self.pg = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=args.collective_timeout))
            self.backend = dist.get_backend()
            # this launch's marker-file tag (Line._watch): rank 0's pid and start time,
            # so a later launch on the same host and port never sees this one's files
            pid0, t0 = self._sync(float(os.getpid()))[0], self._sync(T_START)[0]
            self.run_tag = f"{int(pid0)}_{int(t0 * 1000)}"
            if not self.dry:
                # one process per GPU: which physical GPU each rank drives (PCI
                # domain / bus / device), so the line is right whether every rank
                # sees all GPUs or only its own (per-rank visibility)
                pr = torch.cuda.get_device_properties(self.dev)
                key = float(getattr(pr, "pci_domain_id", 0) * 65536 + getattr(pr, "pci_bus_id", 0) * 256
                            + getattr(pr, "pci_device_id", 0)) if hasattr(pr, "pci_bus_id") else None
                if key is not None:
                    phys = self.gather(key)
                    self.distinct = len(set(phys)) == self.world
                    if self.ndev >= self.world and not self.distinct:
                        raise SystemExit(f"bench.py: ranks share GPUs {phys} although {self.ndev} are visible")
                if not self.distinct and self.rank == 0:
                    print(f"bench.py: rehearsal: {self.world} ranks share GPUs ({self.ndev} visible per rank)",
                          file=sys.stderr)

    # -- the one collective ----------------------------------------------------
    def _inject_here(self):
        """--inject-fail: act if this rank, leg and collective index match."""
        j = self.inject
        if not j or j["rank"] != self.rank or j["leg"] != self.leg or j["at"] != self.leg_sync:
            return
        self.inject = None  # once
        where = f"rank {self.rank}, leg {self.leg}, before collective {self.leg_sync}"
        if j["mode"] == "exit":
            print(f"bench.py: injected exit ({where})", file=sys.stderr, flush=True)
            os._exit(3)
        if j["mode"] == "hang":
            print(f"bench.py: injected hang ({where})", file=sys.stderr, flush=True)
            while True:
                time.sleep(3600)
        raise InjectedFailure(f"injected failure ({where})")

    def _sync(self, x: float = 0.0, fail: bool = False) -> list:
        """All-reduce (sum) of [failures, x on this rank's slot]; returns x of
        every rank in rank order. Raises LegAborted when another rank reported
        a failure, GroupBroken when the collective itself failed."""
        if self.leg is not None:
            if not fail:
                self.leg_sync += 1
                self._inject_here()
        if self.world == 1:
            return [x]
        if self.broken:
            raise GroupBroken(self.broken)
        import torch
        import torch.distributed as dist

        t = torch.zeros(1 + self.world, dtype=torch.float64)
        t[0] = 1.0 if fail else 0.0
        t[1 + self.rank] = x
        try:
            dist.all_reduce(t, group=self.pg)
        except Exception as e:  # timeout (a rank hung) or closed connection (a rank died)
            self.broken = f"collective failed in leg {self.leg}: {type(e).__name__}: {str(e)[:240]}"
            self.touch("abort")  # tells a rank 0 stuck in a GPU call to print (Line._watch)
            raise GroupBroken(self.broken) from None
        if t[0] > 0 and not fail:
            raise LegAborted(int(t[0].item()))
        return [float(a) for a in t[1:].tolist()]

    def barrier(self):
        self._sync()

    def reduce(self, x: float, op: str) -> float:
        v = self._sync(x)
        return {"max": max, "min": min}[op](v)

    def gather(self, x: float) -> list:
        """x of every rank, in rank order."""
        return self._sync(x)

    def _gather_objects(self, obj) -> list:
        if self.world == 1:
            return [obj]
        import torch.distributed as dist

        out = [None] * self.world
        try:
            dist.all_gather_object(out, obj, group=self.pg)
        except Exception as e:
            self.broken = f"collective failed after leg {self.leg}: {type(e).__name__}: {str(e)[:240]}"
            self.touch("abort")
            raise GroupBroken(self.broken) from None
        return out

    # -- legs ------------------------------------------------------------------
    def elapsed_max(self) -> float:
        """Seconds since the slowest rank's process started (one sync)."""
        return self.reduce(time.time() - T_START, "max")

    def run_leg(self, name: str, fn, est_s: float = 0.0, local: bool = False):
        """Run leg `fn` (same collectives on every rank) and return (result,
        None), or (None, {"error" | "skipped": ...}) on EVERY rank when any
        rank failed, the group broke or the time budget rules the leg out --
        never raises. The leg ends with one agreement sync, so a rank's
        fail-sync is always matched inside the leg it failed in. local: a leg
        of this rank alone (no collectives: budget on the local clock)."""
        t0 = time.time()
        err = None
        try:
            if self.broken and not local:
                return None, {"skipped": f"no collectives after an earlier failure ({self.broken})"}
            if est_s > 0:
                # the same elapsed time on every rank (max over ranks), so every rank decides alike
                el = (time.time() - T_START) if local else self.elapsed_max()
                if el + est_s > self.budget:
                    return None, {"skipped": f"time budget: {el:.0f} s elapsed + ~{est_s:.0f} s estimated "
                                              f"> --budget-s {self.budget:.0f}"}
            self.leg, self.leg_sync = name, 0
            self._inject_here()
            res = fn()
            if not local:
                self._sync()  # leg-end agreement: every rank finished the leg
            return res, None
        except LegAborted:
            pass  # this rank was fine; another one failed (its message follows)
        except GroupBroken as e:
            return None, {"error": str(e), "rank": self.rank, "collectives": "broken: later legs skipped"}
        except (Exception, SystemExit) as e:
            import traceback

            err = f"{type(e).__name__}: {e}"[:600]
            print(f"bench.py: rank {self.rank} leg {name} failed:\n{traceback.format_exc()}", file=sys.stderr,
                  flush=True)
            if self.world == 1 or local:
                return None, {"error": err, "rank": self.rank}
            try:
                self._sync(fail=True)  # stands in for the collective the other ranks wait in
            except GroupBroken as g:
                return None, {"error": err, "rank": self.rank, "collectives": f"broken: {g}"}
        finally:
            self.leg = None
            self.leg_seconds[name] = round(time.time() - t0, 2)
            self._free_device()
        # aborted on every rank at the same collective: who failed and why
        try:
            errs = self._gather_objects(err)
        except GroupBroken as g:
            return None, {"error": err or "aborted by another rank", "rank": self.rank,
                          "collectives": f"broken: {g}"}
        failed = [i for i, e in enumerate(errs) if e]
        first = failed[0] if failed else None
        return None, {"error": errs[first] if failed else "aborted", "rank": first, "failed_ranks": failed}

    def marker(self, what: str) -> str | None:
        """Path of this launch's marker file `what` ("abort": a rank's collective
        failed; "printed": rank 0 printed the line), shared by the ranks of
        one launch (same host; tagged with rank 0's pid and start time, so
        launches one after another on one port never share one); None at N = 1."""
        if self.world == 1:
            return None
        import tempfile

        tag = f"{os.environ.get('MASTER_PORT', '')}_{self.run_tag}"
        return os.path.join(tempfile.gettempdir(), f"ecw_bench_{tag}.{what}")

    def touch(self, what: str):
        path = self.marker(what)
        if path:
            try:
                with open(path, "a") as f:
                    f.write(f"{self.rank} {time.time():.3f}\n")
            except OSError:
                pass

    def _free_device(self):
        """Return a finished leg's HBM to the device (never raises: after a GPU
        fault on this rank the context may refuse, and the next legs fail and
        abort on their own)."""
        if not self.dry:
            try:
                import gc

                import torch

                gc.collect()
                torch.cuda.empty_cache()
            except Exception as e:  # noqa: BLE001
                print(f"bench.py: rank {self.rank}: freeing device memory failed: {e}", file=sys.stderr)

    def close(self):
        if self.world > 1:
            import torch.distributed as dist

            try:
                dist.destroy_process_group()
            except Exception:
                pass


class Line:
    """Rank 0's one JSON line. The legs fill it in as they finish; it is
    printed exactly once: at the end, or -- with whatever is in it and an
    `error` -- by a watchdog thread (so a rank stuck inside a GPU call still
    gets its line out) when
      * the hard deadline passes (--deadline-s after the process started),
      * the launcher sends SIGTERM (torch.distributed.run does when another
        rank exits non-zero), or
      * another rank's collective failed (its "abort" marker) and rank 0 has
        not printed --collective-timeout + 30 s later (rank 0 is the stuck one).
    Every other rank exits at its deadline, or 15 s after rank 0 printed (its
    "printed" marker) if it is still running then (a hung rank), so a hang
    never holds the launcher until the deadline."""

    GRACE_AFTER_PRINT_S = 15.0

    def __init__(self, d: Dist, deadline_s: float, collective_timeout: float = 120.0):
        import signal
        import threading

        self.rank, self.data, self.printed = d.rank, {}, False
        self.expected = []  # the optional legs this run meant to measure (run_legs)
        self.lock = threading.Lock()
        self.d = d
        self.deadline = T_START + deadline_s + (0.0 if d.rank == 0 else 5.0)  # rank 0 prints first
        self.abort_grace = collective_timeout + 30.0
        r, w = os.pipe()
        os.set_blocking(w, False)
        signal.signal(signal.SIGTERM, lambda *_: None)  # the watchdog acts on it (set_wakeup_fd)
        signal.set_wakeup_fd(w)
        self._r = r
        threading.Thread(target=self._watch, daemon=True, name="bench-watchdog").start()

    @staticmethod
    def _age(path: str | None) -> float | None:
        try:
            return time.time() - os.path.getmtime(path) if path else None
        except OSError:
            return None

    def _watch(self):
        import select
        import signal

        leg = lambda: self.d.leg or "(between legs)"  # noqa: E731
        while True:
            left = self.deadline - time.time()
            if left <= 0:
                why = f"hard deadline: {self.deadline - T_START:.0f} s after start, still in leg {leg()}"
                break
            ready, _, _ = select.select([self._r], [], [], min(1.0, left))
            # the wakeup fd carries one byte per signal number; only SIGTERM is ours
            if ready and int(signal.SIGTERM) in os.read(self._r, 64):
                why = (f"terminated (SIGTERM) in leg {leg()}"
                       + ("; torch.distributed.run sends it when another rank exits" if self.d.world > 1 else ""))
                break
            if self.d.world > 1:
                if self.rank != 0:
                    age = self._age(self.d.marker("printed"))
                    if age is not None and age > self.GRACE_AFTER_PRINT_S:
                        print(f"bench.py: rank {self.rank} still in leg {leg()} {age:.0f} s after rank 0 printed the "
                              f"line: exiting", file=sys.stderr, flush=True)
                        os._exit(0)
                elif not self.printed:
                    age = self._age(self.d.marker("abort"))
                    if age is not None and age > self.abort_grace:
                        why = (f"rank 0 stuck in leg {leg()}: another rank's collective failed {age:.0f} s ago "
                               f"(a rank hung or died)")
                        break
        rc = 0
        if self.rank == 0:
            self.emit(error=why)
            rc = 0 if self.data.get("value") is not None or self.data.get("dry_run") else 1
        os._exit(rc)  # as main(): 0 whenever the line carries the main leg's `value`

    def update(self, **kv):
        with self.lock:
            self.data.update(kv)

    def set_leg(self, name: str, res, info):
        with self.lock:
            self.data[name] = res if info is None else info

    def emit(self, error: str | None = None):
        """Print the line once (rank 0). Main thread and watchdog race safely:
        the lock serialises them and the second caller finds `printed`."""
        if self.rank != 0:
            return
        with self.lock:
            if self.printed:
                return
            self.printed = True
            line = dict(self.data)
            if error:
                line["error"] = error
            # every leg that has no measurement in the line: failed, skipped, or cut off by `error`
            bad = [x for x in LEG_NAMES if isinstance(line.get(x), dict)
                   and ("error" in line[x] or "skipped" in line[x])]
            if "main_error" in line or line.get("value") is None and not line.get("dry_run"):
                bad = ["main"] + bad
            if error and self.d.leg and self.d.leg not in bad:
                bad.append(self.d.leg)
            # legs the run meant to measure that never reached the line (cut off by `error`)
            bad += [x for x in self.expected if x not in line and x not in bad]
            line["legs_not_measured"] = bad
            line["leg_seconds"] = dict(self.d.leg_seconds)
            sys.stdout.write(json.dumps(line, default=str) + "\n")
            sys.stdout.flush()
            self.d.touch("printed")


def plan(args, d: Dist, free_bytes: int, parity_num: int, fill: bool = False) -> dict:
    """A leg's workload and this rank's share of it (the same on every rank
    except the share). Main leg: args.stripes (default 8) stripes of
    args.block_mib (default 64) MiB PER GPU (weak scaling), or in total with
    --strong. fill: the configs[3] batch -- 256 stripes, B = the largest whole
    MiB at which the WHOLE batch fits one GPU's free HBM (the MIN over ranks,
    so the same B at every N), split by stripe (strong). free_bytes: this
    GPU's free HBM (only read for fill)."""
    from ecwide_amd.shard import hbm_fill_block_mib, plan_rank

    k = args.k
    if fill:
        total = HBM_FILL_STRIPES
        # the whole batch fits ONE GPU at this B, so B is the same at every N
        # (ranks sharing a device in a rehearsal hold the batch between them)
        mib = hbm_fill_block_mib(free_bytes, k, parity_num, total)
        mib = int(d.reduce(float(mib), "min"))
        if mib < 1:
            raise SystemExit(f"bench.py: {free_bytes} B free: too small for {total} stripes")
        block_mib, strong = float(mib), True
    else:
        total = args.stripes if args.stripes is not None else 8
        block_mib = args.block_mib if args.block_mib is not None else 64.0
        strong = args.strong
    B = int(block_mib * (1 << 20))
    align = (chunk_kib(args) << 10) if args.layout == "tiled" else 4096
    share = plan_rank(total, B, d.world, d.rank, strong, per_rank=total, align=align)
    if share["block_bytes"] <= 0:
        raise SystemExit("bench.py: more ranks than column tiles")
    stripes_total = total if strong else total * d.world
    return dict(hbm_fill=fill, strong=strong, stripes_total=stripes_total, block_bytes_full=B, share=share)


def chunk_kib(args) -> int:
    """The tiled layout's column piece of this leg (KiB): --chunk-kib, or the
    slab's default for k (ecwide_amd/slab.py default_chunk)."""
    if args.chunk_kib:
        return args.chunk_kib
    from ecwide_amd.slab import default_chunk

    return default_chunk(args.k) >> 10


def layout_desc(args) -> str:
    return {"blocks": "blocks (each block contiguous, block stride B + 4 KiB, [D.., G.., L..] per stripe)",
            "split": "split (each block contiguous, block stride B + 4 KiB, parity blocks in their own "
                     "region)"}.get(args.layout, f"tiled ({chunk_kib(args)} KiB column pieces: the k data "
                                                 f"pieces contiguous, parities in their own region)")


def workload_of(pl, k, m, r, g, world) -> str:
    """The workload's description: the same at every N (it names the per-GPU
    or total amount, never the rank count)."""
    B, S_total = pl["block_bytes_full"], pl["stripes_total"]
    if pl["hbm_fill"]:
        return (f"configs[3]/[4]: {S_total} independent CL(k={k}, r={r}, m={m}, g={g}) stripes of B={B >> 20} MiB "
                f"blocks (the batch that fills one GPU's HBM, {S_total * (k + m + g) * B / 2**30:.0f} GiB), split "
                f"by stripe over the GPUs: batched encode + repair of D0")
    if pl["strong"]:
        return (f"CL(k={k}, r={r}, m={m}, g={g}) B={B >> 20} MiB, {S_total} stripes in total split by stripe "
                f"over the GPUs: batched encode + repair of D0")
    return (f"CL(k={k}, r={r}, m={m}, g={g}) B={B >> 20} MiB, {pl['share']['stripes']} stripes per GPU (weak "
            f"scaling): batched encode + repair of D0")


def config_of(args, pl, k, m, r, g, world, enc_bytes, rep_bytes) -> dict:
    """The line's `config`: identical at every N apart from stripes_total."""
    sh = pl["share"]
    return {
        "workload": workload_of(pl, k, m, r, g, world),
        "k": k, "r": r, "m": m, "g": g, "block_bytes": pl["block_bytes_full"],
        "block_bytes_per_gpu": sh["block_bytes"],
        "stripes_per_gpu": sh["stripes"], "stripes_total": pl["stripes_total"], "seed": args.seed,
        "parallelism": "stripes partitioned over the GPUs, one process per GPU (no collectives on the data path)",
        "layout": layout_desc(args),
        "encode_bytes_per_step_per_gpu": enc_bytes,
        "repair_bytes_per_step_per_gpu": rep_bytes,
    }


# ---- CPU baseline (oracle: test infrastructure, never the measured product) --
def host_cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or platform.machine()


def cpu_stripe(args, k, m, r, B, threads_list, seconds, literal=False, repair=True, seed=None, kind="avx2"):
    """One whole stripe of CL(k, r, m) B-byte blocks through the reference's CPU
    flow, restated (oracle: test infrastructure, never the product): ECWide-C
    encodeData = ec_encode_data (kernel family `kind`: ISA-L 2.14's AVX2, or
    master's AVX-512 / AVX-512 + GFNI) for the global rows + one pass per local
    group (NativeCodec.cc:137-219), then (repair) decodeData of D0 =
    ec_encode_data of the r survivors with the all-ones table
    (NativeCodec.cc:237-248), both split by byte range over `threads` threads.
    GB/s (algorithmic bytes: inputs + outputs) per thread count, each timed for
    about seconds / len(threads_list) (at least one whole stripe)."""
    import ctypes

    import numpy as np

    import oracle

    orc = oracle.Oracle()
    oc = orc.codec("C", k, m, r, B)
    rng = np.random.default_rng(args.seed if seed is None else seed)
    data = [np.frombuffer(rng.bytes(B), np.uint8) for _ in range(k)]
    par = [np.zeros(B, np.uint8) for _ in range(oc.parity_num)]
    u8p = ctypes.POINTER(ctypes.c_uint8)
    dp = (u8p * k)(*[x.ctypes.data_as(u8p) for x in data])
    pp = (u8p * len(par))(*[x.ctypes.data_as(u8p) for x in par])
    nsrc = min(r, k)
    per_stripe = (k + oc.parity_num + ((nsrc + 1) if repair else 0)) * B
    ones = orc.init_tables_kind(kind, nsrc, 1, np.ones(nsrc, np.uint8))
    rep = np.zeros(B, np.uint8)
    rp = (u8p * 1)(rep.ctypes.data_as(u8p))
    srcs = data[1:nsrc] + [par[m]]
    sp = (u8p * nsrc)(*[x.ctypes.data_as(u8p) for x in srcs])
    kid = oracle.KINDS[kind]

    def run(threads):
        oc.encode_into(dp, pp, B, literal=literal, threads=threads, kind=kind)
        if repair:
            orc.L.orc_encode_data_mt_kind(kid, B, nsrc, 1, ones.ctypes.data_as(u8p), sp, rp, threads)

    run(max(threads_list))  # warm: fault in the output pages outside the timing
    res = {}
    for threads in threads_list:
        n, t0 = 0, time.perf_counter()
        while True:
            run(threads)
            n += 1
            el = time.perf_counter() - t0
            if el > seconds / len(threads_list) or n >= 50:
                break
        res[threads] = round(n * per_stripe / el / 1e9, 3)
    ok = True
    if repair and not literal:
        ok = bool(np.array_equal(rep, data[0]))
    return res, ok


def cpu_meta(orc=None) -> dict:
    from ecwide_amd.shard import host_threads

    import oracle

    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    return {"cores_all": host_threads(), "affinity_cores": affinity, "nproc": os.cpu_count(),
            "cap": 16, "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "host_cpu": host_cpu_model(),
            "isa": {x: (orc or oracle.Oracle()).have_kind(x) for x in ("avx2", "avx512", "gfni")}}


ISAL_FAMILY = {
    "avx2": "ISA-L 2.14's gf_Nvect_dot_prod_avx2 (4-bit split vpshufb, 32-byte vectors): the top of the 2.14 tarball "
            "ECWide-H bundles (isal:erasure_code/ec_multibinary.asm:119-135)",
    "avx512": "ISA-L master's gf_Nvect_dot_prod_avx512 (4-bit split vpshufb, 64-byte vectors)",
    "gfni": "ISA-L master's gf_Nvect_dot_prod_avx512_gfni (one vgf2p8affineqb per source byte and row, "
            "ec_init_tables_gfni 8-byte matrices)",
    "base": "ec_encode_data_base (scalar)",
}


def cpu_baseline(args, k, m, r, B):
    """The headline workload's CPU baseline (rank 0, N=1): one whole stripe
    through the reference's CPU flow in three kernel families. `value` is the
    family ISA-L master's dispatch picks on this host -- ECWide-C as built
    (ECWide-C/makefile:12-14 links /usr/lib/libisal.so from unpinned master,
    ECWide-C/README.md:34-39): AVX-512 + GFNI on the box's Zen 5 -- on 1 thread
    (ECWide-C's one ComputeWorker thread), with the thread scaling 1 -> 2 ->
    4 -> 8 -> the box's per-GPU CPU share (16). The other families (ISA-L
    2.14's AVX2 = what ECWide-H's tarball builds; master's AVX-512 without
    GFNI) at 1 and 16 threads beside it."""
    from ecwide_amd.shard import host_threads

    import oracle

    orc = oracle.Oracle()
    master = orc.isal_master_kind()
    allc = host_threads()
    tl = sorted({t for t in (1, 2, 4, 8) if t < allc} | {allc})
    res, ok = cpu_stripe(args, k, m, r, B, tl, args.cpu_seconds, kind=master)
    if not ok:
        raise SystemExit("CPU baseline repair mismatch")
    per_thread = {t: round(v / t, 3) for t, v in res.items()}
    fam = {master: {"1": res[1], str(allc): res[allc]}}
    for kind in ("avx2", "avx512", "gfni"):
        if kind != master and orc.have_kind(kind):
            rk, ok = cpu_stripe(args, k, m, r, B, sorted({1, allc}), args.cpu_seconds / 2, kind=kind)
            if not ok:
                raise SystemExit(f"CPU baseline repair mismatch ({kind})")
            fam[kind] = {"1": rk[1], str(allc): rk[allc]}
    out = {
        "value": res[1],
        "unit": "GB/s",
        "cores": 1,
        "kind": "port",
        "isal_family": master,
        "sample": (f"1 whole stripe of the workload, CL(k={k},r={r},m={m}) B={B >> 20} MiB: ECWide-C encodeData "
                   f"flow (global + per-group ec_encode_data passes) + decodeData of D0, on "
                   f"{ISAL_FAMILY[master]}; 1 thread = ECWide-C's one ComputeWorker thread"),
        "dispatch_rule": ("ISA-L master's ec_encode_data / ec_init_tables dispatch: AVX-512 (F+BW) + GFNI -> "
                          "avx512_gfni, else AVX-512 -> avx512, else AVX2 -> avx2; ISA-L 2.14 stops at AVX2. "
                          f"This host: {master}"),
        "value_all_cores": res[allc],
        "thread_scaling_GBps": {str(t): v for t, v in res.items()},
        "per_thread_GBps": {str(t): v for t, v in per_thread.items()},
        "families_GBps": fam,
        "ecwide_c_as_built": f"{master} (value, value_all_cores)",
        "ecwide_h_isal_2_14": "avx2 (families_GBps.avx2)",
        "all_cores_note": (f"{allc} threads = this job's CPU share on the GPU box (the pool gives one GPU's job 16 of "
                           f"the host's CPUs and caps worker pools there); the host has more cores, which other "
                           f"jobs use"),
        **cpu_meta(orc),
    }
    for kind in ("avx2", "avx512", "gfni"):
        if kind in fam:
            out[f"value_{kind}"] = fam[kind]["1"]
            out[f"value_{kind}_all_cores"] = fam[kind][str(allc)]
    return out


# ---- verification (outside the timed region) ---------------------------------
def verify(args, slab, out, pl, k, m, r) -> dict:
    """Sampled parity vs the oracle (8 KiB column windows at the first,
    middle and last piece of this rank's first/middle/last stripe; columns
    are independent, so a window is an exact check of those bytes), every
    stripe's D0 repair == D0 on the device, and at the default shape stripe 0
    vs the committed full-size SHA-256 digests of manifest 'cfg3_full'."""
    import hashlib

    import numpy as np
    import torch

    import oracle

    orc = oracle.Oracle()
    sh = pl["share"]
    B, S, s0, off0 = sh["block_bytes"], sh["stripes"], sh["s0"], sh["col_offset"]
    res = {"windows": 0, "repairs": 0, "digests": False}
    W = min(8192, B)
    oc = orc.codec("C", k, m, r, W)
    for s in sorted({0, S // 2, S - 1}):
        par = slab.parity(s)
        for off in sorted({0, (B // 2) // W * W, B - W}):
            want = oc.encode([orc.fill(W, args.seed, s0 + s, j, off0 + off) for j in range(k)])
            for i, w in enumerate(want):
                if not np.array_equal(par[i][off:off + W].cpu().numpy(), w):
                    return dict(res, ok=False, failed=f"stripe {s0 + s} parity {i} at column {off0 + off}")
            res["windows"] += 1
    for s in range(S):
        if not torch.equal(out[s * B:(s + 1) * B], slab.block(s, 0)):
            return dict(res, ok=False, failed=f"stripe {s0 + s} D0 repair")
        res["repairs"] += 1
    mf = os.path.join(REPO, "tests", "golden", "manifest.json")
    if s0 == 0 and off0 == 0 and os.path.exists(mf):
        # the full-size digests of this shape and seed (cfg1_full / cfg2_full / cfg3_full), if committed
        e = next((x for x in json.load(open(mf)).get("full", [])
                  if (x["k"], x["m"], x["r"], x["len"], x["seed"]) == (k, m, r, B, args.seed)), None)
        if e:
            got = [hashlib.sha256(p.cpu().numpy().tobytes()).hexdigest() for p in slab.parity(0)]
            rep = hashlib.sha256(out[:B].cpu().numpy().tobytes()).hexdigest()
            if got != e["parity_sha256"] or rep != e["repair_d0_sha256"]:
                return dict(res, ok=False, failed=f"stripe 0 vs manifest {e['name']} digests")
            res["digests"] = True
            res["digest_entry"] = e["name"]
    return dict(res, ok=True)


def other_layouts(args, E, codec, slab, S, B, out, enc_bytes, rep_bytes, dev) -> dict:
    """Encode / repair rates of the bench workload in whole-block layouts --
    the split slab (data blocks, then parity blocks: ISA-L's separate data /
    coding arrays, batched) and pointer tables over separately allocated 64
    MiB blocks (the reference's per-block pointers, NativeCodec.cc:158-170,
    one ecw_encode_ptrs_dev launch for all stripes) -- timed INTERLEAVED with
    the headline tiled slab (T, S, P in every round, equal steps, one
    process), so the comparison is not confounded by where each allocation
    landed physically."""
    import statistics

    import torch

    n2, rounds = args.other_layout_steps, args.other_layout_rounds
    k, np_ = codec.encodeDataNum, codec.parityNum
    split = E.StripeSlab(codec, stripes=S, block_bytes=B, device=dev, layout="split")
    split.fill_random(seed=args.seed)
    data = [[torch.empty(B, dtype=torch.uint8, device=f"cuda:{dev}") for _ in range(k)] for _ in range(S)]
    par = [[torch.empty(B, dtype=torch.uint8, device=f"cuda:{dev}") for _ in range(np_)] for _ in range(S)]
    for s_ in range(S):
        src = split.data(s_)
        for j in range(k):
            data[s_][j].copy_(src[j])  # the same bytes as the slabs
    batch = E.BlockBatch(codec, data, par)
    outs = [out[s_ * B:(s_ + 1) * B] for s_ in range(S)]
    legs = {
        "tiled": (slab.encode, lambda: slab.repair(0, out)),
        "split": (split.encode, lambda: split.repair(0, out)),
        "pointer": (batch.encode, lambda: batch.repair(0, outs)),
    }
    for enc, rep in legs.values():  # warm every leg once
        enc()
        rep()
    torch.cuda.synchronize()
    rates = {name: ([], []) for name in legs}
    for _ in range(rounds):
        for name, (enc, rep) in legs.items():
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            for _ in range(n2):
                enc()
            e[1].record()
            for _ in range(n2):
                rep()
            e[2].record()
            torch.cuda.synchronize()
            rates[name][0].append(round(enc_bytes * n2 / (e[0].elapsed_time(e[1]) * 1e-3) / 1e9, 1))
            rates[name][1].append(round(rep_bytes * n2 / (e[1].elapsed_time(e[2]) * 1e-3) / 1e9, 1))
    # the pointer leg's parities equal the tiled slab's (same bytes in, same code)
    same = all(torch.equal(par[s_][i], slab.parity(s_)[i]) for s_ in (0, S - 1) for i in (0, np_ - 1))
    desc = {
        "tiled": "tiled slab (the headline layout)",
        "split": "split slab: whole blocks (stride B + 4 KiB), the data blocks of all stripes then their parity "
                 "blocks (ecw_encode_batch_split_dev; encode with the write window, repair with the K=4 diagonal "
                 "XOR schedule + write window: DESIGN.md 4.1, 4.2)",
        "pointer": f"pointer tables: {S * (k + np_)} separately allocated {B >> 20} MiB blocks, one "
                   f"ecw_encode_ptrs_dev / ecw_xor_reduce_ptrs_dev launch over the {S} stripes (encode with the "
                   f"per-XCD tile order + write window, repair with the K=4 diagonal XOR schedule + write window)",
    }
    res = {"interleaved": f"{rounds} rounds x (tiled, split, pointer) x {n2} encodes + {n2} repairs, one process"}
    for name, (en, rp) in rates.items():
        med = statistics.median(en)
        res[name] = {"layout": desc[name], "encode_GBps": med, "repair_GBps": statistics.median(rp),
                     "encode_frac": round(med / HBM_PEAK_GBS, 4), "encode_GBps_rounds": en, "repair_GBps_rounds": rp}
    res["pointer"]["parity_equals_tiled"] = bool(same)
    del split, data, par, batch
    return res


# ---- the PCIe-inclusive rate --------------------------------------------------
PCIE_GEN5_X16_GBPS = 63.0  # per direction: 32 GT/s x 16 lanes x 128/130 / 8


def host_resident_leg(args, d, iters: int) -> dict:
    """PCIe-inclusive rate on EVERY rank at once: each rank's own stripe
    (stripe id = rank) lives in pinned host memory on its GPU's NUMA node
    (ecwide_amd.PinnedHost = ecw_host_alloc: pages preferred on the node of
    the GPU's PCIe root, faulted in, registered); ecw_encode / ecw_repair
    pipeline it through HBM with hipMemcpyAsync in and out (8 MiB column
    slices, 3 HBM slots, H2D / kernel / D2H on three streams). All ranks run
    between two barriers; the aggregate is every rank's bytes over the
    slowest rank's time, so at N = 8 it is what the node's eight PCIe links
    and its DRAM deliver together. Reported beside `value`,
    never as it. `d` None: one rank (the --host-resident mode)."""
    import numpy as np
    import torch

    import ecwide_amd as E

    world, rank, dev = (1, 0, 0) if d is None else (d.world, d.rank, d.dev)
    barrier = (lambda: None) if d is None else d.barrier
    k, m, r = args.k, args.m, args.r
    B = int((args.block_mib or 64.0) * (1 << 20))
    codec = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False, device=dev)
    nblk = k + codec.parityNum
    t0 = time.perf_counter()
    host = None
    if args.pageable:
        hb, node = np.zeros((nblk + 1) * B, np.uint8), -1
    else:
        host = E.PinnedHost((nblk + 1) * B, dev)
        hb, node = host.array, host.numa_node
    alloc_s = time.perf_counter() - t0
    slab = E.StripeSlab(codec, stripes=1, block_bytes=B, device=dev)
    slab.fill_random(seed=args.seed, s0=rank)
    for j in range(k):
        torch.from_numpy(hb[j * B:(j + 1) * B]).copy_(slab.block(0, j))
    slab.encode()  # the expected parities, from the device-resident path
    want = [p.cpu().numpy() for p in slab.parity(0)]
    del slab
    torch.cuda.synchronize()
    views = [hb[i * B:(i + 1) * B] for i in range(nblk)]
    out = hb[nblk * B:(nblk + 1) * B]
    nsrc = len(codec.repairSources(0))
    enc_b, rep_b = nblk * B, (nsrc + 1) * B
    codec.encodeData(views[:k], views[k:])  # warm
    codec.repairBlock(views, 0, out)
    barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        codec.encodeData(views[:k], views[k:])
    t1 = time.perf_counter()
    for _ in range(iters):
        codec.repairBlock(views, 0, out)
    t2 = time.perf_counter()
    barrier()
    el = time.perf_counter() - t0
    ok = np.array_equal(out, views[0]) and all(np.array_equal(a, b) for a, b in zip(views[k:], want))
    h2d = iters * (k * B + nsrc * B) / (t2 - t0) / 1e9  # bytes the pipeline moved host -> device per second
    own = iters * (enc_b + rep_b) / (t2 - t0) / 1e9
    if host is not None:
        host.free()
    gather = (lambda x: [x]) if d is None else d.gather
    reduce = (lambda x, op: x) if d is None else d.reduce
    el_max = reduce(el, "max")
    all_ok = reduce(1.0 if ok else 0.0, "min") > 0.5
    rank_gbps, rank_h2d = gather(own), gather(h2d)
    rank_node = [int(x) for x in gather(float(node))]
    rank_dev_node = [int(x) for x in gather(float(E._lib.lib.ecw_device_numa_node(dev)))]
    return {
        "GBps": round(world * iters * (enc_b + rep_b) / el_max / 1e9, 2),
        "scope": ("all ranks at once, each its own stripe in pinned host memory on its GPU's NUMA node; aggregate "
                  "= every rank's bytes / the slowest rank's time between barriers") if world > 1 else "one rank",
        "encode_GBps": round(iters * enc_b / (t1 - t0) / 1e9, 2),
        "repair_GBps": round(iters * rep_b / (t2 - t1) / 1e9, 2),
        "pcie_bytes_per_step": enc_b + rep_b,
        "h2d_GBps": round(h2d, 2),
        "frac_of_pcie_gen5_x16": round(h2d / PCIE_GEN5_X16_GBPS, 4),
        "rank_GBps": [round(x, 2) for x in rank_gbps],
        "rank_h2d_GBps": [round(x, 2) for x in rank_h2d],
        "rank_numa_node": rank_node,
        "rank_gpu_numa_node": rank_dev_node,
        "numa_local": all(a == b for a, b in zip(rank_node, rank_dev_node)) if not args.pageable else None,
        "alloc_s": round(alloc_s, 2),
        "iters": iters, "verified": bool(all_ok),
        "host_blocks": "pageable" if args.pageable else "pinned, NUMA-local (ecw_host_alloc)",
        "config": f"CL(k={k}, r={r}, m={m}) one stripe of {B >> 20} MiB blocks per rank in host memory: encodeData + "
                  f"repair of D0; 8 MiB column slices, 3 HBM slots, H2D / kernel / D2H on three streams",
    }


def chunkgen_leg(args, cpu_seconds: float = 0.0) -> dict:
    """ECWide-C's ChunkGenerator replay (BASELINE configs[0]; the default
    ECWide-C/config/scheme.ini: CL k=32, groupDataNum=11, m=3, 64 MiB chunks):
    source blocks in pinned host memory (BufferUnit's direct ByteBuffers),
    encodeChunks timed exactly where ChunkGenerator.java:126-131 times it
    (host -> HBM -> host), then generateChunks writes the D/G/L chunk files
    (FileOp.writeFile) into a temporary directory, timed separately."""
    import shutil
    import tempfile

    import numpy as np

    from ecwide_amd.chunk_generator import ChunkGenerator
    from ecwide_amd.codec import CodingScheme

    import oracle

    scheme = CodingScheme.fromConfigText("codeType = CL\nk = 32\ngroupDataNum = 11\nglobalParityNum = 3\n"
                                         "chunkSizeBits = 26\n")
    tmp = tempfile.mkdtemp(prefix="ecw_chunks_")
    try:
        gen = ChunkGenerator(scheme, tmp, "prng")  # the reference's bytes: zero L blocks
        gen.fill_prng(args.seed)
        gen.encode_chunks()  # warm (first-call staging)
        ms = []
        for _ in range(3):
            t0 = time.perf_counter()
            gen.encode_chunks()
            ms.append((time.perf_counter() - t0) * 1e3)
        B, nb = scheme.chunkSize, scheme.k + gen.codec.parityNum
        # parity of the replay: an 8 KiB window of every global parity vs the oracle
        W = 8192
        oc = oracle.Oracle().codec("C", scheme.k, scheme.globalParityNum, scheme.groupDataNum, W)
        want = oc.encode([np.ascontiguousarray(b[:W]) for b in gen.data], literal=True)
        ok = all(np.array_equal(gen.parity[i][:W], w) for i, w in enumerate(want))
        t0 = time.perf_counter()
        paths = gen.generate_chunks(0)
        wms = (time.perf_counter() - t0) * 1e3
        best = min(ms)
        cpu = None
        if cpu_seconds > 0:
            # the reference's own configs[0] timing on this host: encodeChunks on the CPU, i.e. encodeData of
            # the same 64 MiB chunks, literal mode, no repair (ChunkGenerator.java:126-131), one thread
            fam = oracle.Oracle().isal_master_kind()  # ECWide-C as built (ISA-L master's dispatch here)
            res, _ = cpu_stripe(args, scheme.k, scheme.globalParityNum, scheme.groupDataNum, B, [1], cpu_seconds,
                                literal=True, repair=False, seed=args.seed, kind=fam)
            cpu = {"encodeChunks_GBps": res[1], "encodeChunks_ms": round(nb * B / (res[1] * 1e9) * 1e3, 1),
                   "cores": 1, "kind": "port", "isal_family": fam,
                   "sample": "encodeData of one stripe of the default scheme.ini's 64 MiB chunks (literal L), "
                             "ECWide-C's one ComputeWorker thread"}
        return {
            "config": "ChunkGenerator replay, default scheme.ini: CL(k=32, r=11, m=3), 64 MiB chunks, zero L blocks "
                      "(the reference's bytes), pinned source buffers",
            "encodeChunks_ms": [round(x, 3) for x in ms],
            "encodeChunks_GBps": round(nb * B / (best * 1e-3) / 1e9, 2),
            "generateChunks_ms": round(wms, 1), "chunk_files": len(paths),
            "generateChunks_GBps": round(nb * B / (wms * 1e-3) / 1e9, 2), "verified": bool(ok),
            "cpu_baseline": cpu,
        }
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def host_resident(args):
    """--host-resident: the PCIe-inclusive leg on its own, as a JSON line."""
    import torch

    torch.cuda.set_device(0)
    leg = host_resident_leg(args, None, max(1, args.steps // 4))
    line = {"metric": ("host-resident encode + single-block-repair GB/s "
                       + ("(pageable host blocks, e.g. Java direct ByteBuffers)" if args.pageable
                          else "(pinned host blocks, hipMemcpyAsync in/out)")),
            "value": leg["GBps"], "unit": "GB/s", "n_gpus": 1}
    line.update(leg)
    print(json.dumps(line), flush=True)


# ---- ECWide-H's synchronous small calls ----------------------------------------
def small_calls(args):
    """ECWide-H encodes one chunk per synchronous ISA-L call (g_encode:
    ec_encode_data(4096, GK=11, 3, ...), ECWide-H/proxy/encode.cpp:145-175),
    from its proxy threads (proxy.cpp:2001-2012). Here the same calls go
    through libecw_isal.so (the ISA-L-signature shim) to the GPU's resident
    request service; the CPU baseline is the oracle's AVX2 port of ISA-L's
    kernel making the same calls from one thread. Both sides are driven from
    Python through ctypes (same per-call overhead on both)."""
    import ctypes
    import threading

    import numpy as np

    import ecwide_amd  # noqa: F401  (torch first, then libecwide.so)

    k, m, ln = 11, 3, args.small_len
    shim = ctypes.CDLL(os.path.join(REPO, "ecwide_amd", "libecw_isal.so"))
    u8p = ctypes.POINTER(ctypes.c_uint8)
    full = np.zeros((k + m) * k, np.uint8)
    shim.gf_gen_cauchy1_matrix(full.ctypes.data_as(u8p), k + m, k)
    tbl = np.zeros(32 * k * m, np.uint8)
    shim.ec_init_tables(k, m, full[k * k:].copy().ctypes.data_as(u8p), tbl.ctypes.data_as(u8p))
    tp = tbl.ctypes.data_as(u8p)
    rng = np.random.default_rng(args.seed)

    def buffers():
        d = [rng.integers(0, 256, ln, dtype=np.uint8) for _ in range(k)]
        p = [np.zeros(ln, np.uint8) for _ in range(m)]
        return d, p, (u8p * k)(*[x.ctypes.data_as(u8p) for x in d]), (u8p * m)(*[x.ctypes.data_as(u8p) for x in p])

    # parity of the first call vs the oracle (outside the timing)
    import oracle

    orc = oracle.Oracle()
    d0, p0, dp0, pp0 = buffers()
    shim.ec_encode_data(ln, k, m, tp, dp0, pp0)
    want = orc.encode_data(tbl, d0, m, avx2=True)
    verified = all(np.array_equal(a, b) for a, b in zip(p0, want))

    def run_threads(nt, calls, fn):
        bufs = [buffers() for _ in range(nt)]
        for b in bufs:
            fn(b)  # warm
        def work(b):
            for _ in range(calls):
                fn(b)
        th = [threading.Thread(target=work, args=(b,)) for b in bufs]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        el = time.perf_counter() - t0
        n = nt * calls
        return {"threads": nt, "calls": n, "us_per_call_per_thread": round(el / calls * 1e6, 2),
                "calls_per_s": round(n / el), "GBps": round(n * (k + m) * ln / el / 1e9, 3)}

    gpu = [run_threads(nt, args.small_calls_n, lambda b: shim.ec_encode_data(ln, k, m, tp, b[2], b[3]))
           for nt in (1, 4, 16)]
    L = orc.L

    def cpu_call(b):
        L.orc_encode_data_avx2(ln, k, m, tp, b[2], b[3])

    cpu = run_threads(1, max(args.small_calls_n, 20000), cpu_call)
    seq = ecwide_h_sequence(args, shim, orc, ln)
    line = {
        "metric": "synchronous small encode calls GB/s (ECWide-H g_encode: ec_encode_data one 4 KiB chunk per call)",
        "value": gpu[0]["GBps"], "unit": "GB/s", "n_gpus": 1, "higher_is_better": True,
        "config": {"workload": f"RS-Cauchy k={k}, m={m}, {ln} B blocks, one stripe per synchronous call from each "
                               f"thread, through libecw_isal.so (ISA-L signatures) to the resident request service",
                   "bytes_per_call": (k + m) * ln},
        "threads": gpu, "verified": bool(verified), "ecwide_h_sequence": seq,
        "cpu_baseline": dict(cpu, value=cpu["GBps"], unit="GB/s", cores=1, kind="port",
                             sample="the same calls on the oracle's AVX2 port of ISA-L gf_3vect_dot_prod_avx2, "
                                    "1 thread", host_cpu=host_cpu_model()),
    }
    print(json.dumps(line), flush=True)


def ecwide_h_sequence(args, shim, orc, ln: int) -> dict:
    """ECWide-H's whole per-chunk call mix (ECWide-H/proxy/encode.cpp:113-238,
    geometry common.hpp:21-32): l_encode (XOR of LK=11 through the all-ones
    row of gf_gen_rs_matrix), g_encode (Cauchy GK=11 -> 3), l_middle (XOR of
    NODE=4), l_decode (XOR of 5), each rebuilding its matrix and tables per
    call as the reference does. GPU: the shim (the XOR calls take the
    service's plain-XOR path); CPU: the same calls on the oracle's port."""
    import ctypes
    import threading

    import numpy as np

    u8p = ctypes.POINTER(ctypes.c_uint8)
    # (sources, outputs, matrix generator rows, cauchy?)
    calls = [(11, 1, False), (11, 3, True), (4, 1, False), (5, 1, False)]
    nbytes = sum(k + m for k, m, _ in calls) * ln

    def bufs():
        rng = np.random.default_rng(args.seed + 1)
        d = [rng.integers(0, 256, ln, dtype=np.uint8) for _ in range(11)]
        outs = [[np.zeros(ln, np.uint8) for _ in range(m)] for _, m, _ in calls]
        dp = [(u8p * k)(*[x.ctypes.data_as(u8p) for x in d[:k]]) for k, _, _ in calls]
        op = [(u8p * m)(*[x.ctypes.data_as(u8p) for x in o]) for (_, m, _), o in zip(calls, outs)]
        mats = [np.zeros((k + m) * k, np.uint8) for k, m, _ in calls]
        tbls = [np.zeros(32 * k * m, np.uint8) for k, m, _ in calls]
        return d, outs, dp, op, mats, tbls

    def run(gen_rs, gen_cauchy, init, encode, b):
        _, _, dp, op, mats, tbls = b
        for i, (k, m, cauchy) in enumerate(calls):
            mp, tp = mats[i].ctypes.data_as(u8p), tbls[i].ctypes.data_as(u8p)
            (gen_cauchy if cauchy else gen_rs)(mp, k + m, k)
            init(k, m, mats[i][k * k:].ctypes.data_as(u8p), tp)
            encode(ln, k, m, tp, dp[i], op[i])

    L = orc.L
    gpu_run = lambda b: run(shim.gf_gen_rs_matrix, shim.gf_gen_cauchy1_matrix, shim.ec_init_tables,
                            shim.ec_encode_data, b)
    cpu_run = lambda b: run(L.orc_gen_rs_matrix, L.orc_gen_cauchy1_matrix, L.orc_init_tables,
                            L.orc_encode_data_avx2, b)
    # parity of one sequence: GPU outputs == CPU outputs on the same inputs
    bg, bc = bufs(), bufs()
    gpu_run(bg)
    cpu_run(bc)
    verified = all(np.array_equal(x, y) for og, oc in zip(bg[1], bc[1]) for x, y in zip(og, oc))
    n = max(1000, args.small_calls_n // 2)

    def timed(fn, nt, service=False):
        import numpy as np

        import ecwide_amd as E

        bs = [bufs() for _ in range(nt)]
        lat = [[] for _ in range(nt)]

        def work(i):
            for _ in range(n):
                t = time.perf_counter()
                fn(bs[i])
                lat[i].append(time.perf_counter() - t)

        th = [threading.Thread(target=work, args=(i,)) for i in range(nt)]
        c0 = E.service_counters(0) if service else None
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        el = time.perf_counter() - t0
        res = {"threads": nt, "sequences": n * nt, "us_per_sequence_per_thread": round(el / n * 1e6, 2),
               "GBps": round(n * nt * nbytes / el / 1e9, 3)}
        all_lat = np.array([x for row in lat for x in row]) * 1e6
        res["us_per_sequence_p50_p99"] = [round(float(np.percentile(all_lat, q)), 2) for q in (50, 99)]
        if service:
            # every call of a sequence is a service candidate (<= 64 KiB, <= 8 rows)
            c1 = E.service_counters(0)
            served, declined = c1["served"] - c0["served"], c1["declined"] - c0["declined"]
            res["service"] = {"served": served, "declined": declined,
                              "hit_rate": round(served / max(1, served + declined), 4), "broken": c1["broken"]}
        return res

    # one thread each: driven from Python, the 16 ctypes calls of a sequence
    # cost both sides the same interpreter time, and more threads would only
    # measure the GIL (tools/csrc/shim_bench.c `seq` times the GPU side from C)
    return {"calls": "l_encode 11->1 XOR, g_encode 11->3 Cauchy, l_middle 4->1 XOR, l_decode 5->1 XOR, "
                     "tables rebuilt per call; driven from Python on both sides",
            "bytes_per_sequence": nbytes, "verified": bool(verified),
            "gpu": timed(gpu_run, 1, service=True), "cpu_port": timed(cpu_run, 1)}


# ---- the bench ------------------------------------------------------------------
def dry_main(args, d: Dist) -> dict:
    """The main leg without a GPU (--dry-run: the CPU test of the N>1 path):
    the leg's plan, a stand-in timed region (each rank sleeps a rank-dependent
    time) between the same barriers, the same reductions, and the line's
    `config` built exactly as the real run builds it."""
    k, m, r = args.k, args.m, args.r
    g = -(-k // r)
    pl = plan(args, d, int(args.dry_run_free_gib * (1 << 30)), m + g, fill=args.hbm_fill)
    sh = pl["share"]
    enc_bytes = sh["stripes"] * (k + m + g) * sh["block_bytes"]
    rep_bytes = sh["stripes"] * (min(r, k) + 1) * sh["block_bytes"]
    el = dry_timed(d, 0.05)
    el_max = d.reduce(el, "max")
    shares = [d.gather(float(sh[key])) for key in ("s0", "stripes", "block_bytes", "col_offset")]
    per_rank = d.gather(el)
    steps = max(1, args.steps)
    return {"metric": METRIC, "value": None, "unit": "GB/s", "dry_run": True, "n_gpus": d.world,
            "scaling": "strong" if pl["strong"] else "weak",
            "hbm_fill": pl["hbm_fill"], "stripes_total": pl["stripes_total"],
            "block_bytes": pl["block_bytes_full"], "el_max": el_max, "rank_seconds": per_rank,
            "rank_ms_per_step": [round(x / steps * 1e3, 4) for x in per_rank],
            "roofline": {"rank_launch_ms": [round(x * 1e3 / steps, 4) for x in per_rank]},
            "config": config_of(args, pl, k, m, r, g, d.world, enc_bytes, rep_bytes),
            "shares": [dict(s0=int(a), stripes=int(b), block_bytes=int(c), col_offset=int(o))
                       for a, b, c, o in zip(*shares)]}


DRY_SLOW = [1.0]  # --dry-run-slow


def dry_timed(d: Dist, unit_s: float) -> float:
    d.barrier()
    t0 = time.perf_counter()
    time.sleep(unit_s * DRY_SLOW[0] * (1 + d.rank))
    d.barrier()
    return time.perf_counter() - t0


def dry_configs4(args, d: Dist) -> dict:
    k, m, r = args.k, args.m, args.r
    p4 = plan(args, d, int(args.dry_run_free_gib * (1 << 30)), m + -(-k // r), fill=True)
    el = dry_timed(d, 0.02)
    return {"stripes_total": p4["stripes_total"], "block_bytes": p4["block_bytes_full"],
            "stripes_per_gpu": p4["share"]["stripes"],
            "rank_ms_per_step": [round(x / args.configs4_steps * 1e3, 4) for x in d.gather(el)],
            "shares": [dict(s0=int(a), stripes=int(b)) for a, b in
                       zip(*[d.gather(float(p4["share"][key])) for key in ("s0", "stripes")])]}


def dry_shape(args, d: Dist, leg_def) -> dict:
    name, _, sk, sm, sr, mib, stripes, seed = leg_def
    a = argparse.Namespace(**vars(args))
    a.k, a.m, a.r, a.block_mib, a.stripes, a.seed, a.strong = sk, sm, sr, float(mib), stripes, seed, False
    ps = plan(a, d, int(args.dry_run_free_gib * (1 << 30)), sm + -(-sk // sr))
    el = dry_timed(d, 0.01)
    return {"stripes_per_gpu": ps["share"]["stripes"], "stripes_total": ps["stripes_total"],
            "block_bytes": ps["block_bytes_full"],
            "rank_ms_per_step": [round(x / args.shape_steps * 1e3, 4) for x in d.gather(el)]}


def dry_host(args, d: Dist) -> dict:
    """host_resident_leg's orchestration: every rank between two barriers,
    the same gathers (no GPU: no pinning)."""
    hel = d.reduce(dry_timed(d, 0.01), "max")
    return {"el_max": hel, "rank_GBps": d.gather(0.0), "rank_h2d_GBps": d.gather(0.0),
            "rank_numa_node": [int(x) for x in d.gather(-1.0)],
            "rank_gpu_numa_node": [int(x) for x in d.gather(-1.0)], "verified": bool(d.reduce(1.0, "min"))}


def device_leg(args, d: Dist, E, pl: dict, k: int, m: int, r: int, steps: int, warmup: int, layout: str) -> dict:
    """Fill this rank's share of a leg in HBM, time exactly `steps` steps
    (encode of the slab + repair of D0 of every stripe) between barriers and
    synchronisations on both sides, then time each kernel with events on the
    launch stream in a second pass of the same steps (so the timed region
    carries no event overhead). Returns the slab, the times and the max over
    ranks."""
    import torch

    sh = pl["share"]
    B, S, s0 = sh["block_bytes"], sh["stripes"], sh["s0"]
    codec = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False, device=d.dev)
    slab = E.StripeSlab(codec, stripes=S, block_bytes=B, device=d.dev, layout=layout,
                        chunk=chunk_kib(args) << 10, unit_pad=args.unit_pad)
    out = torch.empty(S * B, dtype=torch.uint8, device=f"cuda:{d.dev}")
    slab.fill_random(seed=args.seed, s0=s0, col_offset=sh["col_offset"])
    torch.cuda.synchronize()
    enc_bytes, rep_bytes = slab.encode_bytes(), slab.repair_bytes(0)

    def step(evs=None):
        if evs is not None:
            evs[0].record()
        slab.encode()
        if evs is not None:
            evs[1].record()
        slab.repair(0, out)
        if evs is not None:
            evs[2].record()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    # timed region: exactly `steps` steps
    d.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    d.barrier()
    el = time.perf_counter() - t0
    el_max = d.reduce(el, "max")
    rank_s = d.gather(el)
    # per-kernel durations: events on the launch stream (torch's current
    # stream: slab.encode / repair launch on it)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    for i in range(steps):
        step(evs[i])
    torch.cuda.synchronize()
    enc_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / steps
    rep_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / steps
    return dict(codec=codec, slab=slab, out=out, enc_bytes=enc_bytes, rep_bytes=rep_bytes, el_max=el_max,
                rank_s=rank_s, enc_ms=enc_ms, rep_ms=rep_ms, rank_enc_ms=d.gather(enc_ms),
                enc_ms_max=d.reduce(enc_ms, "max"), rep_ms_max=d.reduce(rep_ms, "max"))


def pmc_traffic(args, k, r, m, B, S, enc_bytes, launches):
    """PMC-measured HBM bytes of one encode launch (profiles/pmc_traffic.json,
    written by tools/prof_summary.py from separate FETCH_SIZE / WRITE_SIZE
    rocprofv3 passes over this very workload), or None."""
    if not os.path.exists(args.pmc):
        return None, None
    try:
        pmc = json.load(open(args.pmc))
        key = f"k{k}_r{r}_m{m}_B{B}_S{S}" + {"tiled": f"_tiled{chunk_kib(args)}k", "split": "_split"}.get(args.layout, "")
        ratio = pmc.get(key, {}).get("traffic_over_algorithmic")
        if not ratio:
            return None, None
        src = (f"profiles/{os.path.basename(args.pmc)}[{key}]: traffic/algorithmic ratio of separate rocprofv3 "
               f"FETCH_SIZE / WRITE_SIZE passes over this workload (committed; not measured in this run)")
        return ratio * enc_bytes / launches, src
    except Exception:
        return None, None


def read_kernel_stats(path: str) -> list:
    """Rows of a rocprofv3 --stats kernel summary (…_kernel_stats.csv):
    (name, calls, average ns)."""
    import csv

    with open(path, newline="") as f:
        return [(row["Name"], int(row["Calls"]), float(row["AverageNs"])) for row in csv.DictReader(f)]


def profile_fracs(args, enc_bytes_per_launch: int, rep_bytes_per_launch: int) -> dict:
    """The roofline recomputed from the committed rocprof summary of this
    workload (--profile-csv): algorithmic bytes per launch / the kernel's
    average rocprof duration / 8 TB/s, for the encode (the most-called
    encode_kernel row) and the repair (the most-called xor_kernel row). Only
    at the default workload, the one the summary was taken on."""
    default = (args.k, args.m, args.r, args.block_mib or 64.0, args.stripes or 8, args.layout, args.chunk_kib or 8,
               args.unit_pad, args.hbm_fill, args.strong) == (128, 3, 27, 64.0, 8, "tiled", 8, 0, False, False)
    rel = os.path.relpath(args.profile_csv, REPO)
    if not default or not os.path.exists(args.profile_csv):
        return {"profile_source": None, "profile_note": f"{rel}: " + ("absent" if default else
                                                                       "taken on the default workload only")}
    rows = read_kernel_stats(args.profile_csv)

    def pick(tag):
        c = [x for x in rows if tag in x[0]]
        return max(c, key=lambda x: x[1]) if c else None

    enc, rep = pick("encode_kernel"), pick("xor_kernel")
    out = {"profile_source": rel}
    if enc:
        out.update(profile_encode_kernel=enc[0], profile_encode_calls=enc[1],
                   profile_launch_ms=round(enc[2] / 1e6, 4),
                   profile_frac=round(enc_bytes_per_launch / (enc[2] * 1e-9) / 1e9 / HBM_PEAK_GBS, 4))
    if rep:
        out.update(profile_repair_kernel=rep[0], profile_repair_calls=rep[1],
                   profile_repair_launch_ms=round(rep[2] / 1e6, 4),
                   profile_repair_frac=round(rep_bytes_per_launch / (rep[2] * 1e-9) / 1e9 / HBM_PEAK_GBS, 4))
    return out


def configs4_leg(args, d: Dist, E, k, m, r) -> dict:
    """configs[4] (configs[3] at N=1): the 256-stripe batch sized to fill ONE
    GPU's HBM, split by stripe over the ranks, timed the same way."""
    import torch

    g = -(-k // r)
    torch.cuda.empty_cache()
    d.barrier()  # every rank has freed the main leg before free HBM is read
    pl = plan(args, d, torch.cuda.mem_get_info(d.dev)[0], m + g, fill=True)
    leg = device_leg(args, d, E, pl, k, m, r, args.configs4_steps, 1, args.layout)
    vres = verify(args, leg["slab"], leg["out"], pl, k, m, r)
    ok = d.reduce(1.0 if vres["ok"] else 0.0, "min") > 0.5
    sh, S_total = pl["share"], pl["stripes_total"]
    total_bytes = (leg["enc_bytes"] + leg["rep_bytes"]) * S_total // sh["stripes"] * args.configs4_steps
    launches = leg["slab"].encode_launches()
    res = {
        "baseline_config": "configs[4]" if d.world > 1 else "configs[3]",
        "workload": workload_of(pl, k, m, r, g, d.world),
        "value": round(total_bytes / leg["el_max"] / 1e9, 2), "unit": "GB/s",
        "ms_per_step": round(leg["el_max"] / args.configs4_steps * 1e3, 4), "steps": args.configs4_steps,
        "scaling": "strong", "stripes_total": S_total, "stripes_per_gpu": sh["stripes"],
        "block_bytes": pl["block_bytes_full"],
        "rank_ms_per_step": [round(x / args.configs4_steps * 1e3, 4) for x in leg["rank_s"]],
        "encode_GBps": round(leg["enc_bytes"] / (leg["enc_ms_max"] * 1e-3) / 1e9, 2),
        "repair_GBps": round(leg["rep_bytes"] / (leg["rep_ms_max"] * 1e-3) / 1e9, 2),
        "encode_frac": round(leg["enc_bytes"] / (leg["enc_ms_max"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "encode_launch_ms": round(leg["enc_ms_max"] / launches, 4), "launches_per_encode": launches,
        "verified": bool(ok),
        "verify": {key: vres[key] for key in ("windows", "repairs")} | ({"failed": vres["failed"]} if not vres["ok"] else {}),
    }
    del leg
    torch.cuda.empty_cache()
    return res


# The other single-GPU BASELINE shapes, each its own timed leg of the line (weak:
# the stripes are per GPU), stripe 0 pinned by the committed full-size digests
# of the same shape and seed (tests/golden/manifest.json).
SHAPE_LEGS = [
    # name, BASELINE config, k, m, r, block MiB, stripes per GPU, seed (= manifest entry)
    ("configs1", "configs[1]: (k=32, 4 local groups, 2 global parities), 16 MiB/block", 32, 2, 8, 16, 32, 102),
    ("configs0_shape", "configs[0]'s default ECWide-C/config/scheme.ini shape (CL k=32, groupDataNum=11, "
                      "globalParityNum=3, chunkSizeBits=26) on the device", 32, 3, 11, 64, 8, 101),
]


def shape_leg(args, d: Dist, E, leg_def) -> dict:
    """One SHAPE_LEGS entry: fill, time `--shape-steps` steps (encode of the
    slab + repair of D0 of every stripe) exactly as the main leg, verify
    (oracle windows, every repair, stripe 0 vs the digests)."""
    import torch

    name, desc, k, m, r, mib, stripes, seed = leg_def
    a = argparse.Namespace(**vars(args))
    a.k, a.m, a.r, a.block_mib, a.stripes, a.seed, a.strong = k, m, r, float(mib), stripes, seed, False
    g = -(-k // r)
    torch.cuda.empty_cache()
    pl = plan(a, d, 0, m + g)
    leg = device_leg(a, d, E, pl, k, m, r, args.shape_steps, 2, args.layout)
    vres = verify(a, leg["slab"], leg["out"], pl, k, m, r)
    ok = d.reduce(1.0 if vres["ok"] else 0.0, "min") > 0.5
    sh = pl["share"]
    total_bytes = (leg["enc_bytes"] + leg["rep_bytes"]) * pl["stripes_total"] // sh["stripes"] * args.shape_steps
    launches = leg["slab"].encode_launches()
    enc = leg["enc_bytes"] / (leg["enc_ms_max"] * 1e-3) / 1e9
    rep = leg["rep_bytes"] / (leg["rep_ms_max"] * 1e-3) / 1e9
    res = {
        "baseline_config": desc,
        "workload": workload_of(pl, k, m, r, g, d.world) + f", seed {seed}",
        "value": round(total_bytes / leg["el_max"] / 1e9, 2), "unit": "GB/s",
        "ms_per_step": round(leg["el_max"] / args.shape_steps * 1e3, 4), "steps": args.shape_steps,
        "scaling": "weak", "stripes_per_gpu": sh["stripes"], "block_bytes": pl["block_bytes_full"],
        "rank_ms_per_step": [round(x / args.shape_steps * 1e3, 4) for x in leg["rank_s"]],
        "encode_GBps": round(enc, 2), "repair_GBps": round(rep, 2),
        "encode_frac": round(enc / HBM_PEAK_GBS, 4), "repair_frac": round(rep / HBM_PEAK_GBS, 4),
        "encode_launch_ms": round(leg["enc_ms_max"] / launches, 4), "launches_per_encode": launches,
        "verified": bool(ok),
        "verify": {key: vres[key] for key in ("windows", "repairs", "digests")}
        | ({"digest_entry": vres["digest_entry"]} if "digest_entry" in vres else {})
        | ({"failed": vres["failed"]} if not vres["ok"] else {}),
    }
    del leg
    torch.cuda.empty_cache()
    return res


def shape_cpu_baseline(args, leg_def) -> dict:
    """A SHAPE_LEGS entry's CPU baseline: one whole stripe of that shape through
    the same encodeData + decodeData flow as the headline's, on the family
    ISA-L master picks here (ECWide-C as built) and on 2.14's AVX2, 1 thread
    and the box's per-GPU share."""
    from ecwide_amd.shard import host_threads

    import oracle

    name, desc, k, m, r, mib, stripes, seed = leg_def
    master = oracle.Oracle().isal_master_kind()
    allc = host_threads()
    res, ok = cpu_stripe(args, k, m, r, int(mib) << 20, sorted({1, allc}), args.cpu_seconds / 3, seed=seed,
                         kind=master)
    r2, ok2 = cpu_stripe(args, k, m, r, int(mib) << 20, sorted({1, allc}), args.cpu_seconds / 4, seed=seed,
                         kind="avx2")
    return {"value": res[1], "unit": "GB/s", "cores": 1, "kind": "port", "isal_family": master,
            "value_all_cores": res[allc], "value_avx2": r2[1], "value_avx2_all_cores": r2[allc],
            "cores_all": allc, "verified": bool(ok and ok2),
            "sample": f"1 whole stripe of CL(k={k},r={r},m={m}) B={mib} MiB: encodeData flow + decodeData of D0"}


def main_leg(args, d: Dist, E, ctx: dict) -> dict:
    """The headline leg: this rank's share of the metric's workload, timed,
    verified; returns the line's main fields (ctx keeps the slab for the
    other_layout leg)."""
    import torch

    k, m, r = args.k, args.m, args.r
    g = -(-k // r)
    pl = plan(args, d, torch.cuda.mem_get_info(d.dev)[0], m + g, fill=args.hbm_fill)
    leg = device_leg(args, d, E, pl, k, m, r, args.steps, args.warmup, args.layout)
    slab, out = leg["slab"], leg["out"]
    enc_bytes, rep_bytes = leg["enc_bytes"], leg["rep_bytes"]
    sh = pl["share"]
    B, S = sh["block_bytes"], sh["stripes"]
    vres = None
    if args.verify:
        vres = verify(args, slab, out, pl, k, m, r)
        ok_all = d.reduce(1.0 if vres["ok"] else 0.0, "min") > 0.5
    # every stripe costs the same bytes; in column mode each stripe's bytes are
    # spread over the ranks in proportion to their column slices
    total_bytes = (enc_bytes + rep_bytes) * pl["block_bytes_full"] // B // S * pl["stripes_total"] * args.steps
    value = total_bytes / leg["el_max"] / 1e9
    launches = slab.encode_launches()  # one encode() = `launches` equal kernel launches
    # the slowest rank's kernel times: a per-GPU roofline that holds for every GPU
    enc_ms, rep_ms = leg["enc_ms_max"], leg["rep_ms_max"]
    achieved = enc_bytes / (enc_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(args, k, r, m, B, S, enc_bytes, launches)
    fields = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": d.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(leg["el_max"] / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if pl["strong"] else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (counter PRNG of include/ecwide.h, uniform random bytes, generated in HBM)",
        "config": config_of(args, pl, k, m, r, g, d.world, enc_bytes, rep_bytes),
        "rank_ms_per_step": [round(x / args.steps * 1e3, 4) for x in leg["rank_s"]],
        "devices_distinct": d.distinct,
        "encode_GBps": round(achieved, 2),
        "repair_GBps": round(rep_bytes / (rep_ms * 1e-3) / 1e9, 2),
        "roofline": {
            "bound": "hbm",
            "kernel": "encode_kernel_asm (ecwide_amd/csrc/ecw_kernels.hip + ecw_encode_asm.hpp)",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "per_gpu": "the slowest rank's launch time" if d.world > 1 else "one GPU",
            # PMC-measured HBM bytes of one launch over this run's launch time
            "traffic_GBps": round(traffic * launches / (enc_ms * 1e-3) / 1e9, 2) if traffic else None,
            # per kernel launch (rocprof's unit); one encode() of the slab = `launches` launches
            "launch_ms": round(enc_ms / launches, 4),
            # every rank's own encode launch time (a slow GPU shows here; launch_ms is their max)
            "rank_launch_ms": [round(x / launches, 4) for x in leg["rank_enc_ms"]],
            "algorithmic_bytes_per_launch": enc_bytes // launches,
            "launches_per_encode": launches,
            "encode_call_ms": round(enc_ms, 4),
            "repair_launch_ms": round(rep_ms, 4),
            "repair_algorithmic_bytes_per_launch": rep_bytes,
            "repair_frac": round(rep_bytes / (rep_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            **profile_fracs(args, enc_bytes // launches, rep_bytes),
        },
        "cpu_baseline": None,
    }
    if vres is not None:
        fields["verified"] = bool(ok_all)
        fields["verify"] = {key: vres[key] for key in ("windows", "repairs", "digests")} | (
            {"failed": vres["failed"]} if not vres["ok"] else {})
    ctx.update(codec=leg["codec"], slab=slab, out=out, S=S, B=B, enc_bytes=enc_bytes, rep_bytes=rep_bytes,
               hbm_fill=pl["hbm_fill"])
    return fields


METRIC = "device-resident encode + single-block-repair GB/s, wide stripe (shards in HBM)"

# Legs of one run, in order; all but `main` are optional (time budget) and none
# can take the line down with it (Dist.run_leg). cpu_baseline and
# chunk_generator run on rank 0 alone.
LEG_NAMES = ("main", "other_layout", "configs4", "configs1", "configs0_shape", "host_resident", "cpu_baseline",
             "chunk_generator")


def leg_estimates(args, world: int) -> dict:
    """Seconds each optional leg takes on an MI355X box (the round-5/6 driver
    lines' leg_seconds, rounded up): what the time budget checks before it
    starts a leg."""
    c = max(0.0, args.cpu_seconds)
    return {
        "other_layout": 25.0 if world == 1 else 0.0,
        "configs4": 40.0,            # fill + time + verify a ~280 GB slab
        "configs1": 12.0, "configs0_shape": 12.0,
        "host_resident": 25.0 + 3.0 * world,  # pinned NUMA-local staging of 8.6 GiB per rank
        "cpu_baseline": (5.5 * c + 10.0) if world == 1 else 0.0,  # r06a: 65.7 s at --cpu-seconds 12
        "chunk_generator": 20.0 + (c / 4 if world == 1 else 0.0),
    }


def run_legs(args, d: Dist, line: Line) -> int:
    """Every leg of the run through Dist.run_leg; the line is filled as they
    finish. Returns the exit code: 0 when the main leg measured `value`."""
    est = leg_estimates(args, d.world)
    startup = round(time.time() - T_START, 1)
    enabled = {
        "other_layout": (d.world == 1 and args.other_layout_steps > 0 and args.other_layout_rounds > 0
                         and not args.hbm_fill and not d.dry),
        "configs4": args.configs4_steps > 0 and not args.hbm_fill,
        "configs1": args.shape_steps > 0 and not args.hbm_fill and not args.strong,
        "configs0_shape": args.shape_steps > 0 and not args.hbm_fill and not args.strong,
        "host_resident": args.host_iters > 0,
        "cpu_baseline": args.cpu_seconds > 0 and d.world == 1,
        "chunk_generator": args.host_iters > 0,
    }
    line.expected = [x for x in LEG_NAMES if x != "main" and enabled.get(x)
                     and (d.rank == 0 or x not in ("cpu_baseline", "chunk_generator"))]
    # the line's frame from the start, so a line cut off inside the main leg still says what it is
    line.update(metric=METRIC, value=None, unit="GB/s", n_gpus=d.world)
    E = None
    if not d.dry:
        import ecwide_amd as E
    ctx = {}
    res, info = d.run_leg("main", (lambda: dry_main(args, d)) if d.dry else (lambda: main_leg(args, d, E, ctx)))
    rc = 0
    if info is None:
        line.update(**res)
    else:
        rc = 1
        line.update(metric=METRIC, value=None, unit="GB/s", n_gpus=d.world, main_error=info)
    line.update(budget={
        "budget_s": args.budget_s, "deadline_s": args.deadline_s, "collective_timeout_s": args.collective_timeout,
        "startup_s": startup, "estimate_s": {x: est[x] for x in est if enabled[x]},
        "estimated_total_s": round(startup + 20.0 + sum(est[x] for x in est if enabled[x]), 1)})
    if enabled["other_layout"] and ctx:
        c = ctx
        line.set_leg("other_layout", *d.run_leg(
            "other_layout", lambda: other_layouts(args, E, c["codec"], c["slab"], c["S"], c["B"], c["out"],
                                                  c["enc_bytes"], c["rep_bytes"], d.dev), est["other_layout"]))
    ctx.clear()
    d._free_device()
    k, m, r = args.k, args.m, args.r
    if enabled["configs4"]:
        line.set_leg("configs4", *d.run_leg("configs4", (lambda: dry_configs4(args, d)) if d.dry else
                                            (lambda: configs4_leg(args, d, E, k, m, r)), est["configs4"]))
    for leg_def in SHAPE_LEGS:
        name = leg_def[0]
        if enabled[name]:
            line.set_leg(name, *d.run_leg(name, (lambda: dry_shape(args, d, leg_def)) if d.dry else
                                          (lambda: shape_leg(args, d, E, leg_def)), est[name]))
    if enabled["host_resident"]:
        # every rank at once: the node's PCIe links and host DRAM together (after
        # every rank's device-resident legs: run_leg's closing sync)
        line.set_leg("host_resident", *d.run_leg(
            "host_resident", (lambda: dry_host(args, d)) if d.dry else
            (lambda: host_resident_leg(args, d, args.host_iters)), est["host_resident"]))
    if d.rank == 0:
        # rank 0 alone, no collectives: the CPU baselines (N = 1: a bounded sample
        # of each workload on this host's cores) and the ChunkGenerator replay
        if enabled["cpu_baseline"]:
            def cpu_all():
                res = {"headline": cpu_baseline(args, k, m, r, int((args.block_mib or 64.0) * (1 << 20)))}
                for leg_def in SHAPE_LEGS:
                    if enabled[leg_def[0]]:
                        res[leg_def[0]] = shape_cpu_baseline(args, leg_def)
                return res

            res, info = d.run_leg("cpu_baseline", (lambda: {"headline": {"dry_run": True}}) if d.dry else cpu_all,
                                  est["cpu_baseline"], local=True)
            if info is not None:
                line.set_leg("cpu_baseline", None, info)
            else:
                line.update(cpu_baseline=res.pop("headline"))
                with line.lock:
                    for name, cb in res.items():
                        if isinstance(line.data.get(name), dict) and "error" not in line.data[name]:
                            line.data[name] = dict(line.data[name], cpu_baseline=cb)
        elif args.cpu_seconds > 0:
            line.update(cpu_baseline_note="measured at N = 1 only (BENCH); the same host CPU path at every N")
        if enabled["chunk_generator"]:
            cs = args.cpu_seconds / 4 if enabled["cpu_baseline"] else 0.0
            line.set_leg("chunk_generator", *d.run_leg(
                "chunk_generator", (lambda: {"dry_run": True}) if d.dry else (lambda: chunkgen_leg(args, cs)),
                est["chunk_generator"], local=True))
    return rc


def main():
    argv = sys.argv[1:]
    args = parse(argv)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # decide before anything touches the GPU; the ranks are fresh processes
        sys.exit(spawn_ranks(args.gpus, argv))
    if args.host_resident:
        host_resident(args)
        return
    if args.small_calls:
        small_calls(args)
        return
    DRY_SLOW[0] = args.dry_run_slow
    d = Dist(args)
    line = Line(d, args.deadline_s, args.collective_timeout)
    rc = 1
    try:
        rc = run_legs(args, d, line)
    except BaseException as e:  # noqa: BLE001 -- the line goes out whatever happened
        line.update(error=f"{type(e).__name__}: {e}"[:600])
        raise
    finally:
        line.emit()
        d.close()
    sys.exit(rc)


if __name__ == "__main__":
    main()

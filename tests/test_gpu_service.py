"""The small-stripe request service (ecw_codec.cpp svc::, ecw_kernels.hip
service_kernel): synchronous small host-memory encodes served by a resident
kernel polling pinned memory — ECWide-H's one-4 KiB-chunk-per-call pattern
(ECWide-H/proxy/encode.cpp:145-175). Bit-exact vs the oracle for every code
shape it takes, from many threads at once, across its idle exit and relaunch,
and the process leaves cleanly right after a call."""
import os
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

from conftest import REPO, golden_blocks

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def E():
    import torch

    assert torch.cuda.is_available()
    import ecwide_amd

    return ecwide_amd


@pytest.mark.parametrize("code,k,m,r,ln,literal", [
    ("R", 11, 3, 0, 4096, False),        # ECWide-H g_encode
    ("C", 32, 3, 11, 4096, False),       # default scheme.ini shape, XOR locals
    ("C", 32, 3, 11, 4096 + 37, True),   # ragged length, ECWide-C literal zero locals
    ("C", 20, 6, 4, 3 * 4096 + 16, False),  # 5-8 global rows (u64 tables)
    ("C", 200, 3, 40, 8192, False),      # > 16 rows per lane round
    ("R", 5, 1, 0, 1, False),            # one byte
    ("C", 128, 3, 27, 64 << 10, False),  # the service's largest block
])
def test_service_encode_vs_oracle(E, orc, code, k, m, r, ln, literal):
    if code == "R":
        c = E.NativeCodec.getRsCodec(E.CodingScheme.getRsScheme(k, m, ln))
    else:
        c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, ln), 1, False,
                                     local_mode="literal" if literal else "xor")
    oc = orc.codec(code, k, m, r if r else k, ln)
    for rep in range(3):
        data = [orc.fill(ln, 900 + rep, rep, j) for j in range(k)]
        par = [np.full(ln, 0xA5, np.uint8) for _ in range(c.parityNum)]
        c.encodeData(data, par)
        want = oc.encode(data, literal=literal)
        for i, w in enumerate(want):
            assert np.array_equal(par[i], w), (rep, i)


def test_service_golden_g_encode(E, orc, manifest):
    """The ECWide-H g_encode golden vector through the service."""
    h = manifest["ecwide_h"]
    gd = [orc.fill(4096, 42, 0, j) for j in range(11)]
    c = E.NativeCodec.getRsCodec(E.CodingScheme.getRsScheme(11, 3, 4096))
    par = [np.zeros(4096, np.uint8) for _ in range(3)]
    c.encodeData(gd, par)
    assert all(np.array_equal(a, b) for a, b in zip(par, golden_blocks(h["g_encode"], 3, 4096)))


def test_service_many_threads_and_idle_relaunch(E, orc):
    """20 threads (more than the 16 slots) x 40 calls on two codecs; then an
    idle gap longer than the service's idle exit, and more calls (relaunch)."""
    codecs = [(E.NativeCodec.getRsCodec(E.CodingScheme.getRsScheme(11, 3, 4096)), orc.codec("R", 11, 3, 11, 4096)),
              (E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(16, 2, 4, 4096), 1, False),
               orc.codec("C", 16, 2, 4, 4096))]
    errors = []

    def worker(t):
        c, oc = codecs[t % 2]
        for n in range(40):
            data = [orc.fill(4096, t, n, j) for j in range(c.encodeDataNum)]
            par = [np.zeros(4096, np.uint8) for _ in range(c.parityNum)]
            c.encodeData(data, par)
            if not all(np.array_equal(a, b) for a, b in zip(par, oc.encode(data))):
                errors.append((t, n))

    for phase in range(2):
        th = [threading.Thread(target=worker, args=(t,)) for t in range(20)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errors, errors[:5]
        time.sleep(0.2)  # > the 20 ms idle exit: the next phase relaunches the service


def test_service_then_device_sync_and_clean_exit(E, orc):
    """A device synchronize right after service calls returns (the resident
    kernel leaves when idle), and a process that exits right after a call
    leaves cleanly (the service is stopped before the runtime goes)."""
    import torch

    c = E.NativeCodec.getRsCodec(E.CodingScheme.getRsScheme(11, 3, 4096))
    data = [orc.fill(4096, 1, 0, j) for j in range(11)]
    par = [np.zeros(4096, np.uint8) for _ in range(3)]
    c.encodeData(data, par)
    t = time.perf_counter()
    torch.cuda.synchronize()
    assert time.perf_counter() - t < 5.0
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import numpy as np, ecwide_amd as E\n"
            "c = E.NativeCodec.getRsCodec(E.CodingScheme.getRsScheme(11, 3, 4096))\n"
            "d = [np.full(4096, j, np.uint8) for j in range(11)]; p = [np.zeros(4096, np.uint8) for _ in range(3)]\n"
            "c.encodeData(d, p); print('ok', int(p[0].sum()))\n") % REPO
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and p.stdout.startswith("ok"), p.stderr[-2000:]


def test_service_alternating_shapes_one_slot(E, orc):
    """One thread (one slot) alternating codecs and lengths call after call:
    the request words change generation every call, and the number of parts
    with work swings between 1 and 8, so parts that sat out a request (and may
    not have seen it yet) must take the next one whole."""
    rs = (E.NativeCodec.getRsCodec(E.CodingScheme.getRsScheme(11, 3, 65536)), orc.codec("R", 11, 3, 11, 65536))
    cl = (E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(24, 2, 5, 65536), 1, False),
          orc.codec("C", 24, 2, 5, 65536))
    for n, ln in enumerate([65536, 1, 40000, 17, 1024, 65536, 3 * 1024 + 5, 1, 65536]):
        for c, oc in (rs, cl):
            data = [orc.fill(ln, 700 + n, 0, j) for j in range(c.encodeDataNum)]
            par = [np.full(ln, 0x3C, np.uint8) for _ in range(c.parityNum)]
            c.encodeData(data, par)
            for i, w in enumerate(oc.encode(data)):
                assert np.array_equal(par[i], w[:ln]), (n, ln, i)


def test_service_exit_after_every_request(E):
    """ECW_SERVICE_IDLE_MS=0: the resident kernel leaves at its first idle
    check after every request, so calls keep racing its exit and relaunch
    (a request posted while the epoch leaves is served by the next one).
    Runs in a child process (the setting is read once per process)."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import numpy as np, ecwide_amd as E, oracle\n"
            "orc = oracle.Oracle()\n"
            "c = E.NativeCodec.getRsCodec(E.CodingScheme.getRsScheme(11, 3, 8192))\n"
            "oc = orc.codec('R', 11, 3, 11, 8192)\n"
            "for n in range(300):\n"
            "    ln = (4096, 8192, 100)[n %% 3]\n"
            "    d = [orc.fill(ln, 50 + n, 0, j) for j in range(11)]\n"
            "    p = [np.zeros(ln, np.uint8) for _ in range(3)]\n"
            "    c.encodeData(d, p)\n"
            "    assert all(np.array_equal(a, b) for a, b in zip(p, oc.encode(d))), n\n"
            "print('ok')\n") % REPO
    env = dict(os.environ, ECW_SERVICE_IDLE_MS="0")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180, env=env)
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), p.stderr[-2000:]


@pytest.mark.parametrize("k", [11, 4, 5])
def test_service_xor_row_matrix_codec(E, orc, k):
    """ECWide-H's l_encode / l_middle / l_decode (k = 11 / 4 / 5): one all-ones
    row through ecw_matrix_codec_create (as the ISA-L shim builds it) takes
    the service's plain-XOR path; ragged and unit-straddling lengths."""
    import ctypes

    from ecwide_amd import _lib

    L = _lib.load()
    ones = np.ones(k, np.uint8)
    h = ctypes.c_void_p()
    assert L.ecw_matrix_codec_create(ones.ctypes.data_as(_lib._u8p), k, 1, 0, ctypes.byref(h)) == 0
    try:
        for n, ln in enumerate([1, 100, 4096, 5000, 3 * 1024 + 7, 65536]):
            d = [orc.fill(ln, 300 + n, 0, j) for j in range(k)]
            p = np.full(ln, 0x77, np.uint8)
            dp = (ctypes.c_void_p * k)(*[x.ctypes.data for x in d])
            pp = (ctypes.c_void_p * 1)(p.ctypes.data)
            assert L.ecw_encode(h, dp, pp, ln) == 0
            assert np.array_equal(p, orc.xor_blocks(d)), (k, ln)
    finally:
        L.ecw_codec_destroy(h)


def test_codec_lifetime_beside_busy_service(E, orc):
    """VERDICT r02 item 5 (ECWide-H's concurrent codec threads,
    ECWide-H/proxy/proxy.cpp:2009-2012): while 4 threads keep the resident
    request service busy with 4 KiB calls, a fifth thread 20 times creates a
    codec, runs two launch-path encodes of host blocks larger than the
    service takes (the second grows the codec's HBM staging) and destroys the
    codec. Freeing device or pinned memory can wait for the device to go idle,
    which it does not while the service runs: growth and teardown defer their
    frees instead, so every grow returns within 50 ms of its own transfer time
    and every destroy within 50 ms, and all outputs are bit-exact."""
    rs = E.NativeCodec.getRsCodec(E.CodingScheme.getRsScheme(11, 3, 4096))
    ors = orc.codec("R", 11, 3, 11, 4096)
    stop = threading.Event()
    errors, calls = [], [0] * 4

    def small(t):
        data = [orc.fill(4096, 70 + t, 0, j) for j in range(11)]
        want = ors.encode(data)
        par = [np.zeros(4096, np.uint8) for _ in range(3)]
        while not stop.is_set():
            rs.encodeData(data, par)
            calls[t] += 1
            if not all(np.array_equal(a, b) for a, b in zip(par, want)):
                errors.append(("small", t))
                return

    th = [threading.Thread(target=small, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    k, m, r = 16, 2, 4
    grow_s, destroy_s, rates = [], [], []
    try:
        time.sleep(0.05)  # the service is up and busy
        for it in range(20):
            c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, 4 << 20), 1, False)
            oc = orc.codec("C", k, m, r, 4 << 20)
            for ln in (1 << 20, 4 << 20):  # > 64 KiB: the launch path; the second call grows the staging
                data = [orc.fill(ln, 90 + it, 0, j) for j in range(k)]
                par = [np.zeros(ln, np.uint8) for _ in range(c.parityNum)]
                t0 = time.perf_counter()
                c.encodeData(data, par, ln)
                el = time.perf_counter() - t0
                if ln > 1 << 20:
                    grow_s.append(el)
                    rates.append((k + c.parityNum) * ln / el / 1e9)
                want = orc.codec("C", k, m, r, ln).encode(data) if ln != 4 << 20 else oc.encode(data)
                if not all(np.array_equal(a, b) for a, b in zip(par, want)):
                    errors.append(("bulk", it, ln))
            t0 = time.perf_counter()
            del c  # ecw_codec_destroy
            destroy_s.append(time.perf_counter() - t0)
    finally:
        stop.set()
        for x in th:
            x.join()
    assert not errors, errors[:5]
    assert min(calls) > 0
    transfer = (k + 6) * (4 << 20) / 20e9  # the grow call's own copies at >= 20 GB/s
    print(f"\nlifetime beside the service: grow {max(grow_s) * 1e3:.1f} ms max, destroy {max(destroy_s) * 1e3:.2f} "
          f"ms max, bulk encode {np.median(rates):.1f} GB/s (median) with {sum(calls)} service calls")
    assert max(destroy_s) < 0.05, destroy_s
    assert max(grow_s) < 0.05 + transfer, grow_s


def test_service_restages_tables_of_a_recreated_codec(E, orc):
    """the service keeps a codec's tables staged in LDS while the
    next request uses the same codec. A codec destroyed and recreated with the
    same shape but another matrix can get the same device table address, so
    the cache is keyed by a per-codec serial: every recreated codec's parities
    must follow its own matrix."""
    import ctypes

    from ecwide_amd import _lib

    L = _lib.load()
    k, rows, ln = 11, 3, 4096
    rng = np.random.default_rng(5)
    data = [orc.fill(ln, 77, 0, j) for j in range(k)]
    dp = (ctypes.c_void_p * k)(*[x.ctypes.data for x in data])
    for it in range(12):
        mat = rng.integers(1, 256, k * rows, dtype=np.uint8)
        h = ctypes.c_void_p()
        assert L.ecw_matrix_codec_create(mat.ctypes.data_as(_lib._u8p), k, rows, 0, ctypes.byref(h)) == 0
        try:
            par = [np.zeros(ln, np.uint8) for _ in range(rows)]
            pp = (ctypes.c_void_p * rows)(*[x.ctypes.data for x in par])
            for _ in range(3):  # the service keeps this codec's tables between calls
                assert L.ecw_encode(h, dp, pp, ln) == 0
            want = orc.encode_data(orc.init_tables(k, rows, mat), data, rows)
            for i, w in enumerate(want):
                assert np.array_equal(par[i], w), (it, i)
        finally:
            L.ecw_codec_destroy(h)


def test_service_small_host_xors_vs_oracle(E, orc):
    """decodeData / partialDecodeData / repairBlock / xorIntemediate on host
    blocks up to 64 KiB are plain XORs served by the resident service (no
    launch, no tables staged): bit-exact at ragged lengths, interleaved with
    encodes of the same codec (whose tables the XOR requests leave staged in
    LDS), and counted as served."""
    k, m, r = 32, 2, 8
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, 65536), 1, False)
    oc = orc.codec("C", k, m, r, 65536)
    before = E.service_counters(c.device)
    calls = 0
    for n, ln in enumerate([4096, 1, 100, 5000, 3 * 1024 + 7, 65536]):
        data = [orc.fill(ln, 400 + n, 0, j) for j in range(k)]
        par = [np.full(ln, 0x5A, np.uint8) for _ in range(c.parityNum)]
        c.encodeData(data, par)
        want_par = orc.codec("C", k, m, r, ln).encode(data) if ln != 65536 else oc.encode(data)
        assert all(np.array_equal(a, b) for a, b in zip(par, want_par)), (n, "encode")
        ddn, pdn = c.decodeDataNum, c.partialDecodeNum
        t = np.full(ln, 0x11, np.uint8)
        c.decodeData(data[:ddn], t)
        assert np.array_equal(t, orc.xor_blocks(data[:ddn])), (n, "decode")
        t = np.full(ln, 0x22, np.uint8)
        c.partialDecodeData(data[1:1 + pdn], t)
        assert np.array_equal(t, orc.xor_blocks(data[1:1 + pdn])), (n, "partial")
        blocks = data + par
        out = np.zeros(ln, np.uint8)
        c.repairBlock(blocks, 0, out)
        assert np.array_equal(out, data[0]), (n, "repair")
        tgt = [np.array(p) for p in par[:m]]
        c.xorIntemediate(par[:m], tgt)
        assert all(not t.any() for t in tgt), (n, "xorIntemediate")  # p ^ p
        calls += 3 + m  # decode, partial decode, repair, m xorIntemediate XORs
    after = E.service_counters(c.device)
    assert not after["broken"]
    assert after["served"] - before["served"] >= calls, (before, after)


def test_service_not_stranded_by_bulk_holds(E, orc):
    """bulk host calls (decodeData of 2 MiB blocks) hold the
    service off while they run. A small request posted to an epoch that a
    bulk call asked to leave must take the launch path at once, not spin
    until every hold has ended (10 s, then the service was turned off for
    good). Two threads keep holds overlapping back to back while a third makes
    small encodes: every small call returns within 1 s, every byte is exact,
    and once the bulk calls stop the service serves again."""
    rs = E.NativeCodec.getRsCodec(E.CodingScheme.getRsScheme(11, 3, 4096))
    ors = orc.codec("R", 11, 3, 11, 4096)
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(32, 2, 8, 2 << 20), 1, False)
    ddn = c.decodeDataNum
    stop = threading.Event()
    errors, lat = [], []

    def bulk(t):
        data = [orc.fill(2 << 20, 600 + t, 0, j) for j in range(ddn)]
        want = orc.xor_blocks(data)
        out = np.zeros(2 << 20, np.uint8)
        while not stop.is_set():
            c.decodeData(data, out)
            if not np.array_equal(out, want):
                errors.append(("bulk", t))
                return

    # every small call encodes different data (a rotation of 16
    # inputs, each against its own oracle output) into zeroed outputs, so a
    # call handed an earlier request's results -- e.g. by a request word that
    # aliases a withdrawn one -- fails instead of matching byte for byte
    sets = [[orc.fill(4096, 650 + i, 0, j) for j in range(11)] for i in range(16)]
    wants = [ors.encode(d) for d in sets]

    def small():
        par = [np.zeros(4096, np.uint8) for _ in range(3)]
        i = 0
        while not stop.is_set():
            data, want = sets[i % 16], wants[i % 16]
            for p in par:
                p[:] = 0
            t0 = time.perf_counter()
            rs.encodeData(data, par)
            lat.append(time.perf_counter() - t0)
            if not all(np.array_equal(a, b) for a, b in zip(par, want)):
                errors.append(("small", i))
                return
            i += 1

    th = [threading.Thread(target=bulk, args=(t,)) for t in range(2)] + [threading.Thread(target=small)]
    for x in th:
        x.start()
    time.sleep(3.0)
    stop.set()
    for x in th:
        x.join()
    assert not errors, errors[:5]
    assert lat and max(lat) < 1.0, (len(lat), max(lat) if lat else None)
    before = E.service_counters(rs.device)
    data = [orc.fill(4096, 651, 0, j) for j in range(11)]
    par = [np.zeros(4096, np.uint8) for _ in range(3)]
    for _ in range(50):
        rs.encodeData(data, par)
    after = E.service_counters(rs.device)
    print(f"\nsmall calls beside bulk holds: {len(lat)} calls, max {max(lat) * 1e3:.1f} ms; counters {after}")
    assert not after["broken"]
    assert after["served"] - before["served"] == 50, (before, after)

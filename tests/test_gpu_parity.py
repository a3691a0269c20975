"""GPU parity: the HIP path through the C ABI vs the golden vectors (made
from the reference's ISA-L arithmetic) and vs the oracle on seeded inputs;
full BASELINE sizes through committed SHA-256 digests and size-independent
properties (encode -> erase -> repair round trips, linearity)."""
import hashlib

import numpy as np
import pytest

from conftest import golden_blocks

pytestmark = pytest.mark.gpu


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def torch():
    import torch as t

    assert t.cuda.is_available()
    return t


@pytest.fixture(scope="module")
def E():
    import ecwide_amd

    return ecwide_amd


@pytest.fixture
def schedule(E):
    """The test sets the process's launch schedule (ecw_set_schedule); it is
    back to the library's own choice (all -1) afterwards."""
    E.set_schedule()
    yield
    E.set_schedule()


def make_codec(E, e, local_mode="xor"):
    t = e["code_type"]
    B = e["len"]
    if t == "C":
        s = E.CodingScheme.getClScheme(e["k"], e["m"], e["r"], B)
        return E.NativeCodec.getClCodec(s, 1, False, local_mode=local_mode)
    if t == "L":
        s = E.CodingScheme.getLrcScheme(e["k"], e["m"], e["r"], B)
        return E.NativeCodec.getLrcCodec(s, 1, local_mode=local_mode)
    if t == "T":
        return E.NativeCodec.getTlCodec(E.CodingScheme.getTlScheme(e["k"], e["m"], B), 1)
    return E.NativeCodec.getRsCodec(E.CodingScheme.getRsScheme(e["k"], e["m"], B))


def dev_blocks(torch, n, length, fill=None):
    # separate allocations, 16-B aligned (caching allocator rounds to 512 B)
    return [torch.zeros(max(length, 1), dtype=torch.uint8, device="cuda")[:length] if fill is None
            else torch.from_numpy(fill[i]).cuda() for i in range(n)]


def test_lib_loaded_from_tree(E):
    import os

    assert os.path.dirname(E.LIB_PATH).endswith("ecwide_amd")
    assert E.device_count() >= 1


def test_encode_host_api_golden(E, orc, manifest):
    """ecw_encode (host buffers) vs golden, both local modes, all configs."""
    for e in manifest["encode"]:
        data = [orc.fill(e["len"], e["seed"], 0, j) for j in range(e["k"])]
        c = make_codec(E, e)
        par = [np.zeros(e["len"], np.uint8) for _ in range(c.parityNum)]
        c.encodeData(data, par)
        want = golden_blocks(e["xor"], c.parityNum, e["len"])
        for i, (g, w) in enumerate(zip(par, want)):
            assert np.array_equal(g, w), (e["name"], i)
        if e["code_type"] in "CL":
            c2 = make_codec(E, e, "literal")
            par2 = [np.full(e["len"], 0xAB, np.uint8) for _ in range(c.parityNum)]
            c2.encodeData(data, par2)
            assert [sha(x) for x in par2] == e["literal_sha256"], e["name"]


def test_encode_device_api_golden(E, torch, orc, manifest):
    """ecw_encode_dev (HBM pointers, separate allocations) vs golden."""
    for e in manifest["encode"]:
        data = [orc.fill(e["len"], e["seed"], 0, j) for j in range(e["k"])]
        c = make_codec(E, e)
        d = dev_blocks(torch, e["k"], e["len"], data)
        p = dev_blocks(torch, c.parityNum, e["len"])
        c.encodeData(d, p)
        torch.cuda.synchronize()
        want = golden_blocks(e["xor"], c.parityNum, e["len"])
        for i, (g, w) in enumerate(zip(p, want)):
            assert np.array_equal(g.cpu().numpy(), w), (e["name"], i)


@pytest.mark.parametrize("layout", ["strided", "reversed"])
def test_encode_device_api_layouts(E, torch, orc, layout):
    """ecw_encode_dev with every block in one buffer: at one stride (taken as a
    one-stripe slab -> the asm tile) and in reverse order (pointer kernel);
    both against the oracle, at shapes with full tiles and a ragged tail."""
    for k, m, r, B in [(32, 3, 11, 3 * 4096 + 48), (128, 3, 27, 1 << 16), (9, 2, 3, 8192)]:
        c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
        np_ = c.parityNum
        stride = (B + 255) // 256 * 256 + 4096
        dbuf = torch.zeros((k, stride), dtype=torch.uint8, device="cuda")
        pbuf = torch.full((np_, stride), 0x5A, dtype=torch.uint8, device="cuda")
        data = [orc.fill(B, 17, 0, j) for j in range(k)]
        for j in range(k):
            dbuf[j, :B].copy_(torch.from_numpy(data[j]))
        drows = [dbuf[j, :B] for j in range(k)]
        prows = [pbuf[i, :B] for i in range(np_)]
        if layout == "reversed":
            order = list(range(k))[::-1]
            for j in range(k):
                dbuf[order[j], :B].copy_(torch.from_numpy(data[j]))
            drows = [dbuf[order[j], :B] for j in range(k)]
            prows = prows[::-1]
        c.encodeData(drows, prows)
        torch.cuda.synchronize()
        want = orc.codec("C", k, m, r, B).encode(data, threads=8)
        for i in range(np_):
            assert np.array_equal(prows[i].cpu().numpy(), want[i]), (layout, k, i)
        assert not pbuf[:, B:].ne(0x5A).any(), "wrote past the block"


def test_column_slices_match_full_encode(E, torch, orc):
    """SURVEY §8e fallback: each "rank" encodes its column_shard slice of
    every block (device pointers into the same blocks); together the slices
    equal the whole-block encode, ragged last slice included."""
    from ecwide_amd.shard import column_shard

    k, m, r, B = 32, 3, 11, 5 * 4096 + 200
    data = [orc.fill(B, 23, 0, j) for j in range(k)]
    want = orc.codec("C", k, m, r, B).encode(data, threads=8)
    stride = (B + 255) // 256 * 256  # device pointers must be 16-byte aligned
    dbuf = torch.zeros((k, stride), dtype=torch.uint8, device="cuda")
    for j in range(k):
        dbuf[j, :B].copy_(torch.from_numpy(data[j]))
    for world in (2, 3, 8):
        pbuf = torch.zeros((len(want), stride), dtype=torch.uint8, device="cuda")
        for rank in range(world):
            off, n = column_shard(B, world, rank)
            if n == 0:
                continue
            c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, n), 1, False)
            c.encodeData([dbuf[j, off:off + n] for j in range(k)], [pbuf[i, off:off + n] for i in range(len(want))])
        torch.cuda.synchronize()
        for i, w in enumerate(want):
            assert np.array_equal(pbuf[i, :B].cpu().numpy(), w), (world, i)


@pytest.mark.parametrize("k,m,r,B,S,tiled", [(128, 3, 27, 4096, 6, True), (32, 6, 8, 4096, 3, True),
                                              (20, 11, 6, 3 * 4096 + 48, 2, False), (9, 2, 3, 5000, 3, False)])
def test_split_layout_encode_vs_oracle(E, torch, orc, k, m, r, B, S, tiled):
    """ecw_encode_batch_split_dev: data and parities in separate regions. tiled:
    4 KiB stripes with contiguous columns (block stride 4096, stripe stride
    k*4096); otherwise padded strides; the padding past each block untouched."""
    from ctypes import c_void_p

    from ecwide_amd._lib import lib

    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    np_ = c.parityNum
    dbs = B if tiled else (B + 255) // 256 * 256 + 4096
    pbs = B if tiled else (B + 255) // 256 * 256 + 512
    dss, pss = k * dbs, np_ * pbs + (0 if tiled else 4096)
    data = torch.empty(S * dss, dtype=torch.uint8, device="cuda")
    par = torch.full((S * pss,), 0x5A, dtype=torch.uint8, device="cuda")
    stream = c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.ecw_fill_random_dev(0, c_void_p(data.data_ptr()), dbs, dss, S, k, B, 31, 0, 0, stream) == 0
    st = lib.ecw_encode_batch_split_dev(c._h, c_void_p(data.data_ptr()), dbs, dss, c_void_p(par.data_ptr()), pbs,
                                        pss, S, B, stream)
    assert st == 0
    torch.cuda.synchronize()
    oc = orc.codec("C", k, m, r, B)
    pn = par.cpu().numpy()
    for s in range(S):
        want = oc.encode([orc.fill(B, 31, s, j) for j in range(k)], threads=8)
        for i in range(np_):
            o = s * pss + i * pbs
            assert np.array_equal(pn[o:o + B], want[i]), (s, i)
            assert (pn[o + B:o + pbs] == 0x5A).all(), ("wrote past the block", s, i)


@pytest.mark.parametrize("k,m,r,B,S,chunk", [(128, 3, 27, 1 << 16, 2, 8192), (32, 6, 8, 4 * 4096, 2, 4096),
                                              (20, 2, 5, 3 * 8192, 3, 8192),
                                              (32, 2, 8, 4 * 16384, 3, 16384)])  # k <= 32 default: K = 4 repair groups
def test_tiled_slab_encode_repair(E, torch, orc, k, m, r, B, S, chunk):
    """StripeSlab(layout="tiled"): every (stripe, piece) unit vs the oracle, and
    the split-layout repair of every D and L block rebuilds it exactly."""
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    slab = E.StripeSlab(c, stripes=S, block_bytes=B, layout="tiled", chunk=chunk)
    slab.fill_random(seed=71)
    slab.encode()
    torch.cuda.synchronize()
    oc = orc.codec("C", k, m, r, chunk)
    for s in range(S):
        data = [slab.block(s, j).cpu().numpy() for j in range(k)]
        par = [p.cpu().numpy() for p in slab.parity(s)]
        for piece in range(slab.pieces):
            sl = slice(piece * chunk, (piece + 1) * chunk)
            assert np.array_equal(data[0][sl], orc.fill(chunk, 71, s, 0, piece * chunk))
            want = oc.encode([d[sl] for d in data])
            for i, w in enumerate(want):
                assert np.array_equal(par[i][sl], w), (s, piece, i)
    out = torch.empty(S * B, dtype=torch.uint8, device="cuda")
    for lost in list(range(k)) + [k + m + t for t in range(c.groupNum)]:
        slab.repair(lost, out)
        torch.cuda.synchronize()
        for s in range(S):
            assert torch.equal(out[s * B:(s + 1) * B], slab.block(s, lost)), (lost, s)


def test_xor_every_source_count(E, torch, orc):
    """XOR reduce at every source count of the straight-line kernels (1..32)
    and past it (the ring kernel: 33, 40, 64, 129), full and ragged tiles,
    against the oracle's XOR (pointer mode)."""
    for n in list(range(1, 34)) + [40, 64, 129]:
        ln = 4096 * 2 + 16 * (n % 7) + (n % 3)  # ragged tail for most n
        data = [orc.fill(ln, 300 + n, 0, j) for j in range(n)]
        d = dev_blocks(torch, n, ln, data)
        out = torch.full((ln,), 0xA5, dtype=torch.uint8, device="cuda")
        E.xor_reduce(d, out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), orc.xor_blocks(data)), n


@pytest.mark.parametrize("layout", ["blocks", "split", "tiled"])
@pytest.mark.parametrize("k,r", [(40, 40), (64, 31), (64, 32), (70, 33), (12, 1)])
def test_repair_group_sizes(E, torch, k, r, layout):
    """CL repair of D0, the group's last block and L0 with r + 1 survivors on
    both sides of the straight-line kernel limit (32 sources), block slab
    and tiled slab."""
    B = 3 * 8192
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, 2, r, B), 1, False)
    kw = {"layout": "tiled", "chunk": 8192} if layout == "tiled" else {}
    slab = E.StripeSlab(c, stripes=2, block_bytes=B, **kw)
    slab.fill_random(seed=7 + r)
    slab.encode()
    o = B if layout == "tiled" else slab.out_stride
    out = torch.empty(2 * o, dtype=torch.uint8, device="cuda")
    for lost in (0, min(r, k) - 1, k + 2):
        slab.repair(lost, out)
        torch.cuda.synchronize()
        for s in range(2):
            assert torch.equal(out[s * o:s * o + B], slab.block(s, lost)), (lost, s)


@pytest.mark.parametrize("k,m,r,B,S,layout,local", [
    (4, 2, 2, 256 << 20, 4, "blocks", "xor"),      # 1 global row pass, parked locals
    (4, 6, 2, 256 << 20, 4, "blocks", "xor"),      # 5-8 rows: the u64-entry (NW=2) tile
    (12, 3, 2, 64 << 20, 16, "blocks", "xor"),     # 6 groups: locals not parked
    (4, 2, 2, 256 << 20, 4, "blocks", "literal"),  # ECWide-C literal mode: zero L blocks
    (8, 3, 4, 128 << 20, 8, "tiled", "xor"),       # the bench's split (tiled) layout, 262,144 tiles
])
def test_ticket_launch_matches_windows(E, torch, orc, k, m, r, B, S, layout, local):
    """A slab of >= 262,144 column tiles is encoded by one ticket-ordered
    launch (ecw_kernels.hip launch_encode); each stripe encoded on its own
    (pointer mode, < 262,144 tiles: the launch-window path) must give the same
    parities, and the last column window (claimed last by the ticket order)
    must match the oracle. A second encode of the slab on the same stream
    reuses the counter (ticket base carried over) and must give the same bytes."""
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False, local_mode=local)
    kw = {"layout": "tiled", "chunk": 8192} if layout == "tiled" else {}
    slab = E.StripeSlab(c, stripes=S, block_bytes=B, **kw)
    assert slab.encode_launches() == 1
    slab.fill_random(seed=404)
    slab.encode()
    np_ = c.parityNum
    W = 8192
    oc = orc.codec("C", k, m, r, W)
    first = [[p[-W:].clone() for p in slab.parity(s)] for s in (0, S - 1)]
    pbuf = torch.empty((np_, B), dtype=torch.uint8, device="cuda")
    for s in (0, S - 1):
        c.encodeData([slab.block(s, j) for j in range(k)], [pbuf[i] for i in range(np_)])
        torch.cuda.synchronize()
        for i, p in enumerate(slab.parity(s)):
            assert torch.equal(p, pbuf[i]), (s, i)
        want = oc.encode([orc.fill(W, 404, s, j, B - W) for j in range(k)], literal=local == "literal")
        for i, w in enumerate(want):
            assert np.array_equal(pbuf[i][B - W:].cpu().numpy(), w), (s, i)
    if layout == "tiled":
        slab.buf[slab.off + slab.parity_offset:].zero_()
    else:
        for p in slab.parity(0) + slab.parity(S - 1):
            p.zero_()
    slab.encode()  # second launch on the same counter
    torch.cuda.synchronize()
    for n, s in enumerate((0, S - 1)):
        for i, p in enumerate(slab.parity(s)):
            assert torch.equal(p[-W:], first[n][i]), ("second encode", s, i)


def test_ticket_launches_on_per_thread_streams(E, torch, orc):
    """ticket-ordered launches from two threads on
    hipStreamPerThread (one stream handle, two real streams) must not share a
    ticket counter. Each thread encodes its own 1 GiB-per-row slab (one
    ticket launch each) four times, concurrently with the other; every
    result equals the oracle on column windows of the first and last stripe
    (tiles skipped by a clobbered counter would leave their parities at the
    0xEE the slabs were poisoned with)."""
    import ctypes
    import threading

    k, m, r, B, S = 4, 2, 2, 256 << 20, 4
    per_thread = ctypes.c_void_p(2)  # hipStreamPerThread
    slabs = []
    for t in range(2):
        c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
        slab = E.StripeSlab(c, stripes=S, block_bytes=B)
        assert slab.encode_launches() == 1  # one ticket-ordered launch
        slab.fill_random(seed=600 + t)
        slabs.append(slab)
    torch.cuda.synchronize()
    errs = []

    def work(t):
        try:
            for _ in range(4):
                for s in range(S):
                    for p in slabs[t].parity(s):
                        p.fill_(0xEE)
                torch.cuda.synchronize()
                slabs[t].encode(stream=per_thread)
                torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=work, args=(t,)) for t in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs
    W = 8192
    oc = orc.codec("C", k, m, r, W)
    for t, slab in enumerate(slabs):
        for s in (0, S - 1):
            par = slab.parity(s)
            for off in (0, B // 2, B - W):
                want = oc.encode([orc.fill(W, 600 + t, s, j, off) for j in range(k)])
                for i, w in enumerate(want):
                    assert np.array_equal(par[i][off:off + W].cpu().numpy(), w), (t, s, off, i)


@pytest.mark.parametrize("k,m,r,local,layout", [
    (128, 3, 27, "xor", "blocks"),    # parked locals (the bench shape's tile); auto = on
    (128, 3, 27, "xor", "tiled"),     # the bench's 8 KiB pieces (4096 units x 2 tiles); auto = on, width 32
    (32, 3, 11, "xor", "tiled"),      # configs[0]'s 16 KiB pieces (2048 units x 4 tiles); auto = 2^10 / 32
    (32, 6, 8, "xor", "blocks"),      # 5-8 rows: the u64-entry (NW=2) tile
    (24, 2, 3, "xor", "split"),       # 8 groups: mid-tile local stores
    (16, 3, 4, "literal", "blocks"),  # zero L blocks
    (32, 3, 11, "xor", "ptr"),        # device pointer tables
    (3, 2, 2, "xor", "blocks"),       # window on = the three-slot ring: its 3-row tail only
    (4, 3, 4, "xor", "ptr"),          # 4-row tail, pointer tables
    (5, 1, 2, "xor", "split"),        # 5-row tail, 3 groups (parked locals)
    (7, 2, 1, "xor", "split"),        # main loop once + 4-row tail, 7 groups (mid-tile local stores)
    (9, 3, 3, "literal", "blocks"),   # main loop once + 3-row tail, zero L blocks
    (10, 4, 10, "xor", "blocks"),     # main loop once + 4-row tail
])
def test_write_window_same_bytes(E, torch, orc, schedule, k, m, r, local, layout):
    """The write window (ecw_kernels.hip set_schedule; ecw_set_schedule's
    enc_window_*) only delays the
    parity stores: encodes with it forced off, on, and at another period give
    identical parities, equal to the oracle on a column window, and the default
    choice ('auto': slabs and pointer modes at k >= 24 (a 2^10-tick period below k = 64),
    <= 4 global rows, blocks or tiled pieces >= 8 KiB, >= 8192 tiles) gives them too. With the window on, the <= 4-row tile keeps
    three rows in flight (ECW_TILE_ASM3): k = 3, 4, 5, 9, 10 reach each tail of
    that ring."""
    B, S = 1 << 20, 32  # 32 stripes x 256 tiles = 8192 tiles
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False, local_mode=local)
    np_ = c.parityNum
    if layout == "ptr":  # data blocks of a filled slab, parities separate allocations
        src = E.StripeSlab(c, stripes=S, block_bytes=B)
        src.fill_random(seed=77)
        data = [[src.block(s, j) for j in range(k)] for s in range(S)]
    outs = {}
    for env in ("off", "on", "10,32", None):
        E.set_schedule(**E.parse_schedule(window=env))
        if layout == "ptr":
            par = [[torch.empty(B, dtype=torch.uint8, device="cuda") for _ in range(np_)] for _ in range(S)]
            E.BlockBatch(c, data, par).encode()
            torch.cuda.synchronize()
            outs[env] = [par[0], par[S - 1]]
        else:
            slab = E.StripeSlab(c, stripes=S, block_bytes=B, layout=layout)
            slab.fill_random(seed=77)
            slab.encode()
            torch.cuda.synchronize()
            outs[env] = [[p.clone() for p in slab.parity(s)] for s in (0, S - 1)]
            del slab
    for env in ("on", "10,32", None):
        for n in range(2):
            for i in range(np_):
                assert torch.equal(outs[env][n][i], outs["off"][n][i]), (env, n, i)
    W = 8192
    oc = orc.codec("C", k, m, r, W)
    for n, s in enumerate((0, S - 1)):
        want = oc.encode([orc.fill(W, 77, s, j, B - W) for j in range(k)], literal=local == "literal")
        for i, w in enumerate(want):
            assert np.array_equal(outs["on"][n][i][B - W:].cpu().numpy(), w), (s, i)


@pytest.mark.parametrize("remap", ["0", "1", None])
def test_xcd_remap_same_bytes(E, torch, orc, schedule, remap):
    """The per-XCD tile order (ecw_set_schedule's xcd_remap; default on for pointer-table
    encodes, off elsewhere) only permutes which workgroup takes which tile:
    pointer-table encode and repair, and the split slab's encode, give the
    oracle's bytes with it on, off and at the default, with a grid that is and
    one that is not a multiple of 8 workgroups."""
    E.set_schedule(**E.parse_schedule(remap=remap))
    k, m, r = 64, 3, 16
    for B, S in ((1 << 20, 32), (3 * 4096 + 64, 5)):  # 8192 tiles; 20 tiles (+ ragged)
        c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
        src = E.StripeSlab(c, stripes=S, block_bytes=B, layout="split")
        src.fill_random(seed=33)
        src.encode()
        data = [[src.block(s, j).clone() for j in range(k)] for s in range(S)]
        par = [[torch.empty(B, dtype=torch.uint8, device="cuda") for _ in range(c.parityNum)] for _ in range(S)]
        batch = E.BlockBatch(c, data, par)
        batch.encode()
        out = [torch.empty(B, dtype=torch.uint8, device="cuda") for _ in range(S)]
        batch.repair(0, out)
        torch.cuda.synchronize()
        W = min(8192, B)
        oc = orc.codec("C", k, m, r, W)
        for s in (0, S - 1):
            for i in range(c.parityNum):
                assert torch.equal(par[s][i], src.parity(s)[i]), (B, s, i)
            want = oc.encode([orc.fill(W, 33, s, j, B - W) for j in range(k)])
            for i, w in enumerate(want):
                assert np.array_equal(par[s][i][B - W:].cpu().numpy(), w), (B, s, i)
            assert torch.equal(out[s], data[s][0]), (B, s)


def test_full_size_tiled_bench_path(E, torch, manifest):
    """The bench's timed bytes at the bench's size: tiled slab, CL(128, 27, 3),
    64 MiB blocks, 8 stripes, seed 103. Stripe 0 is the stripe of manifest
    'cfg3_full' (digests from the reference's ISA-L build): every parity and
    the D0 repair match its SHA-256; every stripe's parities equal the block
    slab's encode of the same bytes and every D0 repair equals D0."""
    e = next(x for x in manifest["full"] if x["name"] == "cfg3_full")
    k, m, r, B, S = e["k"], e["m"], e["r"], e["len"], 8
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    tiled = E.StripeSlab(c, stripes=S, block_bytes=B, layout="tiled", chunk=8192)
    tiled.fill_random(seed=e["seed"])
    tiled.encode()
    out = torch.empty(S * B, dtype=torch.uint8, device="cuda")
    tiled.repair(0, out)
    torch.cuda.synchronize()
    assert [sha(p.cpu().numpy()) for p in tiled.parity(0)] == e["parity_sha256"]
    assert sha(out[:B].cpu().numpy()) == e["repair_d0_sha256"]
    blocks = E.StripeSlab(c, stripes=S, block_bytes=B)
    blocks.fill_random(seed=e["seed"])
    blocks.encode()
    torch.cuda.synchronize()
    for s in range(S):
        assert torch.equal(out[s * B:(s + 1) * B], tiled.block(s, 0)), s
        for i, (a, b) in enumerate(zip(tiled.parity(s), blocks.parity(s))):
            assert torch.equal(a, b), (s, i)
    del tiled, blocks, out
    torch.cuda.empty_cache()


def test_hbm_filling_batch_configs3(E, torch, orc):
    """BASELINE configs[3] as the bench runs it (bench.py --hbm-fill): 256
    stripes, block size sized from free HBM (shard.hbm_fill_block_mib), tiled
    slab, ONE ticket-ordered launch. Oracle windows at the first, middle and
    last column piece of the first, middle and last stripe; stripes 0 and 255
    re-encoded alone (launch-window path) equal; every stripe's D0 repair == D0."""
    from ecwide_amd.shard import hbm_fill_block_mib

    k, m, r, S, W, seed = 128, 3, 27, 256, 8192, 103
    torch.cuda.empty_cache()
    free = torch.cuda.mem_get_info()[0]
    mib = hbm_fill_block_mib(free, k, m + 5, S)
    assert mib >= 1, free
    B = mib << 20
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    slab = E.StripeSlab(c, stripes=S, block_bytes=B, layout="tiled", chunk=W)
    assert slab.encode_launches() == 1
    out = torch.empty(S * B, dtype=torch.uint8, device="cuda")
    slab.fill_random(seed=seed)
    slab.encode()
    slab.repair(0, out)
    torch.cuda.synchronize()
    oc = orc.codec("C", k, m, r, W)
    for s in (0, S // 2, S - 1):
        par = slab.parity(s)
        for off in (0, B // 2, B - W):
            want = oc.encode([orc.fill(W, seed, s, j, off) for j in range(k)])
            for i, w in enumerate(want):
                assert np.array_equal(par[i][off:off + W].cpu().numpy(), w), (s, off, i)
    for s in range(S):
        assert torch.equal(out[s * B:(s + 1) * B], slab.block(s, 0)), s
    del out
    pbuf = torch.empty((c.parityNum, B), dtype=torch.uint8, device="cuda")
    for s in (0, S - 1):
        c.encodeData([slab.block(s, j) for j in range(k)], [pbuf[i] for i in range(c.parityNum)])
        torch.cuda.synchronize()
        for i, p in enumerate(slab.parity(s)):
            assert torch.equal(p, pbuf[i]), (s, i)
    del slab, pbuf
    torch.cuda.empty_cache()


@pytest.mark.parametrize("k,m,r,B,S,local", [
    (128, 3, 27, 1 << 16, 3, "xor"),             # the bench shape, u32-entry asm tile, parked locals
    (20, 6, 4, 3 * 4096 + 48, 2, "xor"),         # 5-8 rows (u64 tile), 5 groups, ragged tail
    (30, 11, 4, 8192, 2, "literal"),             # two passes (8 + 3 rows), 8 groups not parked, zero L
    (1, 2, 1, 5000, 3, "xor"),                   # k = 1: the C++ tile
    (33, 3, 4, 4096 * 3, 4, "xor"),              # odd k, > 5 groups
])
def test_encode_ptrs_dev_vs_oracle(E, torch, orc, k, m, r, B, S, local):
    """ecw_encode_ptrs_dev: a batch of stripes whose blocks are separate
    allocations, one launch, pointers in device tables (BlockBatch /
    NativeCodec.encodeStripes) vs the oracle."""
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False, local_mode=local)
    oc = orc.codec("C", k, m, r, B)
    data = [[torch.from_numpy(orc.fill(B, 500 + s, s, j)).cuda() for j in range(k)] for s in range(S)]
    par = [[torch.full((B + 32,), 0x5A, dtype=torch.uint8, device="cuda") for _ in range(c.parityNum)]
           for _ in range(S)]
    c.encodeStripes(data, [[p[:B] for p in ps] for ps in par])
    torch.cuda.synchronize()
    for s in range(S):
        want = oc.encode([d.cpu().numpy() for d in data[s]], literal=local == "literal", threads=8)
        for i, w in enumerate(want):
            got = par[s][i].cpu().numpy()
            assert np.array_equal(got[:B], w), (s, i)
            assert (got[B:] == 0x5A).all(), ("wrote past the block", s, i)


@pytest.mark.parametrize("n,ln,S", [(1, 4096, 2), (27, 3 * 4096 + 48, 3), (33, 8192, 2), (64, 5000, 2)])
def test_xor_reduce_ptrs_dev_vs_oracle(E, torch, orc, n, ln, S):
    """ecw_xor_reduce_ptrs_dev: dst[s] = XOR of n separately allocated blocks,
    every stripe in one launch (straight-line kernel up to 32 sources, the ring
    kernel beyond), ragged tails, nothing written past the block."""
    from ctypes import c_void_p

    from ecwide_amd._lib import lib

    data = [[orc.fill(ln, 70 + s, s, i) for i in range(n)] for s in range(S)]
    src = [[torch.from_numpy(d).cuda() for d in row] for row in data]
    dst = [torch.full((ln + 32,), 0x5A, dtype=torch.uint8, device="cuda") for _ in range(S)]
    st = torch.tensor([b.data_ptr() for row in src for b in row], dtype=torch.int64, device="cuda")
    dt = torch.tensor([d.data_ptr() for d in dst], dtype=torch.int64, device="cuda")
    assert lib.ecw_xor_reduce_ptrs_dev(0, S, n, c_void_p(st.data_ptr()), c_void_p(dt.data_ptr()), ln,
                                       c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    torch.cuda.synchronize()
    for s in range(S):
        got = dst[s].cpu().numpy()
        assert np.array_equal(got[:ln], orc.xor_blocks(data[s])), s
        assert (got[ln:] == 0x5A).all(), s


@pytest.mark.parametrize("sched", [None, "1,0", "2,0", "4,0", "4,1", "2,1", "1,1", "4,0,11,64", "2,0,11,64",
                                   "2,0,10,32", "1,0,10,32", "4,1,12,128", "4,0+r"])
def test_xor_schedules_same_bytes(E, torch, orc, schedule, sched):
    """Every XOR schedule (ecw_xor.hpp launch_xor_range; ecw_set_schedule's
    xor_* fields, written "K,ORDER[,LOG2P,W]": K column tiles per workgroup read diagonally,
    column-major group order, write window; None = the library's choice) gives
    the oracle's bytes through all four source forms (pointer mode, device
    pointer tables, split slab, block slab), with whole groups of K tiles, a
    ragged last group and a ragged last tile, at several fan-ins, and writes
    nothing past a block."""
    from ctypes import c_void_p

    from ecwide_amd._lib import lib

    base, _, r = (sched or "").partition("+")  # "+r": with the per-XCD group order
    E.set_schedule(**E.parse_schedule(xor=base or None, remap="1" if r == "r" else None))
    ln, S = 5 * 16384 + 2 * 4096 + 48, 3
    strm = c_void_p(torch.cuda.current_stream().cuda_stream)
    for n in (1, 5, 27, 32):
        data = [[orc.fill(ln, 500 + n, s, i) for i in range(n)] for s in range(S)]
        want = [orc.xor_blocks(row) for row in data]
        src = [[torch.from_numpy(d).cuda() for d in row] for row in data]
        # pointer mode (XorPtr)
        out = torch.full((ln + 32,), 0xA5, dtype=torch.uint8, device="cuda")
        E.xor_reduce(src[0], out[:ln])
        torch.cuda.synchronize()
        assert np.array_equal(out[:ln].cpu().numpy(), want[0]) and (out[ln:].cpu().numpy() == 0xA5).all(), n
        # device pointer tables (XorTab)
        dst = [torch.full((ln + 32,), 0x5A, dtype=torch.uint8, device="cuda") for _ in range(S)]
        st = torch.tensor([b.data_ptr() for row in src for b in row], dtype=torch.int64, device="cuda")
        dt = torch.tensor([d.data_ptr() for d in dst], dtype=torch.int64, device="cuda")
        assert lib.ecw_xor_reduce_ptrs_dev(0, S, n, c_void_p(st.data_ptr()), c_void_p(dt.data_ptr()), ln, strm) == 0
        torch.cuda.synchronize()
        for s in range(S):
            got = dst[s].cpu().numpy()
            assert np.array_equal(got[:ln], want[s]) and (got[ln:] == 0x5A).all(), (n, s)
    # slabs (XorSplit, XorSlab): CL repair of D0 from its group
    k, r = 40, 27
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, 2, r, ln), 1, False)
    for layout in ("split", "blocks"):
        slab = E.StripeSlab(c, stripes=S, block_bytes=ln, layout=layout)
        slab.fill_random(seed=91)
        slab.encode()
        out = torch.full((S * slab.out_stride,), 0x33, dtype=torch.uint8, device="cuda")
        for lost in (0, k + 2):
            slab.repair(lost, out)
            torch.cuda.synchronize()
            for s in range(S):
                assert torch.equal(out[s * slab.out_stride:s * slab.out_stride + ln], slab.block(s, lost)), \
                    (layout, lost, s)


@pytest.mark.parametrize("sched", [None, "1,0", "2,0", "2,0,11,64", "2,1,11,64", "4,0", "4,1", "4,0,11,64"])
@pytest.mark.parametrize("pieces", [8, 7])
def test_tiled_repair_schedules_same_bytes(E, torch, orc, schedule, sched, pieces):
    """The tiled slab's repair (8 KiB units = 2 column tiles; ecw_xor.hpp) under
    every schedule -- K = 4 takes pairs of units (XorSplitPair) when the unit
    count is even and falls back to ragged groups when it is odd -- rebuilds
    every lost D and L block exactly, with the default (K = 2 + window at
    >= 8192 tiles) among them."""
    E.set_schedule(**E.parse_schedule(xor=sched))
    k, m, r, S = 40, 2, 27, 3
    B = pieces * 8192  # 3 x 8 = 24 units (pairs) or 3 x 7 = 21 (odd: no pairing)
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    slab = E.StripeSlab(c, stripes=S, block_bytes=B, layout="tiled", chunk=8192)
    slab.fill_random(seed=57)
    slab.encode()
    out = torch.full((S * B,), 0x33, dtype=torch.uint8, device="cuda")
    for lost in (0, 26, 27, k + m, k + m + 1):
        slab.repair(lost, out)
        torch.cuda.synchronize()
        for s_ in range(S):
            assert torch.equal(out[s_ * B:(s_ + 1) * B], slab.block(s_, lost)), (sched, pieces, lost, s_)
    # the bench's unit count with the window's launch floor reached (>= 8192 tiles)
    Bb, Sb = 4 << 20, 16  # 16 stripes x 512 units x 2 tiles = 16384 tiles
    cb = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(128, 3, 27, Bb), 1, False)
    big = E.StripeSlab(cb, stripes=Sb, block_bytes=Bb, layout="tiled", chunk=8192)
    big.fill_random(seed=58)
    big.encode()
    outb = torch.empty(Sb * Bb, dtype=torch.uint8, device="cuda")
    big.repair(0, outb)
    torch.cuda.synchronize()
    for s_ in (0, Sb - 1):
        assert torch.equal(outb[s_ * Bb:(s_ + 1) * Bb], big.block(s_, 0)), (sched, s_)


def test_block_batch_encode_repair(E, torch, orc):
    """BlockBatch: a batch of stripes of separately allocated blocks, encoded and
    every D and L block repaired through device pointer tables, one launch each."""
    k, m, r, B, S = 40, 3, 9, 3 * 8192, 3
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    data = [[torch.from_numpy(orc.fill(B, 12, s, j)).cuda() for j in range(k)] for s in range(S)]
    par = [[torch.empty(B, dtype=torch.uint8, device="cuda") for _ in range(c.parityNum)] for _ in range(S)]
    batch = E.BlockBatch(c, data, par)
    batch.encode()
    oc = orc.codec("C", k, m, r, B)
    torch.cuda.synchronize()
    for s in range(S):
        want = oc.encode([d.cpu().numpy() for d in data[s]])
        assert all(np.array_equal(p.cpu().numpy(), w) for p, w in zip(par[s], want)), s
    out = [torch.empty(B, dtype=torch.uint8, device="cuda") for _ in range(S)]
    for lost in list(range(0, k, 7)) + [k - 1] + [k + m + t for t in range(c.groupNum)]:
        batch.repair(lost, out)
        torch.cuda.synchronize()
        for s in range(S):
            want = data[s][lost] if lost < k else par[s][lost - k]
            assert torch.equal(out[s], want), (lost, s)


@pytest.mark.parametrize("k,m,r,B,S", [(4, 2, 2, 256 << 20, 4), (64, 2, 32, 64 << 20, 16)])
def test_encode_ptrs_dev_ticket_and_errors(E, torch, orc, k, m, r, B, S):
    """>= 262,144 tiles through the pointer tables take the ticket-ordered
    launch (twice on one stream: the counter carries over); the result equals
    the split slab's encode of the same bytes. At k = 64 the pointer-table
    launch also holds its stores for the write window (the split slab does
    not), 68 GiB. Misaligned tables and m = 0 are refused."""
    from ctypes import c_void_p

    from ecwide_amd._lib import lib

    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    slab = E.StripeSlab(c, stripes=S, block_bytes=B, layout="split")
    slab.fill_random(seed=8)
    slab.encode()
    par = [[torch.empty(B, dtype=torch.uint8, device="cuda") for _ in range(c.parityNum)] for _ in range(S)]
    batch = E.BlockBatch(c, [slab.data(s) for s in range(S)], par)
    batch.encode()
    batch.encode()
    torch.cuda.synchronize()
    for s in range(S):
        for i, p in enumerate(slab.parity(s)):
            assert torch.equal(p, par[s][i]), (s, i)
    if k != 4:
        del slab, batch, par
        torch.cuda.empty_cache()
        return
    st = lib.ecw_encode_ptrs_dev(c._h, S, c_void_p(batch.dtab.data_ptr() + 4), c_void_p(batch.ptab.data_ptr()), B,
                                 c_void_p(torch.cuda.current_stream().cuda_stream))
    assert st == -4
    c0 = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(8, 0, 4, 4096), 1, False)
    st = lib.ecw_encode_ptrs_dev(c0._h, 1, c_void_p(batch.dtab.data_ptr()), c_void_p(batch.ptab.data_ptr()), 4096,
                                 c_void_p(torch.cuda.current_stream().cuda_stream))
    assert st == -5
    del slab, batch, par
    torch.cuda.empty_cache()


def test_decode_partial_xor_golden(E, torch, orc, manifest):
    for e in manifest["xor_reduce"]:
        data = [orc.fill(e["len"], e["seed"], 0, j) for j in range(e["n"])]
        want = golden_blocks(e, 1, e["len"])[0]
        d = dev_blocks(torch, e["n"], e["len"], data)
        out = torch.zeros(e["len"], dtype=torch.uint8, device="cuda")
        E.xor_reduce(d, out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), want), e["n"]
    # decodeData / partialDecodeData through a CL codec (cfg#3 geometry: ddn 9, pdn 4)
    s = E.CodingScheme.getClScheme(128, 3, 27, 4096)
    c = E.NativeCodec.getClCodec(s, 1, False)
    assert (c.decodeDataNum, c.partialDecodeNum) == (9, 4)
    data = [orc.fill(4096, 50, 0, j) for j in range(9)]
    t = np.zeros(4096, np.uint8)
    c.decodeData(data, t)
    assert np.array_equal(t, orc.xor_blocks(data))
    c.partialDecodeData(data[:4], t)
    assert np.array_equal(t, orc.xor_blocks(data[:4]))
    # the same natives on HBM blocks (ecw_decode_dev / ecw_partial_decode_dev:
    # the requestor's and a relayer's stage of the CL repair, ECTaskProcessor.java:
    # 293-332), ragged length, against the oracle's decode over the codec's tables
    oc = orc.codec("C", 128, 3, 27, 4096)
    for ln in (4096, 3000, 17):
        data = [orc.fill(ln, 51, 0, j) for j in range(9)]
        d = dev_blocks(torch, 9, ln, data)
        t = torch.zeros(ln, dtype=torch.uint8, device="cuda")
        c.decodeData(d, t)
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy(), oc.decode(data)), ln
        c.partialDecodeData(d[:4], t)
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy(), oc.partial_decode(data[:4])), ln


def test_xor_intermediate_literal_and_xor(E, torch, orc, manifest):
    e = manifest["xor_intermediate"]
    m, ln = e["m"], e["len"]
    s1, s2, s3 = e["seeds"]
    src1 = [orc.fill(ln, s1, 0, j) for j in range(m)]
    tgt = [orc.fill(ln, s2, 0, j) for j in range(m)]
    src2 = [orc.fill(ln, s3, 0, j) for j in range(m)]
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(8, m, 4, ln), 1, False)
    c.setXorIntermediateMode("literal")
    c.xorIntemediate(src1, tgt)
    assert [sha(x) for x in tgt] == e["first"]
    c.xorIntemediate(src2, tgt)
    want = golden_blocks(e["second"], m, ln)
    assert all(np.array_equal(a, b) for a, b in zip(tgt, want))
    # device path, XOR mode
    c2 = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(8, m, 4, ln), 1, False)
    ds = dev_blocks(torch, m, ln, src2)
    dt = dev_blocks(torch, m, ln, src1)
    c2.xorIntemediate(ds, dt)
    torch.cuda.synchronize()
    for i in range(m):
        assert np.array_equal(dt[i].cpu().numpy(), src1[i] ^ src2[i])


def test_ecwide_h_wrappers(E, orc, manifest):
    """ECWide-H g_encode = Cauchy(GN=14, GK=11) -> an RS codec k=11, m=3;
    l_encode / l_middle / l_decode = XOR of 11 / 4 / 5 blocks."""
    h = manifest["ecwide_h"]
    gd = [orc.fill(4096, 42, 0, j) for j in range(11)]
    c = E.NativeCodec.getRsCodec(E.CodingScheme.getRsScheme(11, 3, 4096))
    par = [np.zeros(4096, np.uint8) for _ in range(3)]
    c.encodeData(gd, par)
    assert all(np.array_equal(a, b) for a, b in zip(par, golden_blocks(h["g_encode"], 3, 4096)))
    for key, seed, n in [("l_encode", 41, 11), ("l_middle", 43, 4), ("l_decode", 44, 5)]:
        d = [orc.fill(4096, seed, 0, j) for j in range(n)]
        cc = E.NativeCodec.getRsCodec(E.CodingScheme.getRsScheme(n, 1, 4096))
        t = np.zeros(4096, np.uint8)
        cc.decodeData(d, t)
        assert np.array_equal(t, golden_blocks(h[key], 1, 4096)[0]), key


def test_fill_kernel_matches_oracle(E, torch, orc):
    s = E.CodingScheme.getClScheme(10, 2, 4, 5000)
    c = E.NativeCodec.getClCodec(s, 1, False)
    slab = E.StripeSlab(c, stripes=3, block_bytes=5000)
    slab.fill_random(seed=123, s0=4)
    torch.cuda.synchronize()
    for st in range(3):
        for j in range(10):
            assert np.array_equal(slab.block(st, j).cpu().numpy(), orc.fill(5000, 123, 4 + st, j)), (st, j)


@pytest.mark.parametrize("chunk,col_offset", [(8192, 0), (4096, 0), (8192, 3 * 8192)])
def test_fill_same_bytes_in_every_layout(E, torch, orc, chunk, col_offset):
    """The tiled slab's blocks hold exactly the block slab's bytes (the PRNG is
    keyed by stripe, block and byte offset, scattered by column piece), also
    for a column slice starting at col_offset (a column-sharded rank)."""
    k, B = 12, 4 * 8192
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, 2, 5, B), 1, False)
    blocks = E.StripeSlab(c, stripes=3, block_bytes=B)
    tiled = E.StripeSlab(c, stripes=3, block_bytes=B, layout="tiled", chunk=chunk)
    blocks.fill_random(seed=55, s0=2, col_offset=col_offset)
    tiled.fill_random(seed=55, s0=2, col_offset=col_offset)
    torch.cuda.synchronize()
    for st in range(3):
        for j in range(k):
            assert torch.equal(tiled.block(st, j), blocks.block(st, j)), (st, j)
            assert np.array_equal(tiled.block(st, j).cpu().numpy(), orc.fill(B, 55, 2 + st, j, col_offset)), (st, j)


@pytest.mark.parametrize("k,m,r,B,S", [(32, 3, 11, 1 << 20, 2), (32, 2, 8, (1 << 18) + 48, 3),
                                       (128, 3, 27, 1 << 18, 2), (20, 8, 6, 70000, 2), (40, 11, 9, 12345, 2),
                                       (5, 5, 2, 4096, 4), (250, 6, 50, 8192, 1), (7, 1, 7, 16, 5),
                                       # asm tile (slab, <= 4 global rows): odd k (3-row epilogue), the
                                       # minimum k = 2, one group, > 5 groups (stores not parked)
                                       (33, 3, 4, 3 * 4096 + 100, 2), (31, 4, 31, 8192, 2), (2, 1, 1, 8192, 3),
                                       (3, 2, 2, 8192, 2), (128, 3, 8, 1 << 16, 2), (6, 4, 1, 4096, 2),
                                       # the 5-8-row asm tile: parked (<= 5 groups) and not, k = 2 / 3
                                       (128, 6, 27, 1 << 16, 2), (40, 8, 7, 3 * 4096 + 48, 2),
                                       (3, 7, 2, 8192, 2), (2, 5, 1, 4096, 2)])
@pytest.mark.parametrize("layout", ["blocks", "split"])
def test_slab_encode_repair_vs_oracle(E, torch, orc, k, m, r, B, S, layout):
    """Batched slab encode vs oracle at mid sizes, in-slab parities (ChunkGenerator
    order) and the split slab; repair of every data and local block equals
    the erased block."""
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    slab = E.StripeSlab(c, stripes=S, block_bytes=B, layout=layout)
    slab.fill_random(seed=99)
    slab.encode()
    torch.cuda.synchronize()
    oc = orc.codec("C", k, m, r, B)
    for st in range(S):
        data = [orc.fill(B, 99, st, j) for j in range(k)]
        want = oc.encode(data, threads=8)
        for i, p in enumerate(slab.parity(st)):
            assert np.array_equal(p.cpu().numpy(), want[i]), (st, i)
    out = torch.empty(S * slab.out_stride, dtype=torch.uint8, device="cuda")
    o = slab.out_stride
    g = c.groupNum
    lost_list = sorted({0, k - 1, min(r, k - 1)} | {k + m + t for t in range(min(g, 2))})
    for lost in lost_list:
        slab.repair(lost, out)
        torch.cuda.synchronize()
        for st in range(S):
            assert torch.equal(out[st * o:st * o + B], slab.block(st, lost)), (lost, st)


def test_random_sweep_vs_oracle(E, torch, orc):
    """Seeded random CL shapes (k, m, r, B, stripes, local mode) against the
    oracle: covers the asm tile's row loop / 2-3-row epilogue / group
    boundaries / parked and unparked locals / ragged tails in combination,
    in slab mode and in pointer mode (block j stored at slot k-1-j, so the
    pointers are not one stride apart)."""
    rng = np.random.default_rng(2026)
    for trial in range(32):
        k = int(rng.integers(2, 160))
        m = int(rng.integers(1, 9))  # 1-4 rows: the u32-entry tile, 5-8: the u64-entry tile
        r = int(rng.integers(1, k + 1))
        B = int(rng.choice([4096, 8192, 4096 * int(rng.integers(1, 4)) + 16 * int(rng.integers(1, 256))]))
        S = int(rng.integers(1, 3))
        literal = trial % 4 == 3
        c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False,
                                     local_mode="literal" if literal else "xor")
        oc = orc.codec("C", k, m, r, B)
        slab = E.StripeSlab(c, stripes=S, block_bytes=B)
        slab.fill_random(seed=1000 + trial)
        slab.encode()
        torch.cuda.synchronize()
        wants = []
        for st in range(S):
            want = oc.encode([orc.fill(B, 1000 + trial, st, j) for j in range(k)], literal=literal, threads=8)
            wants.append(want)
            for i, p in enumerate(slab.parity(st)):
                assert np.array_equal(p.cpu().numpy(), want[i]), (trial, k, m, r, B, st, i)
        np_ = c.parityNum
        dbuf = torch.empty((k, B), dtype=torch.uint8, device="cuda")
        pbuf = torch.full((np_, B), 0x5A, dtype=torch.uint8, device="cuda")
        for j in range(k):
            dbuf[k - 1 - j].copy_(slab.block(0, j))
        c.encodeData([dbuf[k - 1 - j] for j in range(k)], [pbuf[np_ - 1 - i] for i in range(np_)])
        torch.cuda.synchronize()
        for i in range(np_):
            assert np.array_equal(pbuf[np_ - 1 - i].cpu().numpy(), wants[0][i]), ("ptr", trial, k, m, r, B, i)


@pytest.mark.parametrize("code,k,m,r,B,S", [
    ("R", 128, 12, 0, 3 * 4096 + 80, 2),   # RS(128, 12): one pass of the 16-row asm tile + its ragged tail
    ("R", 20, 9, 0, 4096, 3),              # 9 rows
    ("C", 64, 16, 10, 8192 + 16, 2),       # 16 global rows + 7 XOR locals
    ("C", 200, 10, 40, 4096 + 1, 1),       # wide k: 100 KiB of tables (> 64 KiB of dynamic LDS)
    ("C", 128, 9, 27, 8192, 3),            # 9 rows + 5 parked XOR locals
    ("R", 128, 20, 0, 4096, 1),            # 20 rows: a 16-row pass and a 4-row pass
    ("R", 21, 10, 0, 4096 + 16, 2),        # k = 21: the three-slot ring's 3-row tail, every addressing mode
    ("C", 21, 6, 5, 4096, 2),              # the same tail in the 5-8-row tile (5 groups, parked)
])
def test_more_than_8_global_rows(E, torch, orc, code, k, m, r, B, S):
    """ECWide-C's RS / TL / CL codecs take any m (NativeCodec.java:20-54):
    9-16 global rows run in ONE pass over the data (the 16-row asm tile:
    16-byte packed entries, ds_read_b128), more in passes of 16; slab mode, pointer mode
    (blocks in reverse order) and device pointer tables, vs the oracle."""
    if code == "R":
        c = E.NativeCodec.getRsCodec(E.CodingScheme.getRsScheme(k, m, B))
    else:
        c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    oc = orc.codec(code, k, m, r if r else k, B)
    slab = E.StripeSlab(c, stripes=S, block_bytes=B)
    slab.fill_random(seed=77)
    slab.encode()
    torch.cuda.synchronize()
    wants = [oc.encode([orc.fill(B, 77, s, j) for j in range(k)], threads=8) for s in range(S)]
    for s in range(S):
        for i, p in enumerate(slab.parity(s)):
            assert np.array_equal(p.cpu().numpy(), wants[s][i]), ("slab", s, i)
    np_ = c.parityNum
    Bp = (B + 15) // 16 * 16  # rows 16-byte aligned
    dbuf = torch.empty((k, Bp), dtype=torch.uint8, device="cuda")
    pbuf = torch.full((np_, Bp), 0x5A, dtype=torch.uint8, device="cuda")
    for j in range(k):
        dbuf[k - 1 - j, :B].copy_(slab.block(0, j))
    c.encodeData([dbuf[k - 1 - j, :B] for j in range(k)], [pbuf[np_ - 1 - i, :B] for i in range(np_)])
    torch.cuda.synchronize()
    for i in range(np_):
        assert np.array_equal(pbuf[np_ - 1 - i, :B].cpu().numpy(), wants[0][i]), ("ptr", i)
    data = [[slab.block(s, j).clone() for j in range(k)] for s in range(S)]
    par = [[torch.full((B,), 0xA5, dtype=torch.uint8, device="cuda") for _ in range(np_)] for _ in range(S)]
    c.encodeStripes(data, par)
    torch.cuda.synchronize()
    for s in range(S):
        for i in range(np_):
            assert np.array_equal(par[s][i].cpu().numpy(), wants[s][i]), ("tables", s, i)


@pytest.mark.parametrize("B", [(20 << 20) + 37, (8 << 20), 4096 * 3 + 5])
def test_host_pipeline_multi_chunk_and_repair(E, torch, orc, B):
    """ecw_encode / ecw_repair on host buffers larger than one 8 MiB pipeline
    slice (ragged tail), pageable and pinned, vs the oracle."""
    k, m, r = 10, 2, 4
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    data = [orc.fill(B, 77, 0, j) for j in range(k)]
    want = orc.codec("C", k, m, r, B).encode(data, threads=8)
    par = [np.zeros(B, np.uint8) for _ in range(c.parityNum)]
    c.encodeData(data, par)
    for i, (g, w) in enumerate(zip(par, want)):
        assert np.array_equal(g, w), i
    pinned = [torch.empty(B, dtype=torch.uint8, pin_memory=True).numpy() for _ in range(k + c.parityNum)]
    for j in range(k):
        pinned[j][:] = data[j]
    c.encodeData(pinned[:k], pinned[k:])
    assert all(np.array_equal(a, b) for a, b in zip(pinned[k:], want))
    blocks = data + par
    for lost in (0, k - 1, k + m):
        out = np.zeros(B, np.uint8)
        c.repairBlock([b if i != lost else None for i, b in enumerate(blocks)], lost, out)
        assert np.array_equal(out, blocks[lost]), lost


def test_pinned_host_numa_local_pipeline(E, orc):
    """ecw_host_alloc (PinnedHost): zeroed, pinned host memory on the GPU's NUMA
    node (when the host reports one); the host pipeline encodes and repairs
    through it bit-exact vs the oracle; freeing twice is refused, not a crash."""
    k, m, r, B = 20, 3, 5, (9 << 20) + 48  # two 8 MiB pipeline slices + a ragged tail
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    np_ = c.parityNum
    h = E.PinnedHost((k + np_ + 1) * B, c.device)
    assert h.array.size == (k + np_ + 1) * B and not h.array[:: 1 << 20].any()
    if h.device_numa_node >= 0:
        assert h.numa_node == h.device_numa_node, (h.numa_node, h.device_numa_node)
    v = [h.array[i * B:(i + 1) * B] for i in range(k + np_ + 1)]
    data = [orc.fill(B, 31, 0, j) for j in range(k)]
    for j in range(k):
        v[j][:] = data[j]
    c.encodeData(v[:k], v[k:k + np_])
    want = orc.codec("C", k, m, r, B).encode(data, threads=8)
    assert all(np.array_equal(a, b) for a, b in zip(v[k:k + np_], want))
    c.repairBlock(v[:k + np_], 0, v[k + np_])
    assert np.array_equal(v[k + np_], data[0])
    ptr = h.ptr
    h.free()
    from ctypes import c_void_p

    assert E._lib.lib.ecw_host_free(c_void_p(ptr)) == -1  # already freed: refused


@pytest.mark.parametrize("k,m,r,B", [(32, 3, 11, 65536 + 16), (128, 3, 27, 1 << 16), (20, 2, 5, 4096)])
def test_multinode_encode_chain(E, torch, orc, k, m, r, B):
    """Multi-node CL encode (ECTaskProcessor.java:267-291): each of the g
    nodes encodes its own group on the GPU, partials are merged along the
    chain with xorIntemediate; the result equals single-node encodeData
    (the oracle), and each node's local parity is its group's XOR. (The
    reference's own slice is misaligned, so this is pinned to the
    single-node code, not to a reference multi-node run.)"""
    s = E.CodingScheme.getClScheme(k, m, r, B)
    g = s.groupNum
    data = [orc.fill(B, 21, 0, j) for j in range(k)]
    want = orc.codec("C", k, m, r, B).encode(data, threads=8)
    chain = None
    for node in range(1, g + 1):
        c = E.NativeCodec.getClCodec(s, node, True)
        c0 = (g - node) * r
        mine = [torch.from_numpy(d).cuda() for d in data[c0:c0 + c.encodeDataNum]]
        par = [torch.zeros(B, dtype=torch.uint8, device="cuda") for _ in range(m + 1)]
        c.encodeData(mine, par)
        torch.cuda.synchronize()
        t = c0 // r
        assert np.array_equal(par[m].cpu().numpy(), want[m + t]), ("local", node)
        if chain is None:
            chain = par[:m]
        else:
            c.xorIntemediate(par[:m], chain)  # chain ^= this node's partials
    torch.cuda.synchronize()
    for i in range(m):
        assert np.array_equal(chain[i].cpu().numpy(), want[i]), i


@pytest.mark.parametrize("k,m,r", [(32, 2, 8), (33, 3, 4), (128, 6, 27)])
def test_literal_mode_slab_writes_zero_locals(E, torch, orc, k, m, r):
    """ECWide-C literal mode: every L block is written as zeros (parked and
    unparked asm paths); the global parities are unchanged."""
    B = 65536 + 100
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False, local_mode="literal")
    slab = E.StripeSlab(c, stripes=2, block_bytes=B)
    slab.buf.fill_(0x5A)
    slab.fill_random(seed=3)
    slab.encode()
    torch.cuda.synchronize()
    oc = orc.codec("C", k, m, r, B)
    for st in range(2):
        want = oc.encode([orc.fill(B, 3, st, j) for j in range(k)], threads=8)
        par = slab.parity(st)
        for i in range(m):
            assert np.array_equal(par[i].cpu().numpy(), want[i]), (st, i)
        for L in par[m:]:
            assert not L.any()


def full_digest_case(E, torch, name, manifest, layout="blocks"):
    e = next(x for x in manifest["full"] if x["name"] == name)
    k, m, r, B = e["k"], e["m"], e["r"], e["len"]
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    slab = E.StripeSlab(c, stripes=1, block_bytes=B, layout=layout)  # tiled: the default piece for k
    slab.fill_random(seed=e["seed"])
    slab.encode()
    out = torch.empty(B, dtype=torch.uint8, device="cuda")
    slab.repair(0, out)
    torch.cuda.synchronize()
    got = [sha(p.cpu().numpy()) for p in slab.parity(0)]
    assert got == e["parity_sha256"]
    assert sha(out.cpu().numpy()) == e["repair_d0_sha256"]
    # size-independent: the repair rebuilt D0 exactly
    assert torch.equal(out, slab.block(0, 0))


def test_full_cfg2_k32_16MiB_digests(E, torch, manifest):
    full_digest_case(E, torch, "cfg2_full", manifest)


def test_full_cfg3_k128_64MiB_digests(E, torch, manifest):
    full_digest_case(E, torch, "cfg3_full", manifest)


def test_full_cfg1_k32_64MiB_digests(E, torch, manifest):
    full_digest_case(E, torch, "cfg1_full", manifest)


@pytest.mark.parametrize("name", ["cfg1_full", "cfg2_full"])
def test_full_k32_digests_tiled_default_piece(E, torch, manifest, name):
    """The k = 32 BASELINE shapes in the tiled slab at its default piece for
    k = 32 (16 KiB, ecwide_amd/slab.py default_chunk; the bench's configs1 /
    configs0_shape legs): the same full-size digests as the block layout."""
    from ecwide_amd.slab import default_chunk

    assert default_chunk(32) == 16384
    full_digest_case(E, torch, name, manifest, layout="tiled")


def test_linearity_full_size(E, torch):
    """encode(a ^ b) == encode(a) ^ encode(b) at the bench shape (k=128, 64 MiB)."""
    B = 1 << 26
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(128, 3, 27, B), 1, False)
    slab = E.StripeSlab(c, stripes=3, block_bytes=B)
    slab.fill_random(seed=1)
    for j in range(128):
        slab.block(2, j).copy_(slab.block(0, j) ^ slab.block(1, j))
    slab.encode()
    torch.cuda.synchronize()
    for i in range(c.parityNum):
        assert torch.equal(slab.parity(2)[i], slab.parity(0)[i] ^ slab.parity(1)[i]), i


def test_max_block_size_1GiB(E, torch, orc):
    """The reference's largest chunkSize (int lengths, powers of two <= 2^30,
    SURVEY §8b) at k=128: 137 GiB of HBM. Column windows at the start, the
    middle (odd offset) and the very end of every block vs the oracle on the
    same window (columns are independent), every L block and D0 rebuilt
    exactly over the whole GiB."""
    k, m, r, B = 128, 3, 27, 1 << 30
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, B), 1, False)
    slab = E.StripeSlab(c, stripes=1, block_bytes=B)
    slab.fill_random(seed=77)
    slab.encode()
    out = torch.empty(B, dtype=torch.uint8, device="cuda")
    slab.repair(0, out)
    torch.cuda.synchronize()
    assert torch.equal(out, slab.block(0, 0))
    W = 1 << 16
    oc = orc.codec("C", k, m, r, W)
    par = slab.parity(0)
    for off in (0, B // 2 + 7 * 4096 + 16, B - W):
        data = [slab.block(0, j)[off:off + W].cpu().numpy() for j in range(k)]
        want = oc.encode(data, threads=8)
        for i, w in enumerate(want):
            assert np.array_equal(par[i][off:off + W].cpu().numpy(), w), (off, i)
    # local parities over the whole block: XOR of each group equals its L
    g = c.groupNum
    for t in range(g):
        acc = torch.zeros(B, dtype=torch.uint8, device="cuda")
        for j in range(t * r, min(k, (t + 1) * r)):
            acc ^= slab.block(0, j)
        assert torch.equal(acc, par[m + t]), t
    del slab, out, acc
    torch.cuda.empty_cache()


def test_errors_are_loud(E, torch):
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(4, 2, 2, 4096), 1, False)
    base = torch.zeros(4096 * 8 + 64, dtype=torch.uint8, device="cuda")
    d = [base[1 + 4096 * j:1 + 4096 * (j + 1)] for j in range(4)]  # misaligned
    p = [base[4096 * (4 + j):4096 * (5 + j)] for j in range(4)]
    with pytest.raises(E.EcwError) as ei:
        c.encodeData(d, p)
    assert ei.value.status == -4
    with pytest.raises(E.EcwError):
        c.repairSources(4)  # a G block: "not yet" in the reference


def test_chunk_generator_replay(E, orc, tmp_path):
    """BASELINE config #1 plumbing: ChunkGenerator with the default-style
    scheme (CL k=32, r=11, m=3; small chunk) writes D/G/L files whose bytes
    equal the reference's: the oracle's encode of the same source blocks with
    ECWide-C's all-zero L blocks by default (NativeCodec.cc:181-186, as the JNI
    drop-in), the XOR locals with --xor."""
    import os

    from ecwide_amd.chunk_generator import main

    (tmp_path / "scheme.ini").write_text("codeType = CL\nk = 32\ngroupDataNum = 11\nglobalParityNum = 3\n"
                                         "chunkSizeBits = 16\n")
    names = [f"{36 + i}_G_{i}" for i in range(3)] + ["12_L_0", "24_L_1", "35_L_2"]
    for extra, literal in (([], True), (["--xor"], False)):
        out = tmp_path / ("chunks_xor" if extra else "chunks")
        (tmp_path / "settings.ini").write_text(f"chunksDir = {out}\nmultiNodeEncode = true\n")
        assert main(["urandom", "toy", "--scheme", str(tmp_path / "scheme.ini"),
                     "--settings", str(tmp_path / "settings.ini"), *extra]) == 0
        files = sorted(os.listdir(out))
        assert len(files) == 38
        data = [np.fromfile(out / f"{j + 1 + j // 11}_D_{j}", np.uint8) for j in range(32)]
        want = orc.codec("C", 32, 3, 11, 1 << 16).encode(data, literal=literal)
        for n, w in zip(names, want):
            assert np.array_equal(np.fromfile(out / n, np.uint8), w), n
        if literal:
            assert all(not np.fromfile(out / n, np.uint8).any() for n in names[3:])  # zero L files

"""CPU tests of the product's host side through the C ABI: the library
loads, exports everything include/ecwide.h declares, and computes the
reference's geometry, matrices and tables. No kernel launches here."""
import ctypes
import os

import numpy as np
import pytest

import ecwide_amd as E
from ecwide_amd import _lib

# ECWide-C/config/scheme.ini (the reference's default scheme, verbatim data)
DEFAULT_INI = "codeType = CL\nk = 32\ngroupDataNum = 11\nglobalParityNum = 3\nchunkSizeBits = 26"


def test_exports_every_header_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = _lib.header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.SIGNATURES), "ctypes signatures out of sync with the header"
    assert _lib.lib.ecw_abi_version() == 1


def test_library_is_hip_code_for_gfx950():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data  # offload bundle for MI355X
    assert b"encode_kernel" in data and b"xor_kernel" in data


def test_default_scheme_ini(tmp_path):
    p = tmp_path / "scheme.ini"
    p.write_text(DEFAULT_INI)
    s = E.CodingScheme.getFromConfig(str(p))
    assert (s.codeType, s.k, s.groupDataNum, s.m, s.chunkSize) == ("CL", 32, 11, 3, 1 << 26)
    assert (s.groupNum, s.rackNodesNum, s.rackNum, s.chunkSizeBits) == (3, 4, 10, 26)


@pytest.mark.parametrize("text,code,fields", [
    ("codeType = LRC\nk = 12\ngroupDataNum = 4\nglobalParityNum = 2\nchunkSizeBits = 12\n", "LRC", (12, 2, 4, 3, -1, -1)),
    ("codeType = TL\nk = 12\nglobalParityNum = 3\nchunkSizeBits = 10", "TL", (12, 3, -1, 0, 3, 5)),
    ("codeType = RS\nk = 6\nglobalParityNum = 3\nchunkSizeBits = 4\n\n", "RS", (6, 3, -1, 0, 0, 0)),
    ("k = 128\nglobalParityNum = 3\ngroupDataNum = 27\nchunkSizeBits = 26", "CL", (128, 3, 27, 5, 4, 35)),
])
def test_ini_code_types(text, code, fields):
    s = E.CodingScheme.fromConfigText(text)
    assert s.codeType == code
    assert (s.k, s.m, s.groupDataNum, s.groupNum, s.rackNodesNum, s.rackNum) == fields


@pytest.mark.parametrize("text", ["k = 32\nglobalParityNum = 3\nchunkSizeBits = 26",  # CL without r
                                  "codeType = CL\nk = x\ngroupDataNum = 11\nglobalParityNum = 3\nchunkSizeBits = 26",
                                  "codeType = CL\nk 32\n", "codeType = RS\nk = 300\nglobalParityNum = 3\nchunkSizeBits = 4"])
def test_ini_errors(text):
    with pytest.raises(E.EcwError):
        E.CodingScheme.fromConfigText(text)


def test_ini_missing_file():
    with pytest.raises(E.EcwError) as ei:
        E.CodingScheme.getFromConfig("/nonexistent/scheme.ini")
    assert ei.value.status == -7


CODECS = [("C", 32, 3, 11), ("C", 32, 2, 8), ("C", 128, 3, 27), ("C", 10, 4, 3), ("C", 64, 3, 11), ("C", 64, 3, 7),
          ("C", 5, 1, 5), ("L", 12, 2, 4), ("L", 16, 2, 4), ("T", 12, 3, -1), ("T", 13, 4, -1), ("R", 12, 4, -1)]


def _nodes(t, k, m, r):
    if t == "C":
        g = -(-k // r)
        return range(1, k + g + m + 1)
    return range(1, k + m + 1)


@pytest.mark.parametrize("t,k,m,r", CODECS)
def test_codec_geometry_matches_oracle(orc, t, k, m, r):
    code = {"C": "CL", "L": "LRC", "T": "TL", "R": "RS"}[t]
    s = E.CodingScheme._make(code, k, m, r, 4096)
    for node in _nodes(t, k, m, r):
        c = E.NativeCodec(s, node, False)
        o = orc.codec(t, k, m, r, 4096, node)
        assert (c.encodeDataNum, c.decodeDataNum, c.partialDecodeNum) == (
            o.encode_data_num, o.decode_data_num, o.partial_decode_num), node
        assert c.groupNum == o.group_num and c.parityNum == o.parity_num
        if t == "C":
            assert c.rackPerGroup == o.rack_per_group
    c = E.NativeCodec(s, 1, False)
    o = orc.codec(t, k, m, r, 4096, 1)
    assert np.array_equal(c.getEncodeMatrix(), o.encode_matrix())
    assert np.array_equal(c.getEncodeGftbl(), o.encode_gftbl())
    ones = orc.init_tables(c.decodeDataNum, 1, np.ones(c.decodeDataNum, np.uint8))
    assert np.array_equal(c.getDecodeGftbl(), ones)


def test_matrices_vs_golden(manifest):
    for key, hexv in manifest["matrices"].items():
        kind, a, b = key.split("_")
        if kind != "cauchy":
            continue
        c = E.NativeCodec.getRsCodec(E.CodingScheme.getRsScheme(int(a), int(b), 64))
        assert c.getEncodeMatrix().tobytes().hex() == hexv, key


def test_paper_stripe_geometry():
    """(n,k,r,z) = (136,128,27,34) CL: 5 groups, 34+1 racks of 4 (paper p.238)."""
    s = E.CodingScheme.getClScheme(128, 3, 27, 1 << 26)
    c = E.NativeCodec.getClCodec(s, 1, False)
    assert (s.groupNum, s.rackNodesNum, s.rackNum) == (5, 4, 35)
    assert (c.decodeDataNum, c.partialDecodeNum, c.rackPerGroup) == (9, 4, 7)
    assert c.repairSources(0) == list(range(1, 27)) + [131]
    assert c.repairSources(135) == list(range(108, 128))  # last local parity: its 20 data blocks
    assert c.repairSources(127) == list(range(108, 127)) + [135]


def test_errors():
    s = E.CodingScheme.getClScheme(8, 2, 4, 64)
    with pytest.raises(E.EcwError):
        E.NativeCodec(s, 0, False)  # node indices are 1-based
    with pytest.raises(E.EcwError):
        E.CodingScheme.getClScheme(250, 7, 10, 64)  # k + m > 256
    with pytest.raises(E.EcwError):
        E.NativeCodec.getRsCodec(E.CodingScheme.getRsScheme(4, 2, 64)).repairSources(0)  # no local groups
    c = E.NativeCodec(s, 1, True)  # multi-node: node 1 holds the last group
    assert (c.encodeDataNum, c.parityNum) == (4, 3)
    with pytest.raises(E.EcwError):
        E.NativeCodec(s, 3, True)  # only groupNum (= 2) encode nodes exist


def test_multinode_matrix_columns(orc):
    """Node i's partial-parity matrix = columns of group g-i of the stripe's
    Cauchy rows (ClMetadataManager.getMultinodeEncodeTask runs nodes 1..g)."""
    k, m, r = 32, 3, 11
    s = E.CodingScheme.getClScheme(k, m, r, 64)
    full = orc.cauchy1(k + m, k)[k:]
    g = s.groupNum
    cols = []
    for node in range(1, g + 1):
        c = E.NativeCodec(s, node, True)
        c0 = (g - node) * r
        assert c.encodeDataNum == (k - c0 if node == 1 else r)
        mat = c.getEncodeMatrix().reshape(m, c.encodeDataNum)
        assert np.array_equal(mat, full[:, c0:c0 + c.encodeDataNum])
        cols += list(range(c0, c0 + c.encodeDataNum))
    assert sorted(cols) == list(range(k))


@pytest.mark.skipif(E.device_count() > 0, reason="checks the no-GPU failure mode")
def test_device_calls_fail_loudly_without_gpu():
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(4, 2, 2, 64), 1, False)
    with pytest.raises(E.EcwError) as ei:
        c.encodeData([np.zeros(64, np.uint8)] * 4, [np.zeros(64, np.uint8)] * 4)
    assert ei.value.status == -3


@pytest.mark.skipif(E.device_count() > 0, reason="checks the no-GPU failure mode")
def test_small_host_xors_fail_loudly_without_gpu():
    """The small host XORs (decodeData, partialDecodeData, repairBlock) that
    the request service takes on a GPU report ECW_EDEVICE here, never a CPU
    result; the service counters stay zero and the service is not off."""
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(8, 2, 4, 4096), 1, False)
    for call in (lambda: c.decodeData([np.zeros(4096, np.uint8)] * c.decodeDataNum, np.zeros(4096, np.uint8)),
                 lambda: c.partialDecodeData([np.zeros(4096, np.uint8)] * c.partialDecodeNum, np.zeros(4096, np.uint8)),
                 lambda: c.repairBlock([np.zeros(4096, np.uint8)] * (8 + c.parityNum), 0, np.zeros(4096, np.uint8))):
        with pytest.raises(E.EcwError) as ei:
            call()
        assert ei.value.status == -3
    assert E.service_counters(0) == {"served": 0, "declined": 0, "epochs": 0, "broken": False}
    assert _lib.lib.ecw_service_counters(-1, (ctypes.c_uint64 * 4)()) == -1


def test_status_strings():
    for st in range(0, -8, -1):
        assert _lib.lib.ecw_status_string(st)


def test_chunk_generator_names():
    """generateChunks naming (ChunkGenerator.java:59-103) for the default
    scheme: toy names carry the 1-based node position of the CL layout."""
    from ecwide_amd.chunk_generator import chunk_file_names

    s = E.CodingScheme.fromConfigText(DEFAULT_INI)
    toy = chunk_file_names(s, -1)
    assert len(toy) == 32 + 3 + 3
    assert toy[:3] == ["1_D_0", "2_D_1", "3_D_2"]
    assert toy[10:13] == ["11_D_10", "13_D_11", "14_D_12"]  # group boundary skips L's position
    assert toy[31] == "34_D_31"
    assert toy[32:35] == ["36_G_0", "37_G_1", "38_G_2"]
    assert toy[35:] == ["12_L_0", "24_L_1", "35_L_2"]
    st = chunk_file_names(s, 7)
    assert st[0] == "D_7_0" and st[32] == "G_7_0" and st[-1] == "L_7_2"
    rs = chunk_file_names(E.CodingScheme.getRsScheme(4, 2, 64), -1)
    assert rs == ["1_D_0", "2_D_1", "3_D_2", "4_D_3", "5_G_0", "6_G_1"]


# ---- launch schedule (ecw_set_schedule): set / get / validation, no launch ----
def test_schedule_set_get_roundtrip():
    prev = E.set_schedule()
    try:
        assert E.get_schedule() == {f: -1 for f in E.codec.SCHEDULE_FIELDS}
        E.set_schedule(xor_skew=2, xor_order=1, xor_window_width=32, xcd_remap=1)
        got = E.get_schedule()
        # a window with only the width given takes the default period (2^11)
        assert got == dict(xor_skew=2, xor_order=1, xor_window_log2p=11, xor_window_width=32,
                           enc_window_log2p=-1, enc_window_width=-1, xcd_remap=1)
        E.set_schedule(enc_window_log2p=10)  # only the period: the default width (64)
        assert (E.get_schedule()["enc_window_log2p"], E.get_schedule()["enc_window_width"]) == (10, 64)
        assert _lib.lib.ecw_set_schedule(None) == 0
        assert E.get_schedule() == {f: -1 for f in E.codec.SCHEDULE_FIELDS}
    finally:
        E.set_schedule(**{k: v for k, v in prev.items() if v != -1})


@pytest.mark.parametrize("bad", [dict(xor_skew=3), dict(xor_skew=8), dict(xor_skew=0), dict(xor_order=2),
                                 dict(xor_window_log2p=3), dict(enc_window_log2p=25), dict(xcd_remap=2),
                                 dict(enc_window_width=-5)])
def test_schedule_rejects_out_of_range(bad):
    """a skew the library was not built with (or any value out of
    range) is refused with ECW_EINVAL and changes nothing -- never silently
    run as K = 1."""
    E.set_schedule(xor_skew=4)
    try:
        with pytest.raises(E.EcwError):
            E.set_schedule(**bad)
        assert E.get_schedule()["xor_skew"] == 4
    finally:
        E.set_schedule()


def test_parse_schedule_strings():
    assert E.parse_schedule(xor="2,1") == dict(xor_skew=2, xor_order=1, xor_window_width=0)
    assert E.parse_schedule(xor="4,0,10,32") == dict(xor_skew=4, xor_order=0, xor_window_log2p=10,
                                                     xor_window_width=32)
    assert E.parse_schedule(window="off", remap="1") == dict(enc_window_width=0, xcd_remap=1)
    assert E.parse_schedule(window="12,128") == dict(enc_window_log2p=12, enc_window_width=128)
    assert E.parse_schedule(xor="auto", window=None) == {}


def test_schedule_seeded_from_environment_once():
    """The environment seeds the schedule once (a fresh process); malformed
    values are reported and ignored."""
    import subprocess
    import sys

    code = ("import ecwide_amd as E, os; print(E.get_schedule()); os.environ['ECW_XCD_REMAP'] = '0'; "
            "print(E.get_schedule())")
    env = dict(os.environ, ECW_XOR_SCHED="2,1,10,32", ECW_WRITE_WINDOW="off", ECW_XCD_REMAP="1")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    first, second = [eval(x) for x in out.stdout.strip().splitlines()]
    assert first == dict(xor_skew=2, xor_order=1, xor_window_log2p=10, xor_window_width=32,
                         enc_window_log2p=-1, enc_window_width=0, xcd_remap=1)
    assert second == first  # read once: a later setenv changes nothing
    env = dict(os.environ, ECW_XOR_SCHED="3,0", ECW_WRITE_WINDOW="bogus")
    out = subprocess.run([sys.executable, "-c", "import ecwide_amd as E; print(E.get_schedule())"], env=env,
                         capture_output=True, text=True, check=True,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert eval(out.stdout.strip()) == {f: -1 for f in E.codec.SCHEDULE_FIELDS}
    assert "ECW_XOR_SCHED" in out.stderr and "ECW_WRITE_WINDOW" in out.stderr


def test_host_alloc_without_gpu_fails_cleanly():
    """ecw_host_alloc / ecw_host_free / ecw_device_numa_node on a host without
    a GPU: status codes, no crash, nothing leaked or mapped."""
    from ctypes import byref, c_int, c_void_p

    p, node = c_void_p(), c_int(7)
    assert _lib.lib.ecw_host_alloc(0, 1 << 20, byref(p), byref(node)) == -3  # ECW_EDEVICE
    assert p.value is None and node.value == -1
    assert _lib.lib.ecw_host_alloc(0, 0, byref(p), None) == -1  # ECW_EINVAL
    assert _lib.lib.ecw_host_free(None) == 0
    assert _lib.lib.ecw_host_free(c_void_p(4096)) == -1  # not ours
    assert _lib.lib.ecw_device_numa_node(0) == -1
    assert _lib.lib.ecw_host_alloc_node(0, 2000, 4096, byref(p), None) == -1  # node out of range
    assert _lib.lib.ecw_host_alloc_node(0, -1, 4096, byref(p), byref(node)) == -3
    with pytest.raises(E.EcwError):
        E.PinnedHost(4096)
    with pytest.raises(E.EcwError):
        E.PinnedHost(4096, node=0)

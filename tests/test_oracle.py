"""Pin the oracle (our C restatement) to the reference's own arithmetic.

The golden vectors were produced by tests/golden/gen_golden.py from
oracle/_ref (ISA-L 2.14.0 ec_base.c compiled from the reference tarball).
Where oracle/_ref is present (this container) it is also checked directly.
"""
import hashlib

import numpy as np
import pytest

import oracle
from conftest import golden_blocks


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def mix64(z):
    z = np.uint64(z)
    z ^= z >> np.uint64(30)
    z *= np.uint64(0xBF58476D1CE4E5B9)
    z ^= z >> np.uint64(27)
    z *= np.uint64(0x94D049BB133111EB)
    z ^= z >> np.uint64(31)
    return z


def np_fill(length, seed, stripe, block):
    """Independent numpy statement of the ecwide.h counter PRNG."""
    G = np.uint64(0x9E3779B97F4A7C15)
    with np.errstate(over="ignore"):
        key = mix64(np.uint64(seed) + G * np.uint64(1 + stripe * 65536 + block))
        w = np.arange((length + 7) // 8, dtype=np.uint64)
        z = key + w * G
        z ^= z >> np.uint64(30)
        z *= np.uint64(0xBF58476D1CE4E5B9)
        z ^= z >> np.uint64(27)
        z *= np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return z.view(np.uint8)[:length]


@pytest.mark.parametrize("length,seed,stripe,block", [(1, 1, 0, 0), (17, 3, 2, 5), (4096, 9, 7, 127),
                                                      (1000, 2**40 + 5, 1000, 300)])
def test_prng_matches_numpy(orc, length, seed, stripe, block):
    assert np.array_equal(orc.fill(length, seed, stripe, block), np_fill(length, seed, stripe, block))


def test_gf_tables(orc, manifest):
    mul = np.array([[orc.gf_mul(a, b) for b in range(256)] for a in range(256)], np.uint8)
    assert sha(mul) == manifest["gf"]["mul_sha256"]
    inv = bytes(orc.gf_inv(a) for a in range(256))
    assert inv.hex() == manifest["gf"]["inv"]


def test_matrices(orc, manifest):
    for key, hexv in manifest["matrices"].items():
        kind, a, b = key.split("_")
        a, b = int(a), int(b)
        if kind == "cauchy":
            got = orc.cauchy1(a + b, a)[a:]
        else:
            got = orc.rs_matrix(a, b)
        assert got.tobytes().hex() == hexv, key


def test_tables(orc, manifest):
    t = manifest["tables"]
    for k, m in [(32, 3), (32, 2), (128, 3)]:
        mat = orc.cauchy1(k + m, k)[k:]
        assert sha(orc.init_tables(k, m, mat)) == t[f"gftbl_{k}_{m}"]
    mat = orc.cauchy1(6, 4)[4:]
    assert orc.init_tables(4, 2, mat).tobytes().hex() == t["gftbl_4_2_hex"]


def test_codec_encode_golden(orc, manifest):
    for e in manifest["encode"]:
        c = orc.codec(e["code_type"], e["k"], e["m"], max(e["r"], 1) if e["code_type"] in "CL" else e["r"], e["len"])
        f = e["fields"]
        assert c.encode_data_num == f["edn"] and c.decode_data_num == f["ddn"], e["name"]
        assert c.partial_decode_num == f["pdn"] and c.group_num == f["group_num"], e["name"]
        data = [orc.fill(e["len"], e["seed"], 0, j) for j in range(e["k"])]
        for avx2 in (False, True):
            got = c.encode(data, literal=False, avx2=avx2)
            want = golden_blocks(e["xor"], len(got), e["len"])
            for i, (g, w) in enumerate(zip(got, want)):
                assert np.array_equal(g, w), (e["name"], "xor", avx2, i)
            lit = c.encode(data, literal=True, avx2=avx2)
            assert [sha(x) for x in lit] == e["literal_sha256"], (e["name"], "literal", avx2)
        if e["code_type"] in "CL":
            lit = c.encode(data, literal=True)
            assert all(not x.any() for x in lit[e["m"]:]), "ECWide-C literal L blocks must be zero"


def test_codec_threaded_matches(orc):
    c = orc.codec("C", 32, 3, 11, 1 << 16)
    data = [orc.fill(1 << 16, 5, 0, j) for j in range(32)]
    a = c.encode(data, avx2=False)
    b = c.encode(data, threads=4)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))


def test_xor_reduce_golden(orc, manifest):
    for e in manifest["xor_reduce"]:
        data = [orc.fill(e["len"], e["seed"], 0, j) for j in range(e["n"])]
        want = golden_blocks(e, 1, e["len"])[0]
        assert np.array_equal(orc.xor_blocks(data), want)
        c = orc.codec("R", e["n"], 1, -1, e["len"])  # decodeDataNum = k for RS: all-ones table XOR
        assert np.array_equal(c.decode(data), want)


def test_xor_intermediate_quirk(orc, manifest):
    e = manifest["xor_intermediate"]
    m, ln = e["m"], e["len"]
    s1, s2, s3 = e["seeds"]
    src1 = [orc.fill(ln, s1, 0, j) for j in range(m)]
    tgt = [orc.fill(ln, s2, 0, j) for j in range(m)]
    src2 = [orc.fill(ln, s3, 0, j) for j in range(m)]
    c = orc.codec("C", 8, m, 4, ln)
    c.xor_intermediate(src1, tgt, literal=True)
    assert [sha(x) for x in tgt] == e["first"]
    assert all(not x.any() for x in tgt)
    c.xor_intermediate(src2, tgt, literal=True)
    want = golden_blocks(e["second"], m, ln)
    assert all(np.array_equal(a, b) for a, b in zip(tgt, want))


def test_ecwide_h_wrappers(orc, manifest):
    h = manifest["ecwide_h"]
    ld = [orc.fill(4096, 41, 0, j) for j in range(11)]
    assert np.array_equal(orc.xor_blocks(ld), golden_blocks(h["l_encode"], 1, 4096)[0])
    gd = [orc.fill(4096, 42, 0, j) for j in range(11)]
    mat = orc.cauchy1(14, 11)[11:]
    got = orc.encode_data(orc.init_tables(11, 3, mat), gd, 3)
    assert all(np.array_equal(a, b) for a, b in zip(got, golden_blocks(h["g_encode"], 3, 4096)))
    md = [orc.fill(4096, 43, 0, j) for j in range(4)]
    assert np.array_equal(orc.xor_blocks(md), golden_blocks(h["l_middle"], 1, 4096)[0])
    dd = [orc.fill(4096, 44, 0, j) for j in range(5)]
    assert np.array_equal(orc.xor_blocks(dd), golden_blocks(h["l_decode"], 1, 4096)[0])


@pytest.mark.skipif(not oracle.have_ref(), reason="oracle/_ref not built here")
def test_oracle_vs_ref_random_sweep(orc):
    ref = oracle.RefIsal()
    rng = np.random.default_rng(11)  # ISA-L's own TEST_SEED
    for _ in range(40):
        k = int(rng.integers(1, 60))
        m = int(rng.integers(1, 12))
        ln = int(rng.integers(1, 700))
        mat = ref.cauchy1(k + m, k)
        assert np.array_equal(mat, orc.cauchy1(k + m, k))
        tb = ref.init_tables(k, m, mat[k:])
        assert np.array_equal(tb, orc.init_tables(k, m, mat[k:]))
        data = [rng.integers(0, 256, ln, dtype=np.uint8) for _ in range(k)]
        want = ref.encode_data(tb, data, m)
        for avx2 in (False, True):
            got = orc.encode_data(tb, data, m, avx2=avx2)
            assert all(np.array_equal(a, b) for a, b in zip(got, want)), (k, m, ln, avx2)


# ---- ISA-L master's kernel families (the CPU baseline as ECWide-C builds it) ----
def test_gfni_matrix_is_gf_mul(orc):
    """The 8x8 GF(2) matrix of x -> c*x in vgf2p8affineqb's layout, checked
    through the scalar model of the instruction for every (c, x)."""
    rng = np.random.default_rng(3)
    for c in range(256):
        m = orc.L.orc_gfni_matrix(c)
        for x in rng.integers(0, 256, 24):
            assert orc.L.orc_gfni_affine_byte(m, int(x)) == orc.gf_mul(c, int(x)), (c, int(x))
        assert orc.L.orc_gfni_affine_byte(m, 1) == c and orc.L.orc_gfni_affine_byte(m, 0) == 0


@pytest.mark.skipif(not oracle.have_ref(), reason="oracle/_ref not built here")
@pytest.mark.parametrize("kind", ["base", "avx2", "avx512", "gfni"])
def test_kernel_families_vs_ref_random_sweep(orc, kind):
    """Every family's ec_encode_data, with its own table format, equals the
    reference's ec_encode_data_base (oracle/_ref) byte for byte; lengths
    cover the < 64 scalar path, the overlapped last vector and several
    threads. On a CPU without the ISA the scalar model runs (and says so)."""
    ref = oracle.RefIsal()
    rng = np.random.default_rng(11)
    for it in range(40):
        k = int(rng.integers(1, 60))
        m = int(rng.integers(1, 14))
        ln = int(rng.integers(1, 1500)) if it % 4 else int(rng.integers(8192, 20000))
        mat = ref.cauchy1(k + m, k)[k:]
        data = [rng.integers(0, 256, ln, dtype=np.uint8) for _ in range(k)]
        want = ref.encode_data(ref.init_tables(k, m, mat), data, m)
        tb = orc.init_tables_kind(kind, k, m, mat)
        for threads in (1, 3):
            got = orc.encode_data_kind(kind, tb, data, m, threads=threads)
            assert all(np.array_equal(a, b) for a, b in zip(got, want)), (kind, k, m, ln, threads)


@pytest.mark.parametrize("kind", ["avx512", "gfni"])
def test_codec_encode_golden_kernel_families(orc, manifest, kind):
    """The whole encodeData flow (global rows + per-group passes, XOR and
    literal modes) on the AVX-512 / GFNI families against the golden
    vectors made from oracle/_ref."""
    for e in manifest["encode"]:
        c = orc.codec(e["code_type"], e["k"], e["m"], max(e["r"], 1) if e["code_type"] in "CL" else e["r"], e["len"])
        data = [orc.fill(e["len"], e["seed"], 0, j) for j in range(e["k"])]
        got = c.encode(data, kind=kind)
        want = golden_blocks(e["xor"], len(got), e["len"])
        assert all(np.array_equal(g, w) for g, w in zip(got, want)), (e["name"], kind)
        assert [sha(x) for x in c.encode(data, literal=True, kind=kind, threads=2)] == e["literal_sha256"]


def test_isal_master_dispatch_rule(orc):
    """ISA-L master picks AVX-512 + GFNI, else AVX-512, else AVX2, else base."""
    order = [x for x in ("gfni", "avx512", "avx2") if orc.have_kind(x)]
    assert orc.isal_master_kind() == (order[0] if order else "base")

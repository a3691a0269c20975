"""libecw_isal.so: the ISA-L erasure-code API (isal:include/erasure_code.h)
served by the MI355X engine — ECWide-H's ISA-L call sites and NativeCodec.cc
can link it instead of libisal."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
from conftest import REPO, golden_blocks

SHIM = os.path.join(REPO, "ecwide_amd", "libecw_isal.so")
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u8pp = ctypes.POINTER(_u8p)


@pytest.fixture(scope="module")
def shim():
    return load_shim()


def load_shim():
    import ecwide_amd  # noqa: F401  (torch-first runtime order, then the engine)

    L = ctypes.CDLL(SHIM)
    L.gf_mul.restype = ctypes.c_uint8
    L.gf_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
    L.gf_inv.restype = ctypes.c_uint8
    L.gf_inv.argtypes = [ctypes.c_uint8]
    L.gf_gen_rs_matrix.argtypes = [_u8p, ctypes.c_int, ctypes.c_int]
    L.gf_gen_cauchy1_matrix.argtypes = [_u8p, ctypes.c_int, ctypes.c_int]
    L.gf_invert_matrix.argtypes = [_u8p, _u8p, ctypes.c_int]
    L.gf_invert_matrix.restype = ctypes.c_int
    L.ec_init_tables.argtypes = [ctypes.c_int, ctypes.c_int, _u8p, _u8p]
    L.ec_encode_data.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p, _u8pp, _u8pp]
    L.ecw_isal_last_status.restype = ctypes.c_int
    return L


def p(a):
    return a.ctypes.data_as(_u8p)


def pp(arrs):
    return (_u8p * len(arrs))(*[p(a) for a in arrs])


def test_pure_functions_vs_reference_arithmetic(shim, orc, manifest):
    for a in range(0, 256, 7):
        for b in range(0, 256, 5):
            assert shim.gf_mul(a, b) == orc.gf_mul(a, b)
    assert bytes(shim.gf_inv(a) for a in range(256)).hex() == manifest["gf"]["inv"]
    for key, hexv in manifest["matrices"].items():
        kind, a, b = key.split("_")
        a, b = int(a), int(b)
        if kind == "cauchy":
            m = np.zeros((a + b) * a, np.uint8)
            shim.gf_gen_cauchy1_matrix(p(m), a + b, a)
            assert m[a * a:].tobytes().hex() == hexv
        else:
            m = np.zeros(a * b, np.uint8)
            shim.gf_gen_rs_matrix(p(m), a, b)
            assert m.tobytes().hex() == hexv
    mat = orc.cauchy1(6, 4)[4:].copy()
    t = np.zeros(32 * 8, np.uint8)
    shim.ec_init_tables(4, 2, p(mat), p(t))
    assert t.tobytes().hex() == manifest["tables"]["gftbl_4_2_hex"]


def test_invert_matrix(shim, orc):
    rng = np.random.default_rng(11)
    for n in (1, 3, 8, 20):
        while True:
            a = rng.integers(0, 256, n * n, dtype=np.uint8)
            inv = np.zeros(n * n, np.uint8)
            if shim.gf_invert_matrix(p(a.copy()), p(inv), n) == 0:
                break
        # a * inv == I over GF(2^8)
        A, I = a.reshape(n, n), inv.reshape(n, n)
        for i in range(n):
            for j in range(n):
                s = 0
                for t in range(n):
                    s ^= orc.gf_mul(int(A[i, t]), int(I[t, j]))
                assert s == (1 if i == j else 0)
    z = np.zeros(4, np.uint8)
    assert shim.gf_invert_matrix(p(z), p(np.zeros(4, np.uint8)), 2) == -1


@pytest.mark.gpu
def test_ec_encode_data_and_erasure_roundtrip(shim, orc):
    """ISA-L's erasure_code_test pattern (seed 11): Cauchy and RS encode on
    the GPU vs the oracle, then erase m blocks, invert, decode, compare."""
    rng = np.random.default_rng(11)
    for trial in range(12):
        k = int(rng.integers(2, 40))
        m = int(rng.integers(1, 9))
        ln = int(rng.integers(1, 70000))
        n = k + m
        full = np.zeros(n * k, np.uint8)
        (shim.gf_gen_cauchy1_matrix if trial % 2 == 0 else shim.gf_gen_rs_matrix)(p(full), n, k)
        if trial % 2 and k > 8:
            continue  # RS (Vandermonde) rows are only guaranteed invertible for small k
        tbl = np.zeros(32 * k * m, np.uint8)
        shim.ec_init_tables(k, m, p(full[k * k:].copy()), p(tbl))
        data = [rng.integers(0, 256, ln, dtype=np.uint8) for _ in range(k)]
        par = [np.zeros(ln, np.uint8) for _ in range(m)]
        shim.ec_encode_data(ln, k, m, p(tbl), pp(data), pp(par))
        assert shim.ecw_isal_last_status() == 0
        want = orc.encode_data(tbl, data, m)
        assert all(np.array_equal(a, b) for a, b in zip(par, want)), (trial, k, m, ln)
        # erase m random blocks, keep k survivors, decode the erased data blocks
        blocks = data + par
        lost = sorted(rng.choice(n, size=m, replace=False).tolist())
        surv = [i for i in range(n) if i not in lost][:k]
        F = full.reshape(n, k)
        B = np.ascontiguousarray(F[surv]).reshape(-1).copy()
        Binv = np.zeros(k * k, np.uint8)
        assert shim.gf_invert_matrix(p(B), p(Binv), k) == 0
        lost_data = [i for i in lost if i < k]
        if not lost_data:
            continue
        D = np.ascontiguousarray(Binv.reshape(k, k)[lost_data]).reshape(-1).copy()
        dt = np.zeros(32 * k * len(lost_data), np.uint8)
        shim.ec_init_tables(k, len(lost_data), p(D), p(dt))
        rec = [np.zeros(ln, np.uint8) for _ in lost_data]
        shim.ec_encode_data(ln, k, len(lost_data), p(dt), pp([blocks[i] for i in surv]), pp(rec))
        for r_, i in zip(rec, lost_data):
            assert np.array_equal(r_, data[i]), (trial, i)


@pytest.mark.gpu
def test_ecwide_h_call_sequence_binary(manifest):
    """A C program replaying ECWide-H's exact ISA-L calls (encode.cpp:113-238),
    linked against libecw_isal.so, reproduces the reference's outputs."""
    exe = os.path.join(REPO, "tests", "csrc", "ecwide_h_calls")
    src = exe + ".c"
    if not os.path.exists(exe) or os.path.getmtime(exe) < os.path.getmtime(src):
        subprocess.run(["gcc", "-O2", "-o", exe, src, "-L" + os.path.join(REPO, "ecwide_amd"), "-lecw_isal",
                        "-Wl,-rpath," + os.path.join(REPO, "ecwide_amd")], check=True)
    out = subprocess.run([exe], check=True, capture_output=True, timeout=300).stdout
    h = manifest["ecwide_h"]
    want = b"".join(np.concatenate(golden_blocks(h[key], n, 4096)).tobytes()
                    for key, n in [("l_encode", 1), ("g_encode", 3), ("l_middle", 1), ("l_decode", 1)])
    assert out == want


@pytest.mark.gpu
@pytest.mark.parametrize("S", [10, 300, 1000])
def test_encode_stripes_batch(orc, S):
    """ecw_encode_stripes: independent 4 KiB CL stripes in one call -- 10
    (0.7 MiB packed image: zero-copy), 300 (one DMA batch), 1000 (three
    double-buffered DMA batches of <= 32 MiB)."""
    import ecwide_amd as E
    from ecwide_amd._lib import lib

    k, m, r, ln = 11, 3, 4, 4096
    c = E.NativeCodec.getClCodec(E.CodingScheme.getClScheme(k, m, r, ln), 1, False)
    data = [[orc.fill(ln, 5, s, j) for j in range(k)] for s in range(S)]
    par = [[np.zeros(ln, np.uint8) for _ in range(c.parityNum)] for _ in range(S)]
    dptr = (ctypes.c_void_p * (S * k))(*[d.ctypes.data for row in data for d in row])
    pptr = (ctypes.c_void_p * (S * c.parityNum))(*[x.ctypes.data for row in par for x in row])
    assert lib.ecw_encode_stripes(c._h, S, dptr, pptr, ln) == 0
    oc = orc.codec("C", k, m, r, ln)
    for s in range(S):
        want = oc.encode(data[s])
        assert all(np.array_equal(a, b) for a, b in zip(par[s], want)), s


@pytest.mark.gpu
def test_ec_encode_data_concurrent_callers(shim, orc):
    """ECWide-H calls ec_encode_data from several proxy threads at once
    (proxy.cpp:2001-2012): each call is served on a slot of its own by the
    resident request service, and every caller gets exactly its own parities."""
    concurrent_callers(shim, orc)


@pytest.mark.gpu
def test_ec_encode_data_concurrent_callers_batched():
    """The same with the service off (ECW_SERVICE=0, read once per process, so
    in a child process): concurrent calls are group-committed into launches."""
    code = ("import sys; sys.path[:0] = [%r, %r]\n"
            "import ecwide_amd, oracle, test_isal_shim as t\n"
            "t.concurrent_callers(t.load_shim(), oracle.Oracle()); print('ok')\n") % (REPO, os.path.join(REPO, "tests"))
    env = dict(os.environ, ECW_SERVICE="0")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-3000:]


def concurrent_callers(shim, orc):
    import threading

    k, m = 11, 3
    full = np.zeros((k + m) * k, np.uint8)
    shim.gf_gen_cauchy1_matrix(p(full), k + m, k)
    tbl = np.zeros(32 * k * m, np.uint8)
    shim.ec_init_tables(k, m, p(full[k * k:].copy()), p(tbl))
    rng = np.random.default_rng(7)
    lens = [4096, 4096, 4096, 1000, 4096, 65536, 4096, 4096]
    jobs = [[[rng.integers(0, 256, ln, dtype=np.uint8) for _ in range(k)] for _ in range(25)] for ln in lens]
    outs = [[[np.zeros(ln, np.uint8) for _ in range(m)] for _ in range(25)] for ln in lens]
    errors = []

    def worker(t):
        for d, o in zip(jobs[t], outs[t]):
            shim.ec_encode_data(lens[t], k, m, p(tbl), pp(d), pp(o))
            if shim.ecw_isal_last_status() != 0:
                errors.append((t, shim.ecw_isal_last_status()))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(len(lens))]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not errors
    for t in range(len(lens)):
        for d, o in zip(jobs[t], outs[t]):
            want = orc.encode_data(tbl, d, m)
            assert all(np.array_equal(a, b) for a, b in zip(o, want)), t

"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes bindings for two CPU checkers:

* ``liboracle.so`` — our C restatement of the reference path
  (oracle/ecw_oracle.c; every function there cites the reference file:line
  it restates);
* ``_ref/libisal_base.so`` — the reference's own arithmetic: ISA-L 2.14.0
  ``erasure_code/ec_base.c`` + ``ec_highlevel_func.c`` (``ec_init_tables``)
  compiled unmodified from the tarball that
  ECWide-H bundles (oracle/Makefile). Present wherever ``build()`` ran in a
  container that has /root/reference; the prebuilt .so travels to the GPU box.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
may import this package. The product (ecwide_amd) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_char, c_int, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libisal_base.so")

_u8p = POINTER(c_uint8)
_u8pp = POINTER(_u8p)


def build() -> None:
    """Compile liboracle.so (and _ref when the reference is present)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _ptrs(arrs):
    a = (_u8p * len(arrs))()
    for i, x in enumerate(arrs):
        assert x.dtype == np.uint8 and x.flags["C_CONTIGUOUS"]
        a[i] = x.ctypes.data_as(_u8p)
    return a


class Oracle:
    """Our C restatement (liboracle.so)."""

    def __init__(self, path: str = LIB_PATH):
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        self.L = L
        L.orc_gf_mul.restype = c_uint8
        L.orc_gf_mul.argtypes = [c_uint8, c_uint8]
        L.orc_gf_inv.restype = c_uint8
        L.orc_gf_inv.argtypes = [c_uint8]
        L.orc_gen_cauchy1_matrix.argtypes = [_u8p, c_int, c_int]
        L.orc_gen_rs_matrix.argtypes = [_u8p, c_int, c_int]
        L.orc_init_tables.argtypes = [c_int, c_int, _u8p, _u8p]
        for f in (L.orc_encode_data_base, L.orc_encode_data_avx2):
            f.argtypes = [c_int, c_int, c_int, _u8p, _u8pp, _u8pp]
        L.orc_encode_data_avx2_mt.argtypes = [c_int, c_int, c_int, _u8p, _u8pp, _u8pp, c_int]
        L.orc_codec_new.restype = c_void_p
        L.orc_codec_new.argtypes = [c_char, c_int, c_int, c_int, c_int, c_int, c_int]
        L.orc_codec_free.argtypes = [c_void_p]
        L.orc_codec_field.argtypes = [c_void_p, c_int]
        L.orc_codec_matrix.restype = _u8p
        L.orc_codec_matrix.argtypes = [c_void_p]
        L.orc_codec_gftbl.restype = _u8p
        L.orc_codec_gftbl.argtypes = [c_void_p]
        L.orc_nc_encode_len.argtypes = [c_void_p, _u8pp, _u8pp, c_int, c_int, c_int]
        L.orc_nc_encode_mt.argtypes = [c_void_p, _u8pp, _u8pp, c_int, c_int, c_int]
        L.orc_nc_decode.argtypes = [c_void_p, _u8pp, _u8p, c_int]
        L.orc_nc_partial_decode.argtypes = [c_void_p, _u8pp, _u8p, c_int]
        L.orc_nc_xor_intermediate.argtypes = [c_void_p, _u8pp, _u8pp, c_int, c_int]
        L.orc_fill_random.argtypes = [_u8p, c_size_t, c_uint64, c_uint32, c_uint32]
        L.orc_fill_random_at.argtypes = [_u8p, c_size_t, c_size_t, c_uint64, c_uint32, c_uint32]
        L.orc_xor_blocks.argtypes = [_u8pp, c_int, _u8p, c_size_t]
        L.orc_have_avx2.restype = c_int
        # ISA-L master's kernel families (KINDS): the CPU baseline as ECWide-C builds it
        L.orc_encode_data_kind.argtypes = [c_int, c_int, c_int, c_int, _u8p, _u8pp, _u8pp]
        L.orc_encode_data_mt_kind.argtypes = [c_int, c_int, c_int, c_int, _u8p, _u8pp, _u8pp, c_int]
        L.orc_init_tables_kind.argtypes = [c_int, c_int, c_int, _u8p, _u8p]
        L.orc_nc_encode_kind.argtypes = [c_void_p, _u8pp, _u8pp, c_int, c_int, c_int]
        L.orc_nc_encode_mt_kind.argtypes = [c_void_p, _u8pp, _u8pp, c_int, c_int, c_int, c_int]
        L.orc_gfni_matrix.restype = c_uint64
        L.orc_gfni_matrix.argtypes = [c_uint8]
        L.orc_gfni_affine_byte.restype = c_uint8
        L.orc_gfni_affine_byte.argtypes = [c_uint64, c_uint8]
        L.orc_have_kind.argtypes = [c_int]
        L.orc_have_kind.restype = c_int
        L.orc_isal_master_kind.restype = c_int

    # -- arithmetic ----------------------------------------------------
    def gf_mul(self, a: int, b: int) -> int:
        return self.L.orc_gf_mul(a, b)

    def gf_inv(self, a: int) -> int:
        return self.L.orc_gf_inv(a)

    def cauchy1(self, n: int, k: int) -> np.ndarray:
        a = np.zeros(n * k, np.uint8)
        self.L.orc_gen_cauchy1_matrix(a.ctypes.data_as(_u8p), n, k)
        return a.reshape(n, k)

    def rs_matrix(self, n: int, k: int) -> np.ndarray:
        a = np.zeros(n * k, np.uint8)
        self.L.orc_gen_rs_matrix(a.ctypes.data_as(_u8p), n, k)
        return a.reshape(n, k)

    def init_tables(self, k: int, rows: int, a: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(a, np.uint8).reshape(-1)
        g = np.zeros(32 * k * rows, np.uint8)
        self.L.orc_init_tables(k, rows, a.ctypes.data_as(_u8p), g.ctypes.data_as(_u8p))
        return g

    def encode_data(self, tbls: np.ndarray, src: list, rows: int, avx2: bool = False):
        ln = src[0].size
        out = [np.zeros(ln, np.uint8) for _ in range(rows)]
        f = self.L.orc_encode_data_avx2 if avx2 else self.L.orc_encode_data_base
        f(ln, len(src), rows, tbls.ctypes.data_as(_u8p), _ptrs(src), _ptrs(out))
        return out

    def init_tables_kind(self, kind: str, k: int, rows: int, a: np.ndarray) -> np.ndarray:
        """ec_init_tables in kernel family `kind`'s format (32 B per coefficient,
        8 B for "gfni": ec_init_tables_gfni)."""
        a = np.ascontiguousarray(a, np.uint8).reshape(-1)
        g = np.zeros(32 * k * rows, np.uint8)
        self.L.orc_init_tables_kind(KINDS[kind], k, rows, a.ctypes.data_as(_u8p), g.ctypes.data_as(_u8p))
        return g

    def encode_data_kind(self, kind: str, tbls: np.ndarray, src: list, rows: int, threads: int = 1):
        ln = src[0].size
        out = [np.zeros(ln, np.uint8) for _ in range(rows)]
        self.L.orc_encode_data_mt_kind(KINDS[kind], ln, len(src), rows, tbls.ctypes.data_as(_u8p), _ptrs(src),
                                       _ptrs(out), threads)
        return out

    def have_kind(self, kind: str) -> bool:
        return bool(self.L.orc_have_kind(KINDS[kind]))

    def isal_master_kind(self) -> str:
        """The family ISA-L master's ec_encode_data dispatch picks on this CPU."""
        return {v: n for n, v in KINDS.items()}[self.L.orc_isal_master_kind()]

    def fill(self, length: int, seed: int, stripe: int, block: int, offset: int = 0) -> np.ndarray:
        """Bytes [offset, offset + length) of block `block` of stripe `stripe`
        (ecwide.h generator; offset a multiple of 8)."""
        assert offset % 8 == 0
        a = np.zeros(length, np.uint8)
        self.L.orc_fill_random_at(a.ctypes.data_as(_u8p), offset, length, seed, stripe, block)
        return a

    def xor_blocks(self, src: list) -> np.ndarray:
        out = np.zeros(src[0].size, np.uint8)
        self.L.orc_xor_blocks(_ptrs(src), len(src), out.ctypes.data_as(_u8p), out.size)
        return out

    def have_avx2(self) -> bool:
        return bool(self.L.orc_have_avx2())

    def codec(self, code_type: str, k: int, m: int, r: int, chunk: int, node: int = 1,
              multinode: bool = False) -> "OracleCodec":
        return OracleCodec(self, code_type, k, m, r, chunk, node, multinode)


# ec_encode_data kernel families: ISA-L 2.14's base and AVX2 (the tarball ECWide-H
# bundles), and ISA-L master's AVX-512 and AVX-512 + GFNI (what ECWide-C links)
KINDS = {"base": 0, "avx2": 1, "avx512": 2, "gfni": 3}

FIELDS = ("encode_data_num", "decode_data_num", "partial_decode_num", "group_num",
          "rack_nodes_num", "rack_num", "rack_per_group", "group_data_num")


class OracleCodec:
    """NativeCodec restated (ECWide-C/src/NativeCodec.java + native/NativeCodec.cc)."""

    def __init__(self, o: Oracle, code_type, k, m, r, chunk, node, multinode):
        self.o, self.L = o, o.L
        self.h = self.L.orc_codec_new(code_type.encode(), k, m, r, chunk, node, int(multinode))
        self.code_type, self.k, self.m, self.r, self.chunk = code_type, k, m, r, chunk
        for i, f in enumerate(FIELDS):
            setattr(self, f, self.L.orc_codec_field(self.h, i))
        self.parity_num = m + (self.group_num if code_type in "CL" else 0)

    def __del__(self):
        try:
            self.L.orc_codec_free(self.h)
        except Exception:
            pass

    def encode_matrix(self) -> np.ndarray:
        n = self.encode_data_num * self.m
        return np.ctypeslib.as_array(self.L.orc_codec_matrix(self.h), (n,)).copy()

    def encode_gftbl(self) -> np.ndarray:
        n = 32 * self.encode_data_num * self.m
        return np.ctypeslib.as_array(self.L.orc_codec_gftbl(self.h), (n,)).copy()

    def encode(self, data: list, literal: bool = False, avx2: bool = False, threads: int = 0,
               kind: str | None = None):
        ln = data[0].size
        par = [np.zeros(ln, np.uint8) for _ in range(self.parity_num)]
        if kind is not None:
            self.L.orc_nc_encode_mt_kind(self.h, _ptrs(data), _ptrs(par), int(literal), max(1, threads), ln,
                                         KINDS[kind])
        elif threads:
            self.L.orc_nc_encode_mt(self.h, _ptrs(data), _ptrs(par), int(literal), threads, ln)
        else:
            self.L.orc_nc_encode_len(self.h, _ptrs(data), _ptrs(par), int(literal), int(avx2), ln)
        return par

    def encode_into(self, dptrs, pptrs, ln: int, literal: bool = False, threads: int = 1, kind: str = "avx2"):
        """Raw-pointer form used by the bench's cpu_baseline leg."""
        self.L.orc_nc_encode_mt_kind(self.h, dptrs, pptrs, int(literal), threads, ln, KINDS[kind])

    def decode(self, data: list) -> np.ndarray:
        out = np.zeros(data[0].size, np.uint8)
        self.L.orc_nc_decode(self.h, _ptrs(data), out.ctypes.data_as(_u8p), out.size)
        return out

    def partial_decode(self, data: list) -> np.ndarray:
        out = np.zeros(data[0].size, np.uint8)
        self.L.orc_nc_partial_decode(self.h, _ptrs(data), out.ctypes.data_as(_u8p), out.size)
        return out

    def xor_intermediate(self, src: list, tgt: list, literal: bool = True) -> None:
        self.L.orc_nc_xor_intermediate(self.h, _ptrs(src), _ptrs(tgt), src[0].size, int(literal))


class RefIsal:
    """ISA-L 2.14.0 ec_base.c compiled from the reference tarball (oracle/_ref)."""

    def __init__(self, path: str = REF_PATH):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        # lazy binding: the SIMD dispatchers of ec_highlevel_func.c reference
        # NASM kernels that are not built (oracle/Makefile); never called here
        L = ctypes.CDLL(path, mode=os.RTLD_LAZY)
        self.L = L
        L.ec_init_tables.argtypes = [c_int, c_int, _u8p, _u8p]
        L.gf_mul.restype = c_uint8
        L.gf_mul.argtypes = [c_uint8, c_uint8]
        L.gf_inv.restype = c_uint8
        L.gf_inv.argtypes = [c_uint8]
        L.gf_gen_cauchy1_matrix.argtypes = [_u8p, c_int, c_int]
        L.gf_gen_rs_matrix.argtypes = [_u8p, c_int, c_int]
        L.gf_vect_mul_init.argtypes = [c_uint8, _u8p]
        L.ec_encode_data_base.argtypes = [c_int, c_int, c_int, _u8p, _u8pp, _u8pp]

    def cauchy1(self, n: int, k: int) -> np.ndarray:
        a = np.zeros(n * k, np.uint8)
        self.L.gf_gen_cauchy1_matrix(a.ctypes.data_as(_u8p), n, k)
        return a.reshape(n, k)

    def rs_matrix(self, n: int, k: int) -> np.ndarray:
        a = np.zeros(n * k, np.uint8)
        self.L.gf_gen_rs_matrix(a.ctypes.data_as(_u8p), n, k)
        return a.reshape(n, k)

    def init_tables(self, k: int, rows: int, a: np.ndarray) -> np.ndarray:
        """ec_init_tables (isal:erasure_code/ec_highlevel_func.c:33-43), the
        reference's own function."""
        a = np.ascontiguousarray(a, np.uint8).reshape(-1)
        g = np.zeros(32 * k * rows, np.uint8)
        self.L.ec_init_tables(k, rows, a.ctypes.data_as(_u8p), g.ctypes.data_as(_u8p))
        return g

    def encode_data(self, tbls: np.ndarray, src: list, rows: int):
        ln = src[0].size
        out = [np.zeros(ln, np.uint8) for _ in range(rows)]
        self.L.ec_encode_data_base(ln, len(src), rows, tbls.ctypes.data_as(_u8p), _ptrs(src),
                                   _ptrs(out))
        return out


def have_ref() -> bool:
    return os.path.exists(REF_PATH)

"""ctypes binding of libecwide.so (the C ABI declared in include/ecwide.h).

The shared library is the product: HIP kernels for gfx950 behind a plain C
ABI. Importing this module loads it and fails loudly (ImportError) when it is
missing; there is no fallback implementation.
"""
from __future__ import annotations

import ctypes
import os
import re
from ctypes import POINTER, Structure, c_char, c_char_p, c_int, c_size_t, c_uint8, c_uint64, c_void_p

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "libecwide.so")
HEADER = os.path.join(REPO, "include", "ecwide.h")


class ecw_scheme(Structure):
    _fields_ = [
        ("code_type", c_char),
        ("k", c_int),
        ("global_parity_num", c_int),
        ("group_data_num", c_int),
        ("group_num", c_int),
        ("rack_nodes_num", c_int),
        ("rack_num", c_int),
        ("chunk_size_bits", c_int),
        ("chunk_size", c_size_t),
    ]


class ecw_codec_info(Structure):
    _fields_ = [
        ("code_type", c_char),
        ("node_index", c_int),
        ("multinode", c_int),
        ("local_mode", c_int),
        ("encode_data_num", c_int),
        ("decode_data_num", c_int),
        ("partial_decode_num", c_int),
        ("global_num", c_int),
        ("group_num", c_int),
        ("group_data_num", c_int),
        ("rack_per_group", c_int),
        ("parity_num", c_int),
        ("chunk_size", c_size_t),
    ]


class ecw_schedule(Structure):
    _fields_ = [(name, c_int) for name in ("xor_skew", "xor_order", "xor_window_log2p", "xor_window_width",
                                           "enc_window_log2p", "enc_window_width", "xcd_remap")]


_u8p = POINTER(c_uint8)
_pp = POINTER(c_void_p)

# name -> (restype, argtypes)
SIGNATURES = {
    "ecw_abi_version": (c_int, []),
    "ecw_status_string": (c_char_p, [c_int]),
    "ecw_device_count": (c_int, []),
    "ecw_scheme_init": (c_int, [POINTER(ecw_scheme), c_char, c_int, c_int, c_int, c_size_t]),
    "ecw_scheme_from_ini": (c_int, [c_char_p, POINTER(ecw_scheme)]),
    "ecw_scheme_from_ini_text": (c_int, [c_char_p, POINTER(ecw_scheme)]),
    "ecw_codec_create": (c_int, [POINTER(ecw_scheme), c_int, c_int, c_int, c_int, POINTER(c_void_p)]),
    "ecw_codec_destroy": (None, [c_void_p]),
    "ecw_codec_get_info": (c_int, [c_void_p, POINTER(ecw_codec_info)]),
    "ecw_codec_set_xori_mode": (c_int, [c_void_p, c_int]),
    "ecw_codec_encode_matrix": (c_int, [c_void_p, _u8p, c_size_t]),
    "ecw_codec_encode_gftbl": (c_int, [c_void_p, _u8p, c_size_t]),
    "ecw_codec_decode_gftbl": (c_int, [c_void_p, _u8p, c_size_t]),
    "ecw_codec_partial_decode_gftbl": (c_int, [c_void_p, _u8p, c_size_t]),
    "ecw_encode": (c_int, [c_void_p, _pp, _pp, c_size_t]),
    "ecw_decode": (c_int, [c_void_p, _pp, c_void_p, c_size_t]),
    "ecw_partial_decode": (c_int, [c_void_p, _pp, c_void_p, c_size_t]),
    "ecw_xor_intermediate": (c_int, [c_void_p, _pp, _pp, c_size_t]),
    "ecw_repair": (c_int, [c_void_p, _pp, c_int, c_void_p, c_size_t]),
    "ecw_encode_stripes": (c_int, [c_void_p, c_int, _pp, _pp, c_size_t]),
    "ecw_matrix_codec_create": (c_int, [_u8p, c_int, c_int, c_int, POINTER(c_void_p)]),
    "ecw_encode_dev": (c_int, [c_void_p, _pp, _pp, c_size_t, c_void_p]),
    "ecw_encode_ptrs_dev": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
    "ecw_decode_dev": (c_int, [c_void_p, _pp, c_void_p, c_size_t, c_void_p]),
    "ecw_partial_decode_dev": (c_int, [c_void_p, _pp, c_void_p, c_size_t, c_void_p]),
    "ecw_xor_intermediate_dev": (c_int, [c_void_p, _pp, _pp, c_size_t, c_void_p]),
    "ecw_xor_reduce_dev": (c_int, [c_int, _pp, c_int, c_void_p, c_size_t, c_void_p]),
    "ecw_xor_reduce_ptrs_dev": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
    "ecw_encode_batch_dev": (c_int, [c_void_p, c_void_p, c_size_t, c_size_t, c_int, c_size_t, c_void_p]),
    "ecw_encode_batch_split_dev": (c_int, [c_void_p, c_void_p, c_size_t, c_size_t, c_void_p, c_size_t, c_size_t,
                                           c_int, c_size_t, c_void_p]),
    "ecw_repair_batch_split_dev": (c_int, [c_void_p, c_void_p, c_size_t, c_size_t, c_void_p, c_size_t, c_size_t,
                                           c_int, c_int, c_void_p, c_size_t, c_size_t, c_void_p]),
    "ecw_repair_batch_dev": (c_int, [c_void_p, c_void_p, c_size_t, c_size_t, c_int, c_int, c_void_p, c_size_t,
                                     c_size_t, c_void_p]),
    "ecw_repair_sources": (c_int, [c_void_p, c_int, POINTER(c_int), c_int]),
    "ecw_service_counters": (c_int, [c_int, POINTER(c_uint64)]),
    "ecw_set_schedule": (c_int, [POINTER(ecw_schedule)]),
    "ecw_host_alloc": (c_int, [c_int, c_size_t, POINTER(c_void_p), POINTER(c_int)]),
    "ecw_host_alloc_node": (c_int, [c_int, c_int, c_size_t, POINTER(c_void_p), POINTER(c_int)]),
    "ecw_host_free": (c_int, [c_void_p]),
    "ecw_device_numa_node": (c_int, [c_int]),
    "ecw_get_schedule": (c_int, [POINTER(ecw_schedule)]),
    "ecw_fill_random_dev": (c_int, [c_int, c_void_p, c_size_t, c_size_t, c_int, c_int, c_size_t, c_uint64, c_int,
                                    c_int, c_void_p]),
    "ecw_fill_random_pieces_dev": (c_int, [c_int, c_void_p, c_size_t, c_size_t, c_int, c_int, c_size_t, c_size_t,
                                           c_size_t, c_size_t, c_uint64, c_int, c_int, c_void_p]),
}


def header_symbols(path: str = HEADER) -> list:
    """Every function the C header declares (the export contract)."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ecw_[a-z0-9_]+)\s*\(", text)) - {"ecw_status"})


def _torch_runtime_first() -> None:
    """torch bundles its own libamdhip64.so.7 (same SONAME as /opt/rocm's).
    Whichever is loaded first serves the whole process, and torch does not
    see the GPU when it finds a different runtime already loaded. So when
    torch is installed it is imported first and libecwide.so binds to the
    runtime torch brought; C/C++ callers simply get /opt/rocm's."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load(path: str = LIB_PATH, strict: bool = True) -> ctypes.CDLL:
    """Load a libecwide.so build; strict=False skips entry points an older
    build (a tuning variant under build/) does not export."""
    _torch_runtime_first()
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the HIP extension is the only implementation)")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        if not strict and not hasattr(lib, name):
            continue
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = load()

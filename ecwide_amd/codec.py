"""Host-side mirror of ECWide-C's codec interface over the C ABI.

``CodingScheme`` mirrors ECWide-C/src/CodingScheme.java and ``NativeCodec``
mirrors ECWide-C/src/NativeCodec.java (same constructors/factories, field
names and method names: ``encodeData``, ``decodeData``,
``partialDecodeData``, ``xorIntemediate``). Buffers may be host numpy uint8
arrays (the reference's direct ByteBuffers; blocking host entry points) or
torch uint8 CUDA tensors resident in HBM (asynchronous device entry points on
the current torch stream).

Differences from the reference, all deliberate: every call validates its
arguments and raises ``EcwError`` instead of crashing; no static state is
shared between codecs; local parities are XOR by default (``local_mode``
"literal" reproduces ECWide-C's all-zero L blocks, NativeCodec.cc:181-186).
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_int, c_uint64, c_void_p

import numpy as np

from . import _lib
from ._lib import ecw_codec_info, ecw_scheme, lib

LOCAL_MODES = {"xor": 0, "literal": 1}
XORI_MODES = {"xor": 0, "literal": 1}


class EcwError(RuntimeError):
    def __init__(self, status: int, what: str):
        self.status = status
        super().__init__(f"{what}: {lib.ecw_status_string(status).decode()} ({status})")


def _check(st: int, what: str) -> int:
    if st < 0:
        raise EcwError(st, what)
    return st


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def _addr(x) -> int:
    if _is_torch(x):
        if x.dtype.itemsize != 1 or not x.is_contiguous():
            raise ValueError("device blocks must be contiguous uint8 tensors")
        return x.data_ptr()
    if not isinstance(x, np.ndarray) or x.dtype != np.uint8 or not x.flags["C_CONTIGUOUS"]:
        raise ValueError("host blocks must be C-contiguous numpy uint8 arrays")
    return x.ctypes.data


def _nbytes(x) -> int:
    return x.numel() if _is_torch(x) else x.size


def _parr(bufs) -> ctypes.Array:
    a = (c_void_p * max(1, len(bufs)))()
    for i, b in enumerate(bufs):
        a[i] = _addr(b)
    return a


def _on_device(bufs) -> bool:
    kinds = {(_is_torch(b) and b.is_cuda) for b in bufs}
    if len(kinds) != 1:
        raise ValueError("mixing host and device blocks in one call")
    return kinds.pop()


def _stream():
    import torch

    return c_void_p(torch.cuda.current_stream().cuda_stream)


class CodingScheme:
    """CodingScheme.java: k, m/globalParityNum, groupDataNum, groupNum,
    rackNodesNum, rackNum, chunkSize, codeType."""

    CODES = {"RS": b"R", "TL": b"T", "LRC": b"L", "CL": b"C"}

    def __init__(self, s: ecw_scheme):
        self._s = s
        self.codeType = {b"R": "RS", b"T": "TL", b"L": "LRC", b"C": "CL"}[s.code_type]
        self.k = s.k
        self.m = self.globalParityNum = s.global_parity_num
        self.groupDataNum = s.group_data_num
        self.groupNum = s.group_num
        self.rackNodesNum = s.rack_nodes_num
        self.rackNum = s.rack_num
        self.chunkSize = s.chunk_size
        self.chunkSizeBits = s.chunk_size_bits

    @classmethod
    def _make(cls, code: str, k: int, m: int, r: int, chunk: int) -> "CodingScheme":
        s = ecw_scheme()
        _check(lib.ecw_scheme_init(byref(s), cls.CODES[code], k, m, r, chunk), "CodingScheme")
        return cls(s)

    @classmethod
    def getRsScheme(cls, k, m, chunkSize):
        return cls._make("RS", k, m, -1, chunkSize)

    @classmethod
    def getTlScheme(cls, k, m, chunkSize):
        return cls._make("TL", k, m, -1, chunkSize)

    @classmethod
    def getLrcScheme(cls, k, m, groupDataNum, chunkSize):
        return cls._make("LRC", k, m, groupDataNum, chunkSize)

    @classmethod
    def getClScheme(cls, k, m, groupDataNum, chunkSize):
        return cls._make("CL", k, m, groupDataNum, chunkSize)

    @classmethod
    def getFromConfig(cls, path: str) -> "CodingScheme":
        s = ecw_scheme()
        _check(lib.ecw_scheme_from_ini(str(path).encode(), byref(s)), f"getFromConfig({path})")
        return cls(s)

    @classmethod
    def fromConfigText(cls, text: str) -> "CodingScheme":
        s = ecw_scheme()
        _check(lib.ecw_scheme_from_ini_text(text.encode(), byref(s)), "scheme.ini text")
        return cls(s)

    def __repr__(self):
        return (f"CodingScheme({self.codeType}, k={self.k}, m={self.m}, r={self.groupDataNum}, "
                f"chunkSize={self.chunkSize})")


class NativeCodec:
    """NativeCodec.java over libecwide.so."""

    def __init__(self, scheme: CodingScheme, nodeIndex: int = 1, multiNodeEncode: bool = False,
                 local_mode: str = "xor", device: int = 0):
        h = c_void_p()
        _check(lib.ecw_codec_create(byref(scheme._s), nodeIndex, int(multiNodeEncode),
                                    LOCAL_MODES[local_mode], device, byref(h)), "NativeCodec")
        self._h = h
        self.scheme = scheme
        self.device = device
        info = ecw_codec_info()
        _check(lib.ecw_codec_get_info(h, byref(info)), "info")
        self.codeType = info.code_type.decode()
        self.nodeIndex = info.node_index
        self.multiNodeEncode = bool(info.multinode)
        self.encodeDataNum = info.encode_data_num
        self.decodeDataNum = info.decode_data_num
        self.partialDecodeNum = info.partial_decode_num
        self.globalNum = info.global_num
        self.groupNum = info.group_num
        self.groupDataNum = info.group_data_num
        self.rackPerGroup = info.rack_per_group
        self.parityNum = info.parity_num
        self.chunkSize = info.chunk_size

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.ecw_codec_destroy(h)
            self._h = None

    # -- factories (NativeCodec.java:111-125) --------------------------------
    @classmethod
    def getRsCodec(cls, scheme, **kw):
        return cls(scheme, 1, False, **kw)

    @classmethod
    def getTlCodec(cls, scheme, nodeIndex, **kw):
        return cls(scheme, nodeIndex, False, **kw)

    @classmethod
    def getLrcCodec(cls, scheme, nodeIndex, **kw):
        return cls(scheme, nodeIndex, False, **kw)

    @classmethod
    def getClCodec(cls, scheme, nodeIndex, multiNodeEncode, **kw):
        return cls(scheme, nodeIndex, multiNodeEncode, **kw)

    # -- table getters (NativeCodec.java:127-143) ----------------------------
    def _get(self, fn, n):
        out = np.zeros(n, np.uint8)
        _check(fn(self._h, out.ctypes.data_as(_lib._u8p), n), fn.__name__)
        return out

    def getEncodeMatrix(self) -> np.ndarray:
        return self._get(lib.ecw_codec_encode_matrix, self.encodeDataNum * self.globalNum)

    def getEncodeGftbl(self) -> np.ndarray:
        return self._get(lib.ecw_codec_encode_gftbl, 32 * self.encodeDataNum * self.globalNum)

    def getDecodeGftbl(self) -> np.ndarray:
        return self._get(lib.ecw_codec_decode_gftbl, 32 * self.decodeDataNum)

    def getPartialDecodeGftbl(self) -> np.ndarray:
        return self._get(lib.ecw_codec_partial_decode_gftbl,
                         32 * self.partialDecodeNum if self.codeType in "TC" else 0)

    def setXorIntermediateMode(self, mode: str) -> None:
        _check(lib.ecw_codec_set_xori_mode(self._h, XORI_MODES[mode]), "xori mode")

    # -- the natives (NativeCodec.java:205-211) ------------------------------
    def _len(self, bufs, length):
        n = length if length is not None else min(_nbytes(b) for b in bufs)
        return n

    def encodeData(self, data, parity, length=None) -> None:
        if len(data) < self.encodeDataNum or len(parity) < self.parityNum:
            raise ValueError(f"need {self.encodeDataNum} data and {self.parityNum} parity blocks")
        data, parity = list(data[:self.encodeDataNum]), list(parity[:self.parityNum])
        n = self._len(data + parity, length)
        if _on_device(data + parity):
            _check(lib.ecw_encode_dev(self._h, _parr(data), _parr(parity), n, _stream()), "encodeData")
        else:
            _check(lib.ecw_encode(self._h, _parr(data), _parr(parity), n), "encodeData")

    def decodeData(self, data, target, length=None) -> None:
        data = list(data[:self.decodeDataNum])
        if len(data) < self.decodeDataNum:
            raise ValueError(f"need {self.decodeDataNum} blocks")
        n = self._len(data + [target], length)
        if _on_device(data + [target]):
            _check(lib.ecw_decode_dev(self._h, _parr(data), _addr(target), n, _stream()), "decodeData")
        else:
            _check(lib.ecw_decode(self._h, _parr(data), _addr(target), n), "decodeData")

    def partialDecodeData(self, data, target, length=None) -> None:
        data = list(data[:self.partialDecodeNum])
        if len(data) < self.partialDecodeNum:
            raise ValueError(f"need {self.partialDecodeNum} blocks")
        n = self._len(data + [target], length)
        if _on_device(data + [target]):
            _check(lib.ecw_partial_decode_dev(self._h, _parr(data), _addr(target), n, _stream()),
                   "partialDecodeData")
        else:
            _check(lib.ecw_partial_decode(self._h, _parr(data), _addr(target), n), "partialDecodeData")

    def xorIntemediate(self, source, target, length=None) -> None:
        source, target = list(source[:self.globalNum]), list(target[:self.globalNum])
        n = self._len(source + target, length)
        if _on_device(source + target):
            _check(lib.ecw_xor_intermediate_dev(self._h, _parr(source), _parr(target), n, _stream()),
                   "xorIntemediate")
        else:
            _check(lib.ecw_xor_intermediate(self._h, _parr(source), _parr(target), n), "xorIntemediate")

    def repairBlock(self, blocks, lost_block: int, out, length=None) -> None:
        """Flat CL repair of one block from a stripe's blocks ([D.., G.., L..]
        order; the lost entry may be None). Host buffers only."""
        srcs = self.repairSources(lost_block)
        n = length if length is not None else min(_nbytes(blocks[i]) for i in srcs)
        arr = (c_void_p * len(blocks))()
        for i, b in enumerate(blocks):
            arr[i] = _addr(b) if b is not None else None
        _check(lib.ecw_repair(self._h, arr, lost_block, _addr(out), n), "repairBlock")

    def encodeStripes(self, data, parity, length=None) -> None:
        """Encode a batch of stripes: data[s] / parity[s] are stripe s's block
        lists (the encodeData convention, NativeCodec.cc:158-166). HBM blocks
        go through ONE launch for the whole batch (ecw_encode_ptrs_dev, device
        pointer tables); host blocks through ecw_encode_stripes."""
        if not data:
            return
        if _on_device([b for st in data for b in st] + [b for st in parity for b in st]):
            BlockBatch(self, data, parity, length).encode()
            return
        k, np_ = self.encodeDataNum, self.parityNum
        flat_d = [b for st in data for b in list(st)[:k]]
        flat_p = [b for st in parity for b in list(st)[:np_]]
        if len(flat_d) != k * len(data) or len(flat_p) != np_ * len(data):
            raise ValueError(f"every stripe needs {k} data and {np_} parity blocks")
        n = self._len(flat_d + flat_p, length)
        _check(lib.ecw_encode_stripes(self._h, len(data), _parr(flat_d), _parr(flat_p), n), "encodeStripes")

    # -- CL repair fan-in (ClMetadataManager.java:137-257, flattened) --------
    def repairSources(self, lost_block: int) -> list:
        buf = (c_int * 256)()
        n = _check(lib.ecw_repair_sources(self._h, lost_block, buf, 256), "repairSources")
        return list(buf[:n])


class BlockBatch:
    """A batch of stripes whose blocks sit anywhere in HBM (separate
    allocations, the reference's per-block pointers): the block pointers are
    uploaded once as device tables, and every encode() of the batch is ONE
    kernel launch over all stripes (ecw_encode_ptrs_dev)."""

    def __init__(self, codec: NativeCodec, data, parity, length=None):
        import torch

        k, np_ = codec.encodeDataNum, codec.parityNum
        if len(data) != len(parity) or any(len(d) < k for d in data) or any(len(p) < np_ for p in parity):
            raise ValueError(f"every stripe needs {k} data and {np_} parity blocks")
        self.codec, self.stripes = codec, len(data)
        blocks = [b for st in data for b in list(st)[:k]] + [b for st in parity for b in list(st)[:np_]]
        if not _on_device(blocks):
            raise ValueError("BlockBatch holds HBM blocks (torch CUDA tensors)")
        self.len = codec._len(blocks, length)
        dev = blocks[0].device
        self._keep = blocks  # the blocks stay alive as long as their pointers are in the tables
        self.dtab = torch.tensor([_addr(b) for st in data for b in list(st)[:k]], dtype=torch.int64, device=dev)
        self.ptab = torch.tensor([_addr(b) for st in parity for b in list(st)[:np_]], dtype=torch.int64, device=dev)

    def encode(self, stream=None) -> None:
        _check(lib.ecw_encode_ptrs_dev(self.codec._h, self.stripes, c_void_p(self.dtab.data_ptr()),
                                       c_void_p(self.ptab.data_ptr()), self.len,
                                       stream if stream is not None else _stream()), "encodeStripes")

    def encode_bytes(self) -> int:
        return self.stripes * (self.codec.encodeDataNum + self.codec.parityNum) * self.len

    def repair(self, lost_block: int, out, stream=None) -> None:
        """CL single-block repair of `lost_block` (stripe block index: D_j = j,
        L_t = k + m + t) of every stripe into out[s] (HBM tensors), as the XOR of
        its surviving group members (ecw_repair_sources), one launch for the
        batch (ecw_xor_reduce_ptrs_dev)."""
        import torch

        if len(out) != self.stripes:
            raise ValueError(f"need {self.stripes} output blocks")
        k = self.codec.encodeDataNum
        srcs = self.codec.repairSources(lost_block)
        key = (lost_block, tuple(_addr(o) for o in out))
        if getattr(self, "_rkey", None) != key:
            blocks = [self._keep[s * k:(s + 1) * k] + self._keep[self.stripes * k + s * self.codec.parityNum:
                                                                 self.stripes * k + (s + 1) * self.codec.parityNum]
                      for s in range(self.stripes)]
            dev = self.dtab.device
            self._rsrc = torch.tensor([_addr(blocks[s][i]) for s in range(self.stripes) for i in srcs],
                                      dtype=torch.int64, device=dev)
            self._rdst = torch.tensor([_addr(o) for o in out], dtype=torch.int64, device=dev)
            self._rkeep, self._rkey = list(out), key
        _check(lib.ecw_xor_reduce_ptrs_dev(self.codec.device, self.stripes, len(srcs), c_void_p(self._rsrc.data_ptr()),
                                           c_void_p(self._rdst.data_ptr()), self.len,
                                           stream if stream is not None else _stream()), "repair")

    def repair_bytes(self, lost_block: int) -> int:
        return self.stripes * (len(self.codec.repairSources(lost_block)) + 1) * self.len


def xor_reduce(src, dst, length=None, device: int = 0) -> None:
    """dst = XOR of the device blocks in `src` (any fan-in 1..256)."""
    n = length if length is not None else min(_nbytes(b) for b in list(src) + [dst])
    _check(lib.ecw_xor_reduce_dev(device, _parr(list(src)), len(src), _addr(dst), n, _stream()), "xor_reduce")


def device_count() -> int:
    return lib.ecw_device_count()


def service_counters(device: int = 0) -> dict:
    """The resident small-request service's counters on `device`
    (ecw_service_counters): requests served, eligible requests that took the
    launch path, epochs launched, and whether it turned itself off."""
    out = (c_uint64 * 4)()
    _check(lib.ecw_service_counters(device, out), "service_counters")
    return {"served": out[0], "declined": out[1], "epochs": out[2], "broken": bool(out[3])}


SCHEDULE_FIELDS = ("xor_skew", "xor_order", "xor_window_log2p", "xor_window_width", "enc_window_log2p",
                   "enc_window_width", "xcd_remap")


def get_schedule() -> dict:
    """The process's launch schedule (ecwide.h ecw_schedule; -1 = the library's
    per-layout choice)."""
    s = _lib.ecw_schedule()
    _check(lib.ecw_get_schedule(byref(s)), "get_schedule")
    return {f: getattr(s, f) for f in SCHEDULE_FIELDS}


def set_schedule(**fields) -> dict:
    """Set the launch schedule: every field not given goes back to -1 (auto).
    Returns the previous schedule. Tuning only: no field changes a result byte."""
    bad = set(fields) - set(SCHEDULE_FIELDS)
    if bad:
        raise TypeError(f"unknown schedule fields {sorted(bad)}")
    prev = get_schedule()
    s = _lib.ecw_schedule(*[int(fields.get(f, -1)) for f in SCHEDULE_FIELDS])
    _check(lib.ecw_set_schedule(byref(s)), f"set_schedule({fields})")
    return prev


def apply_schedule(L, **fields) -> None:
    """ecw_set_schedule on a given build `L` (a tuning variant loaded with
    _lib.load(path, strict=False)); fields not given go back to -1."""
    s = _lib.ecw_schedule(*[int(fields.get(f, -1)) for f in SCHEDULE_FIELDS])
    _check(L.ecw_set_schedule(byref(s)), f"set_schedule({fields})")


def parse_schedule(xor: str | None = None, window: str | None = None, remap: str | None = None) -> dict:
    """Schedule fields from the string forms the tools and the environment use:
    xor = "K,ORDER[,LOG2P,W]" (a whole XOR schedule: no window unless given),
    window = "off" | "on" | "LOG2P,W" (the encode's write window), remap = "0" | "1"."""
    f = {}
    if xor not in (None, "auto"):
        v = [int(x) for x in xor.split(",")]
        f["xor_skew"], f["xor_window_width"] = v[0], 0
        if len(v) >= 2:
            f["xor_order"] = v[1]
        if len(v) >= 4:
            f["xor_window_log2p"], f["xor_window_width"] = v[2], v[3]
    if window not in (None, "auto"):
        if window in ("off", "0"):
            f["enc_window_width"] = 0
        elif window == "on":
            f["enc_window_log2p"], f["enc_window_width"] = 11, 64
        else:
            f["enc_window_log2p"], f["enc_window_width"] = (int(x) for x in window.split(","))
    if remap not in (None, "auto"):
        f["xcd_remap"] = int(remap)
    return f


class PinnedHost:
    """Host memory on the NUMA node of `device`'s PCIe root (or on `node`),
    pinned for DMA (ecw_host_alloc_node): staging for the host-memory entry points that keeps
    their copies at PCIe rate and off the inter-socket fabric. `.array` is a
    uint8 numpy view; `.numa_node` the node its pages were found on (-1:
    unknown). Freed by free() or when the object is collected."""

    def __init__(self, nbytes: int, device: int = 0, node: int = -1):
        import weakref

        p, got = c_void_p(), c_int(-1)
        _check(lib.ecw_host_alloc_node(device, node, nbytes, byref(p), byref(got)), f"host_alloc({nbytes}, node {node})")
        self.ptr, self.nbytes, self.device = p.value, int(nbytes), device
        self.numa_node = got.value
        self.device_numa_node = lib.ecw_device_numa_node(device)
        raw = (ctypes.c_uint8 * self.nbytes).from_address(self.ptr)
        raw.owner = self  # views of `array` keep the allocation alive (freed when the last one goes)
        self.array = np.ctypeslib.as_array(raw)
        self._fin = weakref.finalize(self, lib.ecw_host_free, c_void_p(self.ptr))

    def free(self) -> None:
        """Unregister and unmap now: views of `array` must not be used after."""
        self.array = None
        self._fin()

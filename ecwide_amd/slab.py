"""Batches of independent stripes resident in HBM (the north_star layout).

A ``StripeSlab`` is one torch uint8 CUDA allocation holding ``stripes``
stripes. Three layouts:

* ``"blocks"`` (default): stripe s starts at ``s * stripe_stride`` and block b
  of a stripe at ``b * block_stride``, blocks ordered [D_0..D_{k-1},
  G_0..G_{m-1}, L_0..L_{g-1}] (the D/G/L order ChunkGenerator.java:51-103
  writes). The block stride is padded past B (default +4 KiB) so the k
  concurrent row streams of a stripe do not all start on the same HBM channel.
* ``"split"``: whole contiguous blocks as in "blocks", but the data blocks of
  all stripes form one region and the parity blocks of all stripes a second
  one after it (ecw_encode_batch_split_dev). Parity rows interleaved with the
  data rows at one stride (the "blocks" slab) cost the encode ~10 %; in a
  region of their own the block layout encodes at the tiled slab's rate
  (the study, tools/rw_layout.py, is in git history:
  `git show 2666ebe:tools/rw_layout.py`).
* ``"tiled"``: every block is cut into ``chunk``-byte column pieces (default
  ``default_chunk(k)``: 8 KiB, 16 KiB at k <= 32); piece c
  of the k data blocks of stripe s is one contiguous run of k * chunk bytes
  (data region), piece c of the m + g parities one run in the parity region
  after it. Each (stripe, piece) is encoded as an independent stripe of
  ``chunk`` bytes (ecw_encode_batch_split_dev); repair writes the rebuilt
  block contiguously. Measured faster for the encode's 128-read / 8-write
  byte mix. ``fill_random`` writes the same block bytes
  in both layouts, so a tiled slab's parities equal the block slab's.
"""
from __future__ import annotations

from ctypes import c_void_p

from .codec import NativeCodec, _check, _stream
from ._lib import lib

DEFAULT_PAD = 4096
DEFAULT_CHUNK = 8192


def default_chunk(k: int) -> int:
    """Column piece of the tiled layout for k data blocks. Interleaved on one
    allocation (tools/layout_ab.py): k = 128 8 KiB (encode 6202 GB/s against
    5877 at 16 KiB and 5909 at 4 KiB; profiles/r04_k128_piece.log, round 2's
    sweep agrees); k = 32 16 KiB (CL(32, 8, 2) 16 MiB: encode 6128 / repair 6222
    against 5986 / 6061 at 8 KiB; CL(32, 11, 3) 64 MiB: 6129 / 5956 against
    6011 / 6001; 32 KiB and above lose; profiles/r04_k32_piece_cfg1/0.log)."""
    return 16384 if k <= 32 else DEFAULT_CHUNK


# launch_encode (ecw_kernels.hip) windows: 256 CUs x ECW_GRID_PER_CU (256) tiles per launch
ENCODE_LAUNCH_TILES = 256 * 256
TICKET_MIN_TILES = 4 * ENCODE_LAUNCH_TILES  # ECW_TICKET_MIN_TILES: one ticket-ordered launch from here on


class StripeSlab:
    def __init__(self, codec: NativeCodec, stripes: int, block_bytes: int | None = None,
                 pad: int = DEFAULT_PAD, device: int | None = None, layout: str = "blocks",
                 chunk: int | None = None, unit_pad: int = 0, base_offset: int = 0):
        import torch

        self.codec = codec
        self.stripes = stripes
        self.len = int(block_bytes if block_bytes is not None else codec.chunkSize)
        self.nblocks = codec.encodeDataNum + codec.parityNum
        self.layout = layout
        self.out_stride = (self.len + 15) // 16 * 16  # default stride of repair outputs
        dev = codec.device if device is None else device
        k, np_ = codec.encodeDataNum, codec.parityNum
        if layout == "blocks":
            self.block_stride = (self.len + pad + 255) // 256 * 256
            self.stripe_stride = self.nblocks * self.block_stride
            nbytes = stripes * self.stripe_stride
        elif layout == "split":
            self.block_stride = (self.len + pad + 255) // 256 * 256
            self.stripe_stride = k * self.block_stride      # data region
            self.pstripe_stride = np_ * self.block_stride   # parity region
            self.parity_offset = stripes * self.stripe_stride
            nbytes = self.parity_offset + stripes * self.pstripe_stride
        elif layout == "tiled":
            if chunk is None:
                chunk = default_chunk(k)
                while self.len % chunk and chunk > 256:  # blocks that are not a multiple of the piece
                    chunk //= 2
            if chunk % 256 or chunk <= 0 or self.len % chunk:
                raise ValueError("tiled layout: chunk must be a positive multiple of 256 dividing the block size")
            if unit_pad % 256:
                raise ValueError("unit_pad must be a multiple of 256")
            self.chunk = chunk
            self.pieces = self.len // chunk           # column pieces per block
            self.units = stripes * self.pieces        # independent (stripe, piece) stripes
            self.unit_stride = k * chunk + unit_pad   # data bytes per unit (+ padding)
            self.punit_stride = np_ * chunk + unit_pad
            self.parity_offset = (self.units * self.unit_stride + 4095) // 4096 * 4096
            nbytes = self.parity_offset + self.units * self.punit_stride
        else:
            raise ValueError(f"unknown layout {layout!r}")
        if base_offset % 256 or base_offset < 0:
            raise ValueError("base_offset must be a non-negative multiple of 256")
        self.off = base_offset  # where the slab starts inside its allocation
        self.buf = torch.empty(nbytes + base_offset, dtype=torch.uint8, device=f"cuda:{dev}")
        self.base = self.buf.data_ptr() + base_offset

    def _split_args(self):
        if self.layout == "split":
            bs = self.block_stride
            return (c_void_p(self.base), bs, self.stripe_stride, c_void_p(self.base + self.parity_offset), bs,
                    self.pstripe_stride)
        ch = self.chunk
        return (c_void_p(self.base), ch, self.unit_stride, c_void_p(self.base + self.parity_offset), ch,
                self.punit_stride)

    # views ------------------------------------------------------------------
    def block(self, s: int, b: int):
        """Block b of stripe s (a view; in the tiled layout a contiguous copy)."""
        if self.layout == "blocks":
            o = self.off + s * self.stripe_stride + b * self.block_stride
            return self.buf[o:o + self.len]
        k, np_ = self.codec.encodeDataNum, self.codec.parityNum
        if self.layout == "split":
            o = self.off + (s * self.stripe_stride + b * self.block_stride if b < k else
                            self.parity_offset + s * self.pstripe_stride + (b - k) * self.block_stride)
            return self.buf[o:o + self.len]
        ch = self.chunk
        if b < k:
            o, step = s * self.pieces * self.unit_stride + b * ch, self.unit_stride
        else:
            o, step = self.parity_offset + s * self.pieces * self.punit_stride + (b - k) * ch, self.punit_stride
        return self.buf.as_strided((self.pieces, ch), (step, 1), self.off + o).reshape(-1)

    def data(self, s: int):
        return [self.block(s, j) for j in range(self.codec.encodeDataNum)]

    def parity(self, s: int):
        k = self.codec.encodeDataNum
        return [self.block(s, k + i) for i in range(self.codec.parityNum)]

    # operations -------------------------------------------------------------
    def fill_random(self, seed: int, s0: int = 0, col_offset: int = 0) -> None:
        """Synthetic data blocks (ecwide.h counter PRNG), stripe ids s0..: data
        block j of stripe s holds bytes [col_offset, col_offset + len) of the
        generator stream (seed, s0 + s, j) in both layouts, so a block reads the
        same through block() whatever the layout (col_offset: this slab holds a
        column slice of longer blocks, e.g. one rank's shard.column_shard)."""
        k = self.codec.encodeDataNum
        if self.layout == "tiled":
            ch = self.chunk
            args = (ch, self.pieces * self.unit_stride, self.stripes, k, self.len, ch, self.unit_stride)
        else:  # blocks / split: the data blocks at block_stride, stripes at stripe_stride
            args = (self.block_stride, self.stripe_stride, self.stripes, k, self.len, max(16, self.out_stride), 0)
        _check(lib.ecw_fill_random_pieces_dev(self.codec.device, c_void_p(self.base), *args, col_offset, seed, s0, 0,
                                              _stream()), "fill_random")

    def encode(self, stream=None) -> None:
        st = stream if stream is not None else _stream()
        if self.layout == "tiled":
            _check(lib.ecw_encode_batch_split_dev(self.codec._h, *self._split_args(), self.units, self.chunk, st),
                   "encode_batch_split")
            return
        if self.layout == "split":
            _check(lib.ecw_encode_batch_split_dev(self.codec._h, *self._split_args(), self.stripes, self.len, st),
                   "encode_batch_split")
            return
        _check(lib.ecw_encode_batch_dev(self.codec._h, c_void_p(self.base), self.block_stride,
                                        self.stripe_stride, self.stripes, self.len, st), "encode_batch")

    def repair(self, lost_block: int, out, out_stride: int | None = None, stream=None) -> None:
        """XOR-rebuild `lost_block` of every stripe into out[s*out_stride:]
        (`out` holds stripes * out_stride bytes; strides are 16-B multiples)."""
        ostride = self.out_stride if out_stride is None else out_stride
        if self.layout == "tiled":
            if ostride != self.len:
                raise ValueError("tiled layout: repair outputs are contiguous blocks (out_stride = block size)")
            _check(lib.ecw_repair_batch_split_dev(self.codec._h, *self._split_args(), self.units, lost_block,
                                                  c_void_p(out.data_ptr()), self.chunk, self.chunk,
                                                  stream if stream is not None else _stream()), "repair_split")
            return
        if self.layout == "split":
            _check(lib.ecw_repair_batch_split_dev(self.codec._h, *self._split_args(), self.stripes, lost_block,
                                                  c_void_p(out.data_ptr()), ostride, self.len,
                                                  stream if stream is not None else _stream()), "repair_split")
            return
        _check(lib.ecw_repair_batch_dev(self.codec._h, c_void_p(self.base), self.block_stride,
                                        self.stripe_stride, self.stripes, lost_block, c_void_p(out.data_ptr()),
                                        ostride, self.len, stream if stream is not None else _stream()),
               "repair_batch")

    def encode_bytes(self) -> int:
        """Algorithmic bytes of one encode of the slab: (k + m + g) * B per stripe."""
        return self.stripes * self.nblocks * self.len

    def encode_launches(self) -> int:
        """Kernel launches one encode() makes: ceil(m / 16) row passes, each in
        windows of ENCODE_LAUNCH_TILES 4 KiB column tiles, or one ticket-ordered
        launch from TICKET_MIN_TILES tiles on (ecw_kernels.hip launch_encode).
        For per-launch timings next to rocprof's."""
        units, ulen = (self.units, self.chunk) if self.layout == "tiled" else (self.stripes, self.len)
        tiles = units * -(-ulen // 4096)
        passes = max(1, -(-self.codec.scheme.globalParityNum // 16))  # kMaxPassRows
        if tiles >= TICKET_MIN_TILES and self.codec.encodeDataNum >= 2:
            return passes  # one ticket-ordered launch per pass
        return passes * -(-tiles // ENCODE_LAUNCH_TILES)

    def repair_bytes(self, lost_block: int) -> int:
        """(survivors + 1) * B per stripe: r reads + 1 write for a data block."""
        return self.stripes * (len(self.codec.repairSources(lost_block)) + 1) * self.len

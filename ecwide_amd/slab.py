"""Batches of independent stripes resident in HBM (the north_star layout).

A ``StripeSlab`` is one torch uint8 CUDA allocation holding ``stripes``
stripes; stripe s starts at ``s * stripe_stride`` and block b of a stripe at
``b * block_stride``, blocks ordered [D_0..D_{k-1}, G_0..G_{m-1},
L_0..L_{g-1}] (the D/G/L order ChunkGenerator.java:51-103 writes). The block
stride is padded past B (default +4 KiB) so the k concurrent row streams of
a stripe do not all start on the same HBM channel.
"""
from __future__ import annotations

from ctypes import c_void_p

from .codec import NativeCodec, _check, _stream
from ._lib import lib

DEFAULT_PAD = 4096


class StripeSlab:
    def __init__(self, codec: NativeCodec, stripes: int, block_bytes: int | None = None,
                 pad: int = DEFAULT_PAD, device: int | None = None):
        import torch

        self.codec = codec
        self.stripes = stripes
        self.len = int(block_bytes if block_bytes is not None else codec.chunkSize)
        self.nblocks = codec.encodeDataNum + codec.parityNum
        self.block_stride = (self.len + pad + 255) // 256 * 256
        self.stripe_stride = self.nblocks * self.block_stride
        self.out_stride = (self.len + 15) // 16 * 16  # default stride of repair outputs
        dev = codec.device if device is None else device
        self.buf = torch.empty(stripes * self.stripe_stride, dtype=torch.uint8, device=f"cuda:{dev}")
        self.base = self.buf.data_ptr()

    # views ------------------------------------------------------------------
    def block(self, s: int, b: int):
        o = s * self.stripe_stride + b * self.block_stride
        return self.buf[o:o + self.len]

    def data(self, s: int):
        return [self.block(s, j) for j in range(self.codec.encodeDataNum)]

    def parity(self, s: int):
        k = self.codec.encodeDataNum
        return [self.block(s, k + i) for i in range(self.codec.parityNum)]

    # operations -------------------------------------------------------------
    def fill_random(self, seed: int, s0: int = 0) -> None:
        """Synthetic data blocks (ecwide.h counter PRNG), stripe ids s0.."""
        _check(lib.ecw_fill_random_dev(self.codec.device, c_void_p(self.base), self.block_stride,
                                       self.stripe_stride, self.stripes, self.codec.encodeDataNum, self.len,
                                       seed, s0, 0, _stream()), "fill_random")

    def encode(self, stream=None) -> None:
        _check(lib.ecw_encode_batch_dev(self.codec._h, c_void_p(self.base), self.block_stride,
                                        self.stripe_stride, self.stripes, self.len,
                                        stream if stream is not None else _stream()), "encode_batch")

    def repair(self, lost_block: int, out, out_stride: int | None = None, stream=None) -> None:
        """XOR-rebuild `lost_block` of every stripe into out[s*out_stride:]
        (`out` holds stripes * out_stride bytes; strides are 16-B multiples)."""
        ostride = self.out_stride if out_stride is None else out_stride
        _check(lib.ecw_repair_batch_dev(self.codec._h, c_void_p(self.base), self.block_stride,
                                        self.stripe_stride, self.stripes, lost_block, c_void_p(out.data_ptr()),
                                        ostride, self.len, stream if stream is not None else _stream()),
               "repair_batch")

    def encode_bytes(self) -> int:
        """Algorithmic bytes of one encode of the slab: (k + m + g) * B per stripe."""
        return self.stripes * self.nblocks * self.len

    def repair_bytes(self, lost_block: int) -> int:
        """(survivors + 1) * B per stripe: r reads + 1 write for a data block."""
        return self.stripes * (len(self.codec.repairSources(lost_block)) + 1) * self.len

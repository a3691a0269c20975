"""ChunkGenerator replay: ECWide-C's offline encoder with the encode on the GPU.

Mirrors ECWide-C/src/ChunkGenerator.java (and FileOp.java / BufferUnit.java
for the buffers and files): read k source blocks, encodeData, write the D/G/L
chunk files with the reference's names. This is BASELINE config #1
("ECWide-C CPU encode ... with default ECWide-C/config").

    python -m ecwide_amd.chunk_generator [zero|urandom|prng] [toy|<stripes>] \
        [--scheme config/scheme.ini] [--settings config/settings.ini] [--chunks-dir DIR]

The chunk files hold the reference's bytes by default: ECWide-C's
encodeData writes all-zero local parities (NativeCodec.cc:181-186: the XOR
table is built from a zeroed matrix), and so does this replay, like the JNI
drop-in libcodec.so; ``--xor`` writes the CL code as designed (L = XOR of the
group, what decodeData's repair assumes).

Differences, deliberate: ChunkGenerator.main parses args[0] (the source) as
the stripe count when args[1] != "toy" (ChunkGenerator.java:118-119), which
throws; here args[1] is the count. "prng" (the ecwide.h counter generator)
is added so runs are reproducible.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np


def read_settings(path: str) -> dict:
    """Settings.getFromFile (Settings.java:35-58): key = value lines."""
    out = {}
    with open(path) as f:
        for line in f:
            if "=" in line:
                k, v = line.split("=", 1)
                out[k.strip()] = v.strip()
    return out


def chunk_file_names(scheme, stripe_id: int) -> list:
    """Names generateChunks writes (ChunkGenerator.java:59-103), in the
    BufferUnit order [D_0..D_{k-1}, G_0..G_{m-1}, L_0..L_{g-1}]."""
    k, m = scheme.k, scheme.globalParityNum
    lrc_cl = scheme.codeType in ("LRC", "CL")
    names = []
    for i in range(k):
        if stripe_id >= 0:
            names.append(f"D_{stripe_id}_{i}")
        else:
            pos = i + 1 + (i // scheme.groupDataNum if lrc_cl else 0)
            names.append(f"{pos}_D_{i}")
    for i in range(m):
        if stripe_id >= 0:
            names.append(f"G_{stripe_id}_{i}")
        else:
            t = scheme.groupNum + k if lrc_cl else k
            names.append(f"{i + 1 + t}_G_{i}")
    if lrc_cl:
        for i in range(scheme.groupNum):
            if stripe_id >= 0:
                names.append(f"L_{stripe_id}_{i}")
            else:
                t = (scheme.groupDataNum + 1) * (i + 1) if i != scheme.groupNum - 1 else scheme.groupNum + k
                names.append(f"{t}_L_{i}")
    return names


class ChunkGenerator:
    def __init__(self, scheme, dir_name: str, source: str, local_mode: str = "literal", pinned: bool = True):
        from .codec import NativeCodec

        self.scheme = scheme
        self.dir_name = dir_name
        self.source = source
        ct = scheme.codeType
        if ct == "CL":
            self.codec = NativeCodec.getClCodec(scheme, 1, False, local_mode=local_mode)
        elif ct == "LRC":
            self.codec = NativeCodec.getLrcCodec(scheme, 1, local_mode=local_mode)
        elif ct == "TL":
            self.codec = NativeCodec.getTlCodec(scheme, 1)
        else:
            self.codec = NativeCodec.getRsCodec(scheme)
        B = scheme.chunkSize
        n = scheme.k + self.codec.parityNum
        # BufferUnit(scheme, isLocalEncode=true): k data + parity buffers of chunkSize
        if pinned:
            import torch

            buf = torch.empty(n * B, dtype=torch.uint8, pin_memory=True).numpy()
        else:
            buf = np.empty(n * B, np.uint8)
        self.blocks = [buf[i * B:(i + 1) * B] for i in range(n)]
        self.data = self.blocks[:scheme.k]
        self.parity = self.blocks[scheme.k:]
        os.makedirs(dir_name, exist_ok=True)

    def get_source_data(self) -> None:
        """getSourceData: FileOp.readFile(b, /dev/zero | /dev/urandom) per block."""
        B = self.scheme.chunkSize
        for b in self.data:
            if self.source in ("zero", "urandom"):
                with open("/dev/zero" if self.source == "zero" else "/dev/urandom", "rb") as f:
                    got = f.readinto(memoryview(b))
                    assert got == B
            else:
                raise ValueError(f"unknown source {self.source}")

    def fill_prng(self, seed: int) -> None:
        """The ecwide.h counter generator, made on the GPU and copied in."""
        import torch

        from .slab import StripeSlab

        slab = StripeSlab(self.codec, stripes=1)
        slab.fill_random(seed)
        torch.cuda.synchronize()
        for j, b in enumerate(self.data):
            b[:] = slab.block(0, j).cpu().numpy()

    def encode_chunks(self) -> None:
        self.codec.encodeData(self.data, self.parity)

    def generate_chunks(self, stripe_id: int) -> list:
        """FileOp.writeFile of every block under its reference name."""
        paths = []
        for name, b in zip(chunk_file_names(self.scheme, stripe_id), self.blocks):
            p = os.path.join(self.dir_name, name)
            with open(p, "wb") as f:
                f.write(memoryview(b))
            paths.append(p)
        return paths


def main(argv=None) -> int:
    from .codec import CodingScheme

    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("source", choices=["zero", "urandom", "prng"])
    ap.add_argument("mode", help="toy or a number of stripes")
    ap.add_argument("--scheme", default="config/scheme.ini")
    ap.add_argument("--settings", default="config/settings.ini")
    ap.add_argument("--chunks-dir", default=None)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--xor", action="store_true",
                    help="XOR local parities (the CL code as designed) instead of ECWide-C's all-zero L blocks")
    a = ap.parse_args(argv)
    gen_num = -1 if a.mode == "toy" else int(a.mode)
    chunks_dir = a.chunks_dir or read_settings(a.settings)["chunksDir"]
    scheme = CodingScheme.getFromConfig(a.scheme)
    gen = ChunkGenerator(scheme, chunks_dir, a.source, local_mode="xor" if a.xor else "literal")
    print("create ChunkGenerator OK")
    if a.source == "prng":
        gen.fill_prng(a.seed)
    else:
        gen.get_source_data()
    print("getSourceData OK")
    t0 = time.perf_counter()
    gen.encode_chunks()
    ms = (time.perf_counter() - t0) * 1e3
    print(f"encodeChunks OK, {ms:.3f} ms")
    if gen_num < 0:
        print("generate toy chunks")
        gen.generate_chunks(-1)
    else:
        for i in range(gen_num):
            gen.generate_chunks(i)
    print("generateChunks OK")
    return 0


if __name__ == "__main__":
    sys.exit(main())

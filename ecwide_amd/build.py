"""Build libecwide.so (HIP kernels + C ABI) and libecw_isal.so (the ISA-L
signature shim over it) in-tree: hipcc, gfx950 only."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SOURCES = [os.path.join(HERE, "csrc", "ecw_codec.cpp"), os.path.join(HERE, "csrc", "ecw_kernels.hip")]
HEADERS = [os.path.join(HERE, "csrc", f) for f in ("ecw_gf.hpp", "ecw_internal.hpp")] + [
    os.path.join(REPO, "include", "ecwide.h")]
OUT = os.path.join(HERE, "libecwide.so")
SHIM_SRC = os.path.join(HERE, "csrc", "ecw_isal_shim.cpp")
SHIM_OUT = os.path.join(HERE, "libecw_isal.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wno-unused-function",
         "-I" + os.path.join(REPO, "include")]


def up_to_date(out=OUT, sources=SOURCES) -> bool:
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    return all(os.path.getmtime(p) <= t for p in sources + HEADERS + [__file__])


def build(force: bool = False) -> str:
    if force or not up_to_date():
        cmd = [HIPCC, *FLAGS, *SOURCES, "-o", OUT + ".tmp"]
        subprocess.run(cmd, check=True)
        os.replace(OUT + ".tmp", OUT)
    if force or not up_to_date(SHIM_OUT, [SHIM_SRC, OUT]):
        # host-only C++; links libecwide.so next to it ($ORIGIN)
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-I" + os.path.join(REPO, "include"),
               SHIM_SRC, "-L" + HERE, "-lecwide", "-Wl,-rpath,$ORIGIN", "-o", SHIM_OUT + ".tmp"]
        subprocess.run(cmd, check=True)
        os.replace(SHIM_OUT + ".tmp", SHIM_OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))

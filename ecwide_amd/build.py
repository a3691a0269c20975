"""Build libecwide.so (HIP kernels + C ABI) and libecw_isal.so (the ISA-L
signature shim over it) in-tree: hipcc, gfx950 only. libcodec.so (the JNI
natives of ECWide-C over the C ABI) is built when a JDK's jni.h is found."""
from __future__ import annotations

import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SOURCES = [os.path.join(HERE, "csrc", f) for f in
           ("ecw_codec.cpp", "ecw_kernels.hip", "ecw_xor_ptr.hip", "ecw_xor_slab.hip", "ecw_service.hip")]
HEADERS = [os.path.join(HERE, "csrc", f) for f in
           ("ecw_gf.hpp", "ecw_internal.hpp", "ecw_tuning.hpp", "ecw_device.hpp", "ecw_encode_asm.hpp", "ecw_xor.hpp")] + [
    os.path.join(REPO, "include", "ecwide.h")]
OUT = os.path.join(HERE, "libecwide.so")
OBJ = os.path.join(REPO, "build", "obj")
SHIM_SRC = os.path.join(HERE, "csrc", "ecw_isal_shim.cpp")
SHIM_OUT = os.path.join(HERE, "libecw_isal.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS_C = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wmissing-field-initializers",
           "-Wno-unused-function", "-I" + os.path.join(REPO, "include")]


def _tmp() -> str:
    """Per-process temporary suffix: concurrent builders (pytest -n) never share
    a half-written file; os.replace publishes the finished one atomically."""
    return f".{os.getpid()}.tmp"


def up_to_date(out=OUT, sources=SOURCES) -> bool:
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    return all(os.path.getmtime(p) <= t for p in sources + HEADERS + [__file__])


def includes(src: str, seen=None) -> set:
    """`src` and every file it includes with #include "..." (recursively)."""
    import re

    seen = set() if seen is None else seen
    src = os.path.normpath(src)
    if src in seen or not os.path.exists(src):
        return seen
    seen.add(src)
    for name in re.findall(r'^#include "([^"]+)"', open(src).read(), flags=re.M):
        includes(os.path.join(os.path.dirname(src), name), seen)
    return seen


def compile_lib(out: str, extra=(), obj_dir: str = OBJ) -> None:
    """Every translation unit to an object in parallel (the kernel TUs take
    minutes each: encode, XOR and service are separate so they compile side
    by side), then one link; `extra` flags (a tuning variant's -D...) apply
    to every TU."""
    from concurrent.futures import ThreadPoolExecutor

    os.makedirs(obj_dir, exist_ok=True)

    stamp = os.path.join(obj_dir, "flags.txt")  # objects built with other flags are rebuilt
    flags = " ".join([*FLAGS_C, *extra])
    same_flags = os.path.exists(stamp) and open(stamp).read() == flags

    def one(src):
        o = os.path.join(obj_dir, os.path.basename(src) + ".o")
        if same_flags and os.path.exists(o) and os.path.getmtime(o) >= max(
                os.path.getmtime(p) for p in [__file__, *includes(src)]):
            return o
        cmd = [HIPCC, *FLAGS_C, *extra, "-c", src, "-o", o + _tmp()]
        subprocess.run(cmd, check=True)
        os.replace(o + _tmp(), o)
        return o

    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(one, SOURCES))
    with open(stamp, "w") as f:
        f.write(flags)
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", out + _tmp()], check=True)
    os.replace(out + _tmp(), out)


def build(force: bool = False) -> str:
    if force or not up_to_date():
        compile_lib(OUT)
    if force or not up_to_date(SHIM_OUT, [SHIM_SRC, OUT]):
        # host-only C++; links libecwide.so next to it ($ORIGIN)
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-I" + os.path.join(REPO, "include"),
               SHIM_SRC, "-L" + HERE, "-lecwide", "-Wl,-rpath,$ORIGIN", "-o", SHIM_OUT + _tmp()]
        subprocess.run(cmd, check=True)
        os.replace(SHIM_OUT + _tmp(), SHIM_OUT)
    return OUT


JNI_SRC = os.path.join(HERE, "csrc", "jni", "ecw_jni.cpp")
JNI_OUT = os.path.join(HERE, "libcodec.so")


def jdk_include_dirs() -> list[str] | None:
    """$JAVA_HOME/include (+ include/linux), else the first /usr/lib/jvm JDK."""
    homes = [os.environ["JAVA_HOME"]] if os.environ.get("JAVA_HOME") else []
    homes += sorted(glob.glob("/usr/lib/jvm/*"))
    for h in homes:
        inc = os.path.join(h, "include")
        if os.path.exists(os.path.join(inc, "jni.h")):
            return [inc, os.path.join(inc, "linux")]
    return None


def build_jni(include_dirs: list[str] | None = None, out: str = JNI_OUT, force: bool = False) -> str | None:
    """libcodec.so: ECWide-C's Java_NativeCodec_* over libecwide.so. Returns its
    path, or None when no jni.h is available (this image has no JDK)."""
    include_dirs = include_dirs or jdk_include_dirs()
    if not include_dirs:
        return None
    build()
    if force or not up_to_date(out, [JNI_SRC, OUT]):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        rpath = os.path.relpath(HERE, os.path.dirname(os.path.abspath(out)))
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-fvisibility=hidden",
               *("-I" + d for d in include_dirs), "-I" + os.path.join(REPO, "include"), JNI_SRC,
               "-L" + HERE, "-lecwide", "-Wl,-rpath,$ORIGIN/" + rpath, "-o", out + _tmp()]
        subprocess.run(cmd, check=True)
        os.replace(out + _tmp(), out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))

"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer.

tests/csrc/asan_host.cpp is linked with ecw_codec.cpp, the kernels' host side,
the ISA-L shim (group-commit batcher from 8 threads), the JNI natives and the
JNI test double, all built with -fsanitize=address,undefined on the host side
only (hipcc -Xarch_host), and run on this GPU-less host: every host-only path
runs for real and every device entry point runs up to its ECW_EDEVICE return.
Any sanitizer report (leaks included) fails the run."""
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

from conftest import REPO

OUT = os.path.join(REPO, "build", "asan")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = [os.path.join(REPO, p) for p in (
    "tests/csrc/asan_host.cpp", "ecwide_amd/csrc/ecw_codec.cpp", "ecwide_amd/csrc/ecw_kernels.hip",
    "ecwide_amd/csrc/ecw_xor_ptr.hip", "ecwide_amd/csrc/ecw_xor_slab.hip",
    "ecwide_amd/csrc/ecw_service.hip", "ecwide_amd/csrc/ecw_isal_shim.cpp", "ecwide_amd/csrc/jni/ecw_jni.cpp", "tests/jni/jvm_double.cpp")]
DEPS = SOURCES + [os.path.join(REPO, p) for p in (
    "include/ecwide.h", "ecwide_amd/csrc/ecw_gf.hpp", "ecwide_amd/csrc/ecw_internal.hpp",
    "ecwide_amd/csrc/ecw_tuning.hpp", "ecwide_amd/csrc/ecw_device.hpp", "ecwide_amd/csrc/ecw_xor.hpp", "ecwide_amd/csrc/ecw_encode_asm.hpp",
    "tests/jni/jni.h")]
FLAGS = ["--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-fno-omit-frame-pointer",
         "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
         "-Xarch_host", "-fno-sanitize-recover=undefined",
         "-I" + os.path.join(REPO, "include"), "-I" + os.path.join(REPO, "tests", "jni")]


def build() -> str:
    exe = os.path.join(OUT, "host_asan")
    if os.path.exists(exe) and os.path.getmtime(exe) >= max(os.path.getmtime(p) for p in DEPS + [__file__]):
        return exe
    os.makedirs(OUT, exist_ok=True)

    def obj(src):
        o = os.path.join(OUT, os.path.basename(src) + ".o")
        subprocess.run([HIPCC, *FLAGS, "-c", src, "-o", o], check=True)
        return o

    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(obj, SOURCES))
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-Xarch_host", "-fsanitize=address", "-Xarch_host",
                    "-fsanitize=undefined", *objs, "-lpthread", "-o", exe + f".{os.getpid()}.tmp"], check=True)
    os.replace(exe + f".{os.getpid()}.tmp", exe)
    return exe


def test_host_paths_clean_under_asan_ubsan():
    exe = build()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    tail = (p.stdout + p.stderr)[-4000:]
    assert p.returncode == 0, tail
    assert "Sanitizer" not in p.stderr and "runtime error" not in p.stderr, tail
    assert " 0 failed" in p.stdout, tail


def test_oracle_families_clean_under_asan_ubsan():
    """The checker too: oracle/ecw_oracle.c's kernel families (the CPU
    baseline's AVX2 / AVX-512 / GFNI ports) equal ec_encode_data_base on
    random shapes and ragged lengths, with no sanitizer report."""
    exe = os.path.join(OUT, "oracle_asan")
    os.makedirs(OUT, exist_ok=True)
    subprocess.run(["gcc", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                    "-fno-omit-frame-pointer", os.path.join(REPO, "tests", "csrc", "asan_oracle.c"),
                    os.path.join(REPO, "oracle", "ecw_oracle.c"), "-lpthread", "-o", exe], check=True)
    p = subprocess.run([exe], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1"))
    tail = (p.stdout + p.stderr)[-4000:]
    assert p.returncode == 0 and "asan oracle ok" in p.stdout, tail
    assert "runtime error" not in p.stderr, tail

"""The C ABI from a plain C program (tests/csrc/c_abi_device.c): no Python, no
torch -- what a C/C++ host of ECWide-C's codec, or the JNI / cgo shim a
maintainer would write, links against. The CPU test builds it
with gcc against include/ecwide.h and checks that it runs up to its first call;
the GPU test runs the fill / batched encode / batched CL repair / host encode
through the ABI and compares every byte with the oracle inside the program."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "csrc", "c_abi_device.c")
EXE = os.path.join(REPO, "build", "c_abi_device")


def build_c_abi_device() -> str:
    """gcc, C11, against the header and the in-tree libraries (rpath relative to
    the binary, so the tree can move)."""
    lib = os.path.join(REPO, "ecwide_amd", "libecwide.so")
    orc = os.path.join(REPO, "oracle", "liboracle.so")
    deps = [SRC, lib, orc, os.path.join(REPO, "include", "ecwide.h")]
    if os.path.exists(EXE) and all(os.path.getmtime(EXE) >= os.path.getmtime(d) for d in deps if os.path.exists(d)):
        return EXE
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    tmp = f"{EXE}.{os.getpid()}.tmp"
    subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__",
                    "-I" + os.path.join(REPO, "include"), "-I/opt/rocm/include", SRC,
                    "-L" + os.path.join(REPO, "ecwide_amd"), "-lecwide", "-L" + os.path.join(REPO, "oracle"), "-loracle",
                    "-L/opt/rocm/lib", "-lamdhip64",
                    "-Wl,-rpath,$ORIGIN/../ecwide_amd:$ORIGIN/../oracle:/opt/rocm/lib", "-o", tmp], check=True)
    os.replace(tmp, EXE)
    return EXE


def test_c_program_builds_against_the_header(orc):
    exe = build_c_abi_device()
    # argument check before any library call: the binary loads (every symbol of
    # the ABI it uses resolves) and refuses a bad shape with status 2
    p = subprocess.run([exe, "1"], capture_output=True, timeout=60)
    assert p.returncode == 2, p.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [["32", "2", "8", "1052689", "3"], ["128", "3", "27", "262144", "2"]])
def test_c_program_device_abi_vs_oracle(orc, shape):
    exe = build_c_abi_device()
    p = subprocess.run([exe, *shape], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and p.stdout.startswith("ok:"), (p.returncode, p.stdout, p.stderr[-2000:])

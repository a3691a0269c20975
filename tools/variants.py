#!/usr/bin/env python3
"""Build tuning variants of libecwide.so into build/variants/<name>.so.

  python tools/variants.py name=-DECW_PREFETCH_ENC=8 other=-DECW_ABLATE=1,-DECW_GRID_PER_CU=4 ...

Each spec is name=comma-separated extra flags. Used with tools/kbench.py on
the GPU box (the .so files travel with the snapshot; build/ is git-ignored).
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import importlib.util  # noqa: E402

_spec = importlib.util.spec_from_file_location("ecw_build", os.path.join(REPO, "ecwide_amd", "build.py"))
b = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(b)

OUT = os.path.join(REPO, "build", "variants")


def one(spec):
    name, _, flags = spec.partition("=")
    extra = [f for f in flags.split(",") if f]
    out = os.path.join(OUT, name + ".so")
    cmd = [b.HIPCC, *b.FLAGS, *extra, *b.SOURCES, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    return name, r.returncode, r.stderr[-2000:]


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    with ThreadPoolExecutor(6) as ex:
        for name, rc, err in ex.map(one, sys.argv[1:]):
            print(f"{name}: {'ok' if rc == 0 else 'FAILED'}")
            if rc:
                print(err)

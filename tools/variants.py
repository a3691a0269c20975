#!/usr/bin/env python3
"""Build tuning variants of libecwide.so into build/variants/<name>.so.

  python tools/variants.py name=-DECW_PREFETCH_ENC=8 other=-DECW_ABLATE=1,-DECW_GRID_PER_CU=4 ...

Each spec is name=comma-separated extra flags: overrides of the compile-time
tunables in ecwide_amd/csrc/ecw_tuning.hpp. (Run-time launch choices -- tile
order, write windows, XOR skew -- need no variant: ecw_set_schedule.) The
round 1-4 diagnostic ablations (math-free, store-free, no-staging builds)
were retired from the product source in round 5; build them from commit
90a4d53 (`git worktree add`). Used with tools/kbench.py on the GPU box (the
.so files travel with the snapshot; build/ is git-ignored).
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
    try:
        b.compile_lib(out, extra, obj_dir=os.path.join(OUT, "obj_" + name))
        return name, 0, ""
    except subprocess.CalledProcessError as e:
        return name, e.returncode, str(e)


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    with ThreadPoolExecutor(2) as ex:  # each build compiles its translation units in parallel
        for name, rc, err in ex.map(one, sys.argv[1:]):
            print(f"{name}: {'ok' if rc == 0 else 'FAILED'}")
            if rc:
                print(err)

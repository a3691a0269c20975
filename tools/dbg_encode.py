"""Tiny host + device encodes through a given libecwide.so build, statuses
printed (debugging aid; ECW_DEBUG_LAUNCH=1 makes the library name each launch)."""
import ctypes
import os
import sys
from ctypes import byref, c_void_p

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402,F401  (one HIP runtime for the process)

from ecwide_amd import _lib  # noqa: E402

L = _lib.load(sys.argv[1], strict=False)
for (k, m, r, B) in [(32, 3, 11, 4096), (32, 3, 11, 8192), (32, 3, 11, 1000), (128, 3, 27, 1 << 20)]:
    sch = _lib.ecw_scheme()
    assert L.ecw_scheme_init(byref(sch), b"C", k, m, r, B) == 0
    h = c_void_p()
    assert L.ecw_codec_create(byref(sch), 1, 0, 0, 0, byref(h)) == 0
    info = _lib.ecw_codec_info()
    L.ecw_codec_get_info(h, byref(info))
    data = [np.random.randint(0, 256, B, dtype=np.uint8) for _ in range(k)]
    par = [np.zeros(B, np.uint8) for _ in range(info.parity_num)]
    dp = (c_void_p * k)(*[d.ctypes.data for d in data])
    pp = (c_void_p * info.parity_num)(*[p.ctypes.data for p in par])
    st = L.ecw_encode(h, dp, pp, B)
    print("host encode", k, B, "->", st, flush=True)
    if st:
        break

"""Diagnostic: cycles per round of a lone wave for the quad, pair and one-lane SHA-256
round code (the floors bench.py prices the digest stage against)."""
import os
os.environ["CHUNKER_AMD_DIAG"] = "1"  # load libchunker_amd_diag.so (make -C chunker_amd/csrc diag)
import ctypes
import json
import sys

import numpy as np

sys.path.insert(0, ".")
from chunker_amd._lib import lib  # noqa: E402

lib.cg_diag_sha_rounds_split.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                         ctypes.c_void_p]
one_lane = hasattr(lib, "cg_diag_sha_rounds")  # (microbench.hip: absent from partial A/B builds)
if one_lane:
    lib.cg_diag_sha_rounds.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
it = 4000
res = {}
for rep in range(3):
    cyc = np.zeros(1, np.uint64)
    lib.cg_diag_sha_rounds_split(it, 1, 64, 1, cyc.ctypes.data)
    res.setdefault("quad", []).append(round(float(cyc[0]) / (it * 64), 2))
    lib.cg_diag_sha_rounds_split(it, 1, 64, 0, cyc.ctypes.data)
    res.setdefault("pair", []).append(round(float(cyc[0]) / (it * 64), 2))
    if one_lane:
        cyc2 = np.zeros(2, np.uint64)
        lib.cg_diag_sha_rounds(it, 1, 64, cyc2.ctypes.data)
        res.setdefault("one_lane", []).append(round(float(cyc2[0]) / (it * 64), 2))
print(json.dumps(res))

"""Diagnostic: BLAKE3 compression throughput without memory traffic
(cg_diag_b3_chain): cycles per compression per SIMD at 1..8 waves per SIMD, for the
product's B3_G4 compression (kind 0) and for K = 1, 2, 4 independent chains per lane
interleaved op by op (kinds 1, 2, 4).  ~720 VALU per compression."""
import os
os.environ["CHUNKER_AMD_DIAG"] = "1"
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")
import ctypes
import json
import sys

sys.path.insert(0, ".")
from chunker_amd._lib import lib  # noqa: E402

lib.cg_diag_b3_chain.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
lib.cg_diag_b3_chain.restype = ctypes.c_float
CUS, CLK = 256, 2.4e6  # clocks per ms
res = {}
for kind in (0, 1, 2, 4):
    K = max(kind, 1)
    for w in (1, 2, 4, 8):
        iters = 64
        ms = min(lib.cg_diag_b3_chain(kind, CUS * w, 256, iters) for _ in range(3))
        # per SIMD: w waves x iters x K compressions
        res[f"kind{kind}_{w}w"] = round(ms * CLK / (w * iters * K), 1)
print(json.dumps({"what": "cycles per compression per SIMD (2.4 GHz assumed)", **res}))

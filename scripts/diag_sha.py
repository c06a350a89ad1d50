"""Diagnostic: cycles per SHA-256 round for 1..N waves (s_memtime on device)."""
import os
os.environ["CHUNKER_AMD_DIAG"] = "1"  # load libchunker_amd_diag.so (make -C chunker_amd/csrc diag)
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")
import ctypes
import json
import sys

import numpy as np
import torch  # noqa: F401  (load torch's HIP runtime first)

sys.path.insert(0, ".")
from chunker_amd._lib import lib  # noqa: E402

lib.cg_diag_sha_rounds.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
res = {}
for blocks, threads in [(1, 64), (1, 128), (1, 256), (1, 512), (1, 1024), (4, 256), (256, 64), (256, 256), (1024, 256)]:
    it = 2000
    waves = blocks * threads // 64
    cyc = np.zeros(2 * waves, np.uint64)
    lib.cg_diag_sha_rounds(it, blocks, threads, cyc.ctypes.data)
    c = cyc[0::2].astype(float) / (it * 64)
    rt = cyc[1::2].astype(float)
    clk = cyc[0::2].astype(float) / (rt / 100e6) / 1e9
    res[f"{blocks}x{threads}"] = {"cycles_per_round_med": float(np.median(c)), "max": float(c.max()),
                                  "clock_GHz": float(np.median(clk))}
lib.cg_diag_sha_rounds_lds.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
for blocks in [1, 16, 256]:
    it = 2000
    cyc = np.zeros(2 * blocks, np.uint64)
    lib.cg_diag_sha_rounds_lds(it, blocks, cyc.ctypes.data)
    c = cyc[0::2].astype(float) / (it * 64)
    res[f"lds_{blocks}x64"] = {"cycles_per_round_med": float(np.median(c)), "max": float(c.max())}
print(json.dumps(res))

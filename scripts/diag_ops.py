"""Diagnostic: issue cost (cycles per instruction per wave) of the integer VALU
instructions the scan / SHA-256 / BLAKE3 kernels are built from, for 1, 4, 8 and 16
waves in one workgroup (s_memtime, shader clocks)."""
import os
os.environ["CHUNKER_AMD_DIAG"] = "1"  # load libchunker_amd_diag.so (make -C chunker_amd/csrc diag)
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")
import ctypes
import argparse
import json
import sys

import numpy as np
import torch  # noqa: F401

sys.path.insert(0, ".")
from chunker_amd._lib import lib  # noqa: E402

NAMES = ["v_add_u32", "v_lshl_add_u64", "v_perm_b32", "v_add_co+v_addc_co", "v_alignbit_b32", "v_bitop3_b32",
         "v_lshlrev_b64", "v_mov_b32_dpp", "v_add3_u32", "v_cndmask_b32", "dep_chain v_lshl_add_u64",
         "dep_chain v_add_u32", "v_xor_b32_dpp quad_perm", "v_add_u32_dpp row_shl:4", "v_mov_b32_dpp row_shl:4",
         "v_mov_b32", "v_mov_b32_sdwa BYTE_1 preserve", "v_perm_b32 (VGPR selector)",
         "v_and_b32", "v_lshlrev_b32", "v_lshl_or_b32", "v_min3_u32", "v_min_u32", "v_bfe_u32", "v_and_or_b32",
         "v_add_co_u32", "v_lshl_add_u32", "v_cmp_eq_u32_e64"]
lib.cg_diag_ops.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
ap = argparse.ArgumentParser()
ap.add_argument("--kinds", default="", help="comma-separated kind indices (default: all)")
args = ap.parse_args()
it = 500
res = {}
kinds = [int(k) for k in args.kinds.split(",")] if args.kinds else range(len(NAMES))
for k in kinds:
    name = NAMES[k]
    row = {}
    for threads in [64, 256, 512, 1024]:
        w = threads // 64
        cyc = np.zeros(w, np.uint64)
        rc = lib.cg_diag_ops(k, it, threads, cyc.ctypes.data)
        assert rc == 0
        row[f"{w}w"] = round(float(np.median(cyc)) / (it * 256), 2)
    res[name] = row
print(json.dumps(res))

"""Diagnostic: candidate-scan stage time on config-2 and config-4 shaped batches.

--variants: 0 product (k_scan_flat: 1 KiB rows, the hash carried across lanes by
linearity, non-temporal loads), 1 round-1 quad-transpose kernel, 2 LDS-staged, 3 page per
wave, 4 k_scan (own 4 KiB segment per lane), 5 k_scan_flat by --modes.  --modes (quad kernel only): 0 off, 1 loads only,
2 loads + transpose, 3 hashing without loads, 4/8/9 partial pipelines; with
--mode-variant 5: bit 0 non-temporal loads, bit 1 16 rows in flight.  Then raw HBM
read patterns (runs of L contiguous bytes per 4 KiB segment)."""
import os
os.environ["CHUNKER_AMD_DIAG"] = "1"  # load libchunker_amd_diag.so (make -C chunker_amd/csrc diag)
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")
import ctypes
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import chunker_amd as ca  # noqa: E402
from chunker_amd.nar import synth_nars_device  # noqa: E402

import argparse  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="0,1,2,3,4")
ap.add_argument("--modes", default="1,2,3")
ap.add_argument("--spw", default="0", help="k_scan_flat segments-per-wave caps to sweep (0 = default)")
ap.add_argument("--mode-variant", type=int, default=1, help="variant the --modes apply to (5: bit 0 nt, bit 1 16 rows)")
ap.add_argument("--configs", default="c2,c4")
ap.add_argument("--no-pattern", action="store_true")
ap.add_argument("--hash", type=int, default=0, help="digest between the timed scans: 0 BLAKE3, 1 SHA-256 (the bench's pipeline)")
ap.add_argument("--flush", action="store_true", help="read a 2 GiB scratch buffer before every timed scan (evicts the batch from the 256 MB MALL)")
args = ap.parse_args()
lib = ca.lib
lib.cg_diag_scan_mode.argtypes = [ctypes.c_uint32]
lib.cg_diag_scan_variant.argtypes = [ctypes.c_uint32]
lib.cg_diag_scan_spw_max.argtypes = [ctypes.c_uint32]
res = {}
scratch = torch.zeros(1 << 29, dtype=torch.int32, device="cuda") if args.flush else None
for name, n, size, params in [("c2", 256, 4 << 20, (256 << 10, 1 << 20, 4 << 20)),
                              ("c4", 4, 1 << 30, (64 << 10, 256 << 10, 1 << 20)),
                              ("c4full", 16, 1 << 30, (64 << 10, 256 << 10, 1 << 20)),
                              ("c5full", 16, 1 << 30, (256 << 10, 1 << 20, 4 << 20)),
                              ("c2x4", 1024, 4 << 20, (256 << 10, 1 << 20, 4 << 20)),
                              ("c5one", 1, 1 << 30, (256 << 10, 1 << 20, 4 << 20))]:
    if name not in args.configs.split(","):
        continue
    d, offs = synth_nars_device(np.full(n, size, np.uint64))
    cap = ca.chunking.batch_capacity(offs, params[0])
    out = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    buf = (ctypes.c_double * 5)()
    runs = [(int(v), 0) for v in args.variants.split(",") if v] + [(args.mode_variant, int(m)) for m in args.modes.split(",") if m]
    runs = [(v, m, int(w)) for v, m in runs for w in args.spw.split(",")]
    for variant, mode, spw in runs:
        lib.cg_diag_scan_variant(variant)
        lib.cg_diag_scan_mode(mode)
        lib.cg_diag_scan_spw_max(spw)
        ms = []
        for it in range(6):
            lib.cg_set_profiling(1)
            if args.flush:
                scratch.add_(1)  # 2 GiB read + written: the MALL holds none of the batch afterwards
                torch.cuda.synchronize()
            ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params, hash=args.hash, stream=sp)
            lib.cg_last_stage_times(buf, 5)
            if it >= 2:
                ms.append(buf[0])
        gib = int(offs[-1]) / 2**30
        res[f"{name}_v{variant}_mode{mode}" + (f"_spw{spw}" if spw else "")] = {"scan_ms": round(float(np.median(ms)), 4),
                                     "GBps": round(int(offs[-1]) / (np.median(ms) * 1e-3) / 1e9, 1)}
    lib.cg_diag_scan_mode(0)
    lib.cg_diag_scan_variant(0)
    lib.cg_diag_scan_spw_max(0)
    del d, out
    torch.cuda.empty_cache()
print(json.dumps(res))

# HBM read patterns: 1 GiB, runs of L contiguous bytes per 4 KiB segment per round
if args.no_pattern:
    sys.exit(0)
lib.cg_diag_read_pattern.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
lib.cg_diag_read_pattern.restype = ctypes.c_float
d = torch.randint(0, 255, (1 << 30,), dtype=torch.uint8, device="cuda")
o = torch.empty(512 * 512, dtype=torch.int32, device="cuda")
pat = {}
for lg in [6, 7, 8, 10, 12]:
    for depth in [2, 4]:
        for nt in [0, 1]:
            code = lg | (nt << 8) | (depth << 12)
            ms = sorted(lib.cg_diag_read_pattern(d.data_ptr(), code, o.data_ptr()) for _ in range(5))[2]
            pat[f"run{1 << lg}_d{depth}{'_nt' if nt else ''}"] = round(2**30 / (ms * 1e-3) / 1e9, 1)
print(json.dumps(pat))

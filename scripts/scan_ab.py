"""A/B of K1 scan kernels, same process, alternating: the scan stage's HIP-event time
(cg_set_profiling(1)) for the persistent k_scan_flat32p and the one-shot
k_scan_flat32 (cg_test_scan_kernel(1)), on config-shaped device batches.  With
CHUNKER_AMD_LIB set, the persistent side is that build (e.g. another CG_SCAN_SPU).
Prints one JSON object: median ms and TB/s per (config, kernel)."""
import argparse
import ctypes
import json
import os
import sys

os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import chunker_amd as ca  # noqa: E402
from chunker_amd.nar import synth_nars_device  # noqa: E402

SHAPES = {"c2": (256, 4 << 20, (256 << 10, 1 << 20, 4 << 20)),
          "c4": (16, 1 << 30, (64 << 10, 256 << 10, 1 << 20)),
          "c5": (16, 1 << 30, (256 << 10, 1 << 20, 4 << 20)),
          "c4q": (4, 1 << 30, (64 << 10, 256 << 10, 1 << 20)),
          "c2x": (300, 4 << 20, (256 << 10, 1 << 20, 4 << 20)),   # 1.17 GiB: not a whole number of rounds
          "c2h": (400, 4 << 20, (256 << 10, 1 << 20, 4 << 20))}   # 1.56 GiB
ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="c2,c4,c5")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--kernels", default="2,1", help="cg_test_scan_kernel values: 2 persistent, 1 one-shot, 0 product choice")
ap.add_argument("--hash", type=int, default=1)
ap.add_argument("--grids", default="0", help="persistent-scan grid overrides to sweep (cg_test_scan_grid; 0 = resident)")
args = ap.parse_args()
torch.cuda.set_device(0)
lib = ca.lib
buf = (ctypes.c_double * 5)()
res = {"lib": os.environ.get("CHUNKER_AMD_LIB", "product"), "resident_wgs": int(lib.cg_test_scan_grid(0))}
grids = [int(g) for g in args.grids.split(",")]
for cfg in args.configs.split(","):
    n, size, params = SHAPES[cfg]
    d, offs = synth_nars_device(np.full(n, size, np.uint64))
    cap = ca.chunking.batch_capacity(offs, params[0])
    out = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    kinds = [(int(k), g) for k in args.kernels.split(",") for g in (grids if int(k) == 2 else [0])]
    ms = {k: [] for k in kinds}
    firsts = {}
    for rep in range(args.reps + 1):
        for k in kinds:
            lib.cg_test_scan_kernel(k[0])
            lib.cg_test_scan_grid(k[1])
            lib.cg_set_profiling(1)
            first = ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params, hash=args.hash, stream=sp)
            lib.cg_last_stage_times(buf, 5)
            if rep:
                ms[k].append(buf[0])
            firsts.setdefault(k, first)
            assert np.array_equal(first, firsts[kinds[0]]), "kernels disagree on the chunk counts"
    lib.cg_set_profiling(0)
    lib.cg_test_scan_kernel(0)
    lib.cg_test_scan_grid(0)
    nbytes = int(offs[-1])
    for k in kinds:
        med = float(np.median(ms[k]))
        res[f"{cfg}_{['product', 'oneshot', 'persistent'][k[0]]}" + (f"_grid{k[1]}" if k[1] else "")] = {
            "ms": round(med, 4), "TBps": round(nbytes / (med * 1e-3) / 1e12, 3),
            "frac_8TBps": round(nbytes / (med * 1e-3) / 8e12, 4), "all_ms": [round(x, 4) for x in ms[k]]}
    del d, out
    torch.cuda.empty_cache()
print(json.dumps(res))

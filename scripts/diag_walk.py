"""Diagnostic: where k_walk's time goes on large NARs (per-NAR phase clocks from the
diagnostics build): the walk loop (piece-list search, run copies, chunk_len calls) and the
warm-up verification, on the config-4 and config-5 shapes."""
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

lib = ca.lib
lib.cg_diag_walk_stats.argtypes = [ctypes.c_uint32, ctypes.c_void_p]
res = {}
for name, n, size, params in [("c4", 16, 1 << 30, (64 << 10, 256 << 10, 1 << 20)),
                              ("c5", 16, 1 << 30, (256 << 10, 1 << 20, 4 << 20)),
                              ("c2", 256, 4 << 20, (256 << 10, 1 << 20, 4 << 20))]:
    d, offs = synth_nars_device(np.full(n, size, np.uint64))
    cap = ca.chunking.batch_capacity(offs, params[0])
    out = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
    ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params)
    lib.cg_diag_walk_stats(n, None)
    lib.cg_set_profiling(1)
    ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params)
    st = (ctypes.c_double * 5)()
    lib.cg_last_stage_times(st, 5)
    lib.cg_set_profiling(0)
    buf = np.zeros(8 * n, np.uint64)
    lib.cg_diag_walk_stats(n, buf.ctypes.data)
    lib.cg_diag_walk_stats(0, None)
    b = buf.reshape(n, 8).astype(float)
    worst = int(np.argmax(b[:, 0] + b[:, 1]))
    clk = 2.4e9 / 1e6  # clocks per us (s_memtime counts shader clocks)
    res[name] = {"walk_stage_ms": st[2], "worst_nar": worst,
                 "us": {k: round(b[worst, i] / clk, 1) for i, k in
                        ((0, "walk_loop"), (1, "verify"), (5, "piece_search"), (6, "run_copy"), (7, "chunk_len"))},
                 "chunks": int(b[worst, 2]), "piece_runs": int(b[worst, 3]), "rewalks": int(b[worst, 4]),
                 "median_us": {"walk_loop": round(float(np.median(b[:, 0])) / clk, 1),
                               "verify": round(float(np.median(b[:, 1])) / clk, 1)}}
    del d, out
print(json.dumps(res, indent=1))

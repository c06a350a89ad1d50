"""Diagnostic: producer/consumer spin shares of the SHA kernel on config-2/4 batches."""
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
from chunker_amd.nar import synth_nars  # noqa: E402

lib = ca.lib
lib.cg_diag_sha_stats.argtypes = [ctypes.c_uint32, ctypes.c_void_p]
lib.cg_diag_sha_mode.argtypes = [ctypes.c_uint32]
res = {}
runs = [("c2", 256, 4 << 20, (256 << 10, 1 << 20, 4 << 20), 0),
        ("c2_mode1", 256, 4 << 20, (256 << 10, 1 << 20, 4 << 20), 1),
        ("c2_mode2", 256, 4 << 20, (256 << 10, 1 << 20, 4 << 20), 2),
        ("c2_again", 256, 4 << 20, (256 << 10, 1 << 20, 4 << 20), 0),
        ("c4_quarter", 4, 1 << 30, (64 << 10, 256 << 10, 1 << 20), 0)]
if len(sys.argv) > 1:
    runs = [r for r in runs if r[0] in sys.argv[1:]]
for name, n, size, params, mode in runs:
    print("run", name, flush=True, file=sys.stderr)
    lib.cg_diag_sha_mode(mode)
    host, offs = synth_nars(np.full(n, size, np.uint64))
    d = torch.from_numpy(host).cuda()
    cap = ca.chunking.batch_capacity(offs, params[0])
    out = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
    first = ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params)
    nwg = (cap + 63) // 64
    lib.cg_diag_sha_stats(nwg, None)
    ca.lib.cg_set_profiling(1)
    first = ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params)
    st = (ctypes.c_double * 5)()
    ca.lib.cg_last_stage_times(st, 5)
    buf = np.zeros(8 * nwg, np.uint64)
    lib.cg_diag_sha_stats(nwg, buf.ctypes.data)
    lib.cg_diag_sha_stats(0, None)
    used = int((int(first[-1]) + 63) // 64)
    b = buf.reshape(-1, 8)[:used, :4].astype(float)
    worst = int(np.argmax(b[:, 3]))
    lens = np.frombuffer(out.cpu().numpy().tobytes()[:48 * int(first[-1])], dtype=np.uint64).reshape(-1, 6)[:, 1]
    max_blocks = int(lens.max()) // 64 + 1
    res[name] = {"digest_ms": st[4], "wgs": used, "mode": mode,
                 "worst_cycles_per_round": b[worst, 3] / (max_blocks * 64),
                 "worst_wg": {"prod_spin": b[worst, 0], "prod_total": b[worst, 1], "cons_spin": b[worst, 2],
                              "cons_total": b[worst, 3]},
                 "median_cons_spin_frac": float(np.median(b[:, 2] / np.maximum(b[:, 3], 1))),
                 "median_prod_spin_frac": float(np.median(b[:, 0] / np.maximum(b[:, 1], 1)))}
    del d, out
lib.cg_diag_sha_mode(0)
print(json.dumps(res, indent=1))

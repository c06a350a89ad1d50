"""Diagnostic: producer/consumer spin shares of the SHA kernel on config-2/4 batches."""
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
res = {}
for name, n, size, params in [("c2", 256, 4 << 20, (256 << 10, 1 << 20, 4 << 20)),
                              ("c4_quarter", 4, 1 << 30, (64 << 10, 256 << 10, 1 << 20))]:
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
    buf = np.zeros(4 * nwg, np.uint64)
    lib.cg_diag_sha_stats(nwg, buf.ctypes.data)
    lib.cg_diag_sha_stats(0, None)
    used = int((int(first[-1]) + 63) // 64)
    b = buf.reshape(-1, 4)[:used].astype(float)
    worst = int(np.argmax(b[:, 3]))
    res[name] = {"digest_ms": st[4], "wgs": used,
                 "worst_wg": {"prod_spin": b[worst, 0], "prod_total": b[worst, 1], "cons_spin": b[worst, 2],
                              "cons_total": b[worst, 3]},
                 "median_cons_spin_frac": float(np.median(b[:, 2] / np.maximum(b[:, 3], 1))),
                 "median_prod_spin_frac": float(np.median(b[:, 0] / np.maximum(b[:, 1], 1)))}
    del d, out
print(json.dumps(res))

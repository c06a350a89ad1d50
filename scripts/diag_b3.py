"""Diagnostic: BLAKE3 digest stage on config 3 by cg_diag_b3_mode (blake3.hip launch_blake3: 0 product, 1 no leaf loads,
2 / 4 / 8 in-wave fold full-exec / none / plain, 16 4-leaf lane subtrees); with and without leaf loads
(cg_diag_b3_mode 1 compresses register words instead: digests garbage), so the
compression's own time and the load path's share can be read apart."""
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
from chunker_amd._lib import lib  # noqa: E402
from chunker_amd.nar import synth_nars  # noqa: E402

lib.cg_diag_b3_mode.argtypes = [ctypes.c_uint32]
params = (256 << 10, 1 << 20, 4 << 20)
host, offs = synth_nars(np.full(256, 4 << 20, np.uint64))
d = torch.empty(len(host) + 256, dtype=torch.uint8, device="cuda")
d[: len(host)].copy_(torch.from_numpy(host))
cap = ca.chunking.batch_capacity(offs, params[0])
out = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
buf = (ctypes.c_double * 5)()
res = {}
for mode in [int(m) for m in (sys.argv[1] if len(sys.argv) > 1 else "0,8,0,8").split(",")]:
    lib.cg_diag_b3_mode(mode)
    lib.cg_set_profiling(1)
    ts = []
    for _ in range(5):
        ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params, hash=0, stream=st)
        lib.cg_last_stage_times(buf, 5)
        ts.append(buf[4])
    lib.cg_set_profiling(0)
    res.setdefault(f"mode{mode}", []).append(round(float(np.median(ts)), 4))
    got = out.cpu().numpy()
    if mode == 0:
        ref = got
    res[f"mode{mode}_same_digests_as_mode0"] = bool(np.array_equal(got, ref))
lib.cg_diag_b3_mode(0)
print(json.dumps(res))

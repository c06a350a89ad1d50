"""Diagnostic: SHA-256 digest stage of a GPU-filling batch (BASELINE config 4 shape,
16 x 1 GiB at 64K/256K/1M) by the number of quad workgroups allowed when the batch
fills the chip (cg_test_sha_quad_fill; 0 = the product's choice) and the number of
pair workgroups (cg_test_sha_split_max)."""
import os
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")
import argparse  # noqa: E402
import ctypes  # noqa: E402
import json  # noqa: E402
import sys  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, ".")
import chunker_amd as ca  # noqa: E402
from chunker_amd.nar import synth_nars_device  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--fill", default="0,8,16,32,64")
ap.add_argument("--pairs", default="256")
ap.add_argument("--nars", type=int, default=16)
ap.add_argument("--quad-max", default="256", help="cg_test_sha_quad_max values (quads outside fill mode)")
ap.add_argument("--params", default="65536,262144,1048576", help="config 4 (default); config 5: 262144,1048576,4194304")
args = ap.parse_args()
params = tuple(int(x) for x in args.params.split(","))
d, offs = synth_nars_device(np.full(args.nars, 1 << 30, np.uint64))
cap = ca.chunking.batch_capacity(offs, params[0])
out = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
sp = torch.cuda.current_stream().cuda_stream
buf = (ctypes.c_double * 5)()
ref = None
res = {}
for qmax, pairs, fill in [(q, p, f) for q in [int(x) for x in args.quad_max.split(",")]
                          for p in [int(x) for x in args.pairs.split(",")]
                          for f in [int(x) for x in args.fill.split(",")]]:
    if True:
        old_f = ca.lib.cg_test_sha_quad_fill(fill)
        old_p = ca.lib.cg_test_sha_split_max(pairs)
        old_q = ca.lib.cg_test_sha_quad_max(qmax)
        old_pf = ca.lib.cg_test_sha_pair_fill(pairs)  # --pairs also sets the GPU-filling pair count
        ms = []
        for it in range(4):
            ca.lib.cg_set_profiling(1)
            first = ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params, hash=1, stream=sp)
            ca.lib.cg_last_stage_times(buf, 5)
            if it >= 1:
                ms.append(buf[4])
        ca.lib.cg_test_sha_quad_fill(old_f)
        ca.lib.cg_test_sha_split_max(old_p)
        ca.lib.cg_test_sha_quad_max(old_q)
        ca.lib.cg_test_sha_pair_fill(old_pf)
        got = out[: int(first[-1]) * 48].cpu().numpy()
        if ref is None:
            ref = got
        assert np.array_equal(got, ref), "digests differ between tier layouts"
        res[f"quadmax{qmax}_pairs{pairs}_quadfill{fill}"] = round(float(np.median(ms)), 3)
print(json.dumps({"digest_ms": res, "chunks": int(first[-1])}))

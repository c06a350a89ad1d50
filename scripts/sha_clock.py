"""The shader clock the SHA-256 digest's longest chain actually ran at, for bench.py's
latency_floor (diagnostics build: k_sha256's per-workgroup record of consumer shader
clocks and consumer start/end on the 100 MHz global clock, cg_diag_sha_stats).

The length order hands the longest chunks to workgroup 0 (quad tier when there is one),
so clock = workgroup 0's consumer shader clocks / its wall time.  Runs the config's batch
(BASELINE shapes, bench.py CONFIGS) twice and reports the second.  Prints one JSON object."""
import os
os.environ["CHUNKER_AMD_DIAG"] = "1"
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")
import argparse  # noqa: E402
import ctypes  # noqa: E402
import json  # noqa: E402
import sys  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import chunker_amd as ca  # noqa: E402
from chunker_amd.nar import synth_nars_device  # noqa: E402

SHAPES = {"c2": (256, 4 << 20, (256 << 10, 1 << 20, 4 << 20)),
          "c4": (16, 1 << 30, (64 << 10, 256 << 10, 1 << 20)),
          "c5": (16, 1 << 30, (256 << 10, 1 << 20, 4 << 20))}
ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2", choices=sorted(SHAPES))
args = ap.parse_args()
n_nars, nar_bytes, params = SHAPES[args.config]
torch.cuda.set_device(0)
lib = ca.lib
lib.cg_diag_sha_stats.argtypes = [ctypes.c_uint32, ctypes.c_void_p]
d, offs = synth_nars_device(np.full(n_nars, nar_bytes, np.uint64))
cap = ca.chunking.batch_capacity(offs, params[0])
out = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
sp = torch.cuda.current_stream().cuda_stream
ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params, hash=1, stream=sp)
nwg = (cap + 7) // 8 + 8
lib.cg_diag_sha_stats(nwg, None)
first = ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params, hash=1, stream=sp)
buf = np.zeros(8 * nwg, np.uint64)
lib.cg_diag_sha_stats(nwg, buf.ctypes.data)
lib.cg_diag_sha_stats(0, None)
tiers = (ctypes.c_uint32 * 4)()
lib.cg_last_sha_tiers(tiers)
nq = int(tiers[0])
wg = buf.reshape(-1, 8).astype(np.float64)
lens = out[: 48 * int(first[-1])].cpu().numpy().view(ca.DESC_DTYPE)["length"].astype(np.int64)
longest = int(lens.max())


def clock(b):
    secs = (wg[b, 5] - wg[b, 4]) / 100e6
    return wg[b, 3] / secs / 1e9 if secs > 0 else None


quads = [clock(b) for b in range(nq) if wg[b, 3] > 0]
res = {"config": args.config, "what": "shader clock of the SHA-256 digest's longest chain (workgroup 0), "
       "consumer shader clocks / consumer wall time on the 100 MHz clock; diagnostics build",
       "clock_GHz": round(clock(0), 4), "longest_chunk_bytes": longest,
       "wg0_consumer_ms": round((wg[0, 5] - wg[0, 4]) / 1e5, 3),
       "quad_clock_GHz_median": round(float(np.median(quads)), 4) if quads else None,
       "cycles_per_round_wg0": round(wg[0, 3] / (((longest + 72) // 64) * 64), 2)}
print(json.dumps(res))

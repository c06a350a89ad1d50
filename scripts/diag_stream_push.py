"""Diagnostic: where a pipelined stream's time goes (cg_stream_*, descriptors only).
One synthetic NAR stream (default 1 GiB, SHA-256, 256K/1M/4M, 8 MiB pushes) per
in-flight budget, after one warm stream of the same budget; per budget the total rate,
the push latencies (median / p90 / max, ms), the time in finish + the final takes, and
the sum of push time.  CHUNKER_AMD_LIB=<other build> A/B-tests another library.
Prints one JSON object."""
import os
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
import argparse  # noqa: E402
import ctypes  # noqa: E402
import json  # noqa: E402
import sys  # noqa: E402
import time  # noqa: E402

import numpy as np  # noqa: E402

sys.path.insert(0, ".")
from chunker_amd._lib import DESC_DTYPE, lib  # noqa: E402
from chunker_amd.nar import synth_nars  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--gib", type=float, default=1.0)
ap.add_argument("--budgets", default="256,512,1024,2048")
ap.add_argument("--slice-mib", type=int, default=8)
ap.add_argument("--group-caps", default="0", help="MiB, 0 = the built-in rule (cg_test_stream_group_cap)")
ap.add_argument("--lanes", default="0", help="0 = the built-in rule (cg_test_stream_max_lanes)")
ap.add_argument("--eager", default="0", help="1 = launch a group whenever a lane is idle (cg_test_stream_eager)")
ap.add_argument("--repeat", type=int, default=1)
ap.add_argument("--fresh", action="store_true", help="push a fresh bytes copy of each slice (a reader's buffers)")
args = ap.parse_args()
N = int(args.gib * (1 << 30))
SL = args.slice_mib << 20
data, _ = synth_nars([N])


def run(inflight, n_bytes):
    st = ctypes.c_int(0)
    h = lib.cg_stream_new(256 << 10, 1 << 20, 4 << 20, 1, SL, inflight, ctypes.byref(st))
    out = np.zeros(8192, DESC_DTYPE)
    n = ctypes.c_size_t(0)
    pushes, cnt = [], 0
    t0 = time.perf_counter()
    keep = []
    for i in range(0, n_bytes, SL):
        if args.fresh:  # a new buffer per slice, as a reader returns (held until the end)
            buf = data[i:i + SL].tobytes()
            keep.append(buf)
            ptr = ctypes.cast(ctypes.c_char_p(buf), ctypes.c_void_p).value
        else:
            ptr = data.ctypes.data + i
        a = time.perf_counter()
        assert lib.cg_stream_push(h, ptr, min(SL, n_bytes - i)) == 0
        pushes.append((time.perf_counter() - a) * 1e3)
        assert lib.cg_stream_take(h, out.ctypes.data, len(out), ctypes.byref(n), 0) == 0
        cnt += n.value
    t1 = time.perf_counter()
    assert lib.cg_stream_finish(h) == 0
    while True:
        assert lib.cg_stream_take(h, out.ctypes.data, len(out), ctypes.byref(n), 1) == 0
        if not n.value:
            break
        cnt += n.value
    t2 = time.perf_counter()
    lib.cg_stream_free(h)
    p = np.array(pushes)
    return {"GiB_per_s": round(n_bytes / (t2 - t0) / 2**30, 3), "chunks": cnt,
            "push_ms": {"median": round(float(np.median(p)), 3), "p90": round(float(np.percentile(p, 90)), 3),
                        "max": round(float(p.max()), 3), "sum": round(float(p.sum()), 1)},
            "loop_ms": round((t1 - t0) * 1e3, 1), "finish_ms": round((t2 - t1) * 1e3, 1)}


res = {"lib": os.environ.get("CHUNKER_AMD_LIB", "default"), "bytes": N, "slice": SL,
       "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}
if not hasattr(lib, "cg_test_stream_eager"):  # an older build: its built-in shape only
    for name in ("cg_test_stream_eager", "cg_test_stream_max_lanes", "cg_test_stream_group_cap"):
        setattr(lib, name, lambda v: 0)
for eager in [int(x) for x in args.eager.split(",")]:
  lib.cg_test_stream_eager(eager)
  for lanes in [int(x) for x in args.lanes.split(",")]:
    lib.cg_test_stream_max_lanes(lanes)
    for cap in [int(x) for x in args.group_caps.split(",")]:
        lib.cg_test_stream_group_cap(cap << 20)
        for b in [int(x) for x in args.budgets.split(",")]:
            for r in range(args.repeat):
                k = f"inflight_{b}MiB_cap{cap}_lanes{lanes}_eager{eager}" + (f"_r{r}" if args.repeat > 1 else "")
                run(b << 20, min(N, 128 << 20))  # warm
                res[k] = run(b << 20, N)
                print(json.dumps({k: res[k]}), file=sys.stderr, flush=True)
lib.cg_test_stream_eager(0)
lib.cg_test_stream_group_cap(0)
lib.cg_test_stream_max_lanes(0)
print(json.dumps(res))

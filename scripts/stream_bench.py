"""Streaming rates: one 1 GiB synthetic NAR stream from
host memory, SHA-256, default params (256K/1M/4M), at the reference's read size
(8 MiB, src/chunking.rs:713-716 with the default cap :417).

* ChunkStream: the pipelined engine stream (cg_stream_*) behind the Python mirror
  (payload objects included), for several in-flight HBM budgets;
* engine_stream: cg_stream_push / cg_stream_take alone (descriptors only: what a Rust
  caller pays before its zero-copy split_to);
* engine_push: the synchronous PushChunker handle (cg_push_*), one round trip per slice;
* cpu_push: the oracle's PushChunker restatement (serial FastCDC, SHA-NI, digests on a
  16-thread pool when a drain emits > 4 chunks, as the reference's par_iter does,
  src/chunking.rs:637-641), 8 MiB pushes, over the same 1 GiB.
Every GPU variant is checked chunk for chunk against the eager result."""
import os
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")  # placeholder GEAR: see tables/README.md
os.environ.pop("CHUNKER_READ_SLICE_CAP_BYTES", None)  # the reference's default sizing
import sys  # noqa: E402

# 16 hardware queues as bench.py, or --hw-queues N; before HIP initialises
os.environ["GPU_MAX_HW_QUEUES"] = sys.argv[sys.argv.index("--hw-queues") + 1] if "--hw-queues" in sys.argv else "16"
import ctypes  # noqa: E402
import io  # noqa: E402
import json  # noqa: E402
import time  # noqa: E402

import numpy as np  # noqa: E402

sys.path.insert(0, ".")
import chunker_amd as ca  # noqa: E402
from chunker_amd._lib import DESC_DTYPE, lib  # noqa: E402
from chunker_amd.nar import synth_nars  # noqa: E402

N = 1 << 30
SL = 8 << 20
data, _ = synth_nars([N])
raw = data.tobytes()
res = {"workload": "1 GiB synthetic NAR stream, SHA-256, 256K/1M/4M, 8 MiB reads",
       "hw_queues": os.environ["GPU_MAX_HW_QUEUES"]}
eager = ca.chunk_descriptors_array(data)
ref = [(int(d["offset"]), int(d["length"]), bytes(d["hash"])) for d in eager]
res["chunks"] = len(ref)


def key(chunks):
    return [(c.offset, c.length, c.hash) for c in chunks]


for inflight in (512 << 20, 1 << 30, 2 << 30):
    os.environ["CHUNKER_AMD_STREAM_INFLIGHT_BYTES"] = str(inflight)
    list(ca.ChunkStream(io.BytesIO(raw[: 64 << 20])))  # warm (allocations)
    t0 = time.perf_counter()
    chunks = list(ca.ChunkStream(io.BytesIO(raw)))
    dt = time.perf_counter() - t0
    assert key(chunks) == ref
    res[f"ChunkStream_inflight_{inflight >> 20}MiB"] = {"GiB_per_s": round(N / dt / 2**30, 3), "s": round(dt, 3)}
    del chunks

for inflight in (512 << 20, 1 << 30, 2 << 30):
    st = ctypes.c_int(0)
    h = lib.cg_stream_new(256 << 10, 1 << 20, 4 << 20, 1, SL, inflight, ctypes.byref(st))
    out = np.zeros(8192, DESC_DTYPE)
    n = ctypes.c_size_t(0)
    got = []
    t0 = time.perf_counter()
    for i in range(0, N, SL):
        assert lib.cg_stream_push(h, data.ctypes.data + i, min(SL, N - i)) == 0
        assert lib.cg_stream_take(h, out.ctypes.data, len(out), ctypes.byref(n), 0) == 0
        got.append(out[: n.value].copy())
    assert lib.cg_stream_finish(h) == 0
    while True:
        assert lib.cg_stream_take(h, out.ctypes.data, len(out), ctypes.byref(n), 1) == 0
        if not n.value:
            break
        got.append(out[: n.value].copy())
    dt = time.perf_counter() - t0
    lib.cg_stream_free(h)
    g = np.concatenate(got)
    assert [(int(x["offset"]), int(x["length"]), bytes(x["hash"])) for x in g] == ref
    res[f"engine_stream_inflight_{inflight >> 20}MiB"] = {"GiB_per_s": round(N / dt / 2**30, 3), "s": round(dt, 3)}

st = ctypes.c_int(0)
h = lib.cg_push_new(256 << 10, 1 << 20, 4 << 20, 1, ctypes.byref(st))
out = np.zeros(4096, DESC_DTYPE)
n = ctypes.c_size_t(0)
got = []
M = 256 << 20  # the synchronous handle is slow: a 256 MiB prefix
t0 = time.perf_counter()
for i in range(0, M, SL):
    assert lib.cg_push_push(h, data.ctypes.data + i, SL, out.ctypes.data, len(out), ctypes.byref(n)) == 0
    got.append(out[:n.value].copy())
dt = time.perf_counter() - t0
lib.cg_push_free(h)
res["engine_push_sync_8MiB"] = {"GiB_per_s": round(M / dt / 2**30, 3), "sample_bytes": M,
                                "ms_per_push": round(dt * 1e3 / (M // SL), 2)}

from oracle import oracle as O  # noqa: E402

for nt in (1, 16):
    p = O.Push(nthreads=nt)
    t0 = time.perf_counter()
    cnt = 0
    for i in range(0, N, SL):
        cnt += len(p.push(data[i:i + SL]))
    cnt += len(p.finish())
    dt = time.perf_counter() - t0
    assert cnt == len(ref)
    res[f"cpu_push_8MiB_{nt}t"] = {"GiB_per_s": round(N / dt / 2**30, 3), "threads": nt, "kind": "port"}
print(json.dumps(res))

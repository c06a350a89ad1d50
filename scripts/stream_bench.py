"""Streaming rates: one 1 GiB xorshift stream from host
memory through ChunkStream (reader slices) and PushChunker (caller slices, the NIF's
pattern), SHA-256, default params.  Reported per slice size; the GPU ChunkStream default
is the 256 MiB slice (chunking.stream_read_size).  CPU: the oracle's PushChunker
restatement (serial scan + serial SHA-NI, one thread) on a 256 MiB sample, 8 MiB pushes."""
import os
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")  # placeholder GEAR: see tables/README.md
import io
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import chunker_amd as ca  # noqa: E402
from chunker_amd.nar import synth_nars  # noqa: E402

N = 1 << 30
data, _ = synth_nars([N])
raw = data.tobytes()
res = {"workload": "1 GiB synthetic NAR stream, SHA-256, 256K/1M/4M"}
ref = None
# ChunkStream: the reference's sizing with its 8 MiB default cap (env pinned), then the
# GPU default (env unset: 256 MiB slices, chunking.stream_read_size)
for cap in (8 << 20, None):
    if cap:
        os.environ["CHUNKER_READ_SLICE_CAP_BYTES"] = str(cap)
    else:
        os.environ.pop("CHUNKER_READ_SLICE_CAP_BYTES", None)
    rs = ca.chunking.stream_read_size(4 << 20)
    t0 = time.perf_counter()
    chunks = ca.chunk_stream(io.BytesIO(raw))
    dt = time.perf_counter() - t0
    key = [(c.offset, c.length, c.hash) for c in chunks]
    ref = ref or key
    assert key == ref
    res[f"stream_read_{rs >> 20}MiB"] = {"GiB_per_s": round(N / dt / 2**30, 3), "s": round(dt, 3),
                                          "chunks": len(chunks)}
for sl in (8 << 20, 64 << 20, 256 << 20):
    p = ca.PushChunker()
    t0 = time.perf_counter()
    out = []
    for i in range(0, N, sl):
        out += p.push(raw[i:i + sl])
    out += p.finish()
    dt = time.perf_counter() - t0
    assert [(c.offset, c.length, c.hash) for c in out] == ref
    res[f"push_{sl >> 20}MiB"] = {"GiB_per_s": round(N / dt / 2**30, 3), "s": round(dt, 3)}
# engine alone: cg_push_push on slices of one host array (descriptors only, no payload
# objects) -- what a Rust caller pays before its zero-copy split_to
import ctypes  # noqa: E402

from chunker_amd._lib import DESC_DTYPE, lib  # noqa: E402

for sl in (8 << 20, 64 << 20, 256 << 20):
    st = ctypes.c_int(0)
    h = lib.cg_push_new(256 << 10, 1 << 20, 4 << 20, 1, ctypes.byref(st))
    out = np.zeros(4096, DESC_DTYPE)
    n = ctypes.c_size_t(0)
    got = []
    t0 = time.perf_counter()
    for i in range(0, N, sl):
        assert lib.cg_push_push(h, data.ctypes.data + i, min(sl, N - i), out.ctypes.data, len(out), ctypes.byref(n)) == 0
        got.append(out[:n.value].copy())
    assert lib.cg_push_finish(h, out.ctypes.data, len(out), ctypes.byref(n)) == 0
    got.append(out[:n.value].copy())
    dt = time.perf_counter() - t0
    lib.cg_push_free(h)
    g = np.concatenate(got)
    assert [(int(x["offset"]), int(x["length"]), bytes(x["hash"])) for x in g] == ref
    res[f"engine_push_{sl >> 20}MiB"] = {"GiB_per_s": round(N / dt / 2**30, 3), "s": round(dt, 3),
                                          "ms_per_push": round(dt * 1e3 / (N // sl + 1), 2)}
eager = ca.chunk_data(raw)
assert [(c.offset, c.length, c.hash) for c in eager] == ref
from oracle import oracle as O  # noqa: E402

S = 256 << 20
p = O.Push()
t0 = time.perf_counter()
n = 0
for i in range(0, S, 8 << 20):
    n += len(p.push(data[i:i + (8 << 20)]))
n += len(p.finish())
dt = time.perf_counter() - t0
res["cpu_push_8MiB"] = {"GiB_per_s": round(S / dt / 2**30, 3), "sample_bytes": S, "threads": 1, "kind": "port"}
print(json.dumps(res))

"""Stream shape sweep: engine stream rates (cg_stream_push / take,
descriptors only) over 1 GiB and 4 GiB synthetic NAR streams, SHA-256, 256K/1M/4M, 8 MiB
pushes, at the process's GPU_MAX_HW_QUEUES (--hw-queues N, default 4 = HIP's default),
for digest-lane counts x group policies (cg_test_stream_max_lanes, cg_test_stream_eager:
0 = launch a group at group_bytes, waiting for a lane; 2 = keep accumulating while every
lane is busy).  Every run is checked chunk for chunk against the eager device result."""
import os
import sys

os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")
os.environ["GPU_MAX_HW_QUEUES"] = sys.argv[sys.argv.index("--hw-queues") + 1] if "--hw-queues" in sys.argv else "4"
import ctypes  # noqa: E402
import json  # noqa: E402
import time  # noqa: E402

import numpy as np  # noqa: E402

sys.path.insert(0, ".")
import chunker_amd as ca  # noqa: E402
from chunker_amd._lib import DESC_DTYPE, lib  # noqa: E402
from chunker_amd.nar import synth_nars  # noqa: E402

SL = 8 << 20
shapes = [(0, 0), (1, 0), (1, 2), (2, 0), (2, 2)]  # (max lanes, eager mode); lanes 0 = the built-in rule
if "--shapes" in sys.argv:
    shapes = [tuple(int(v) for v in s.split(":")) for s in sys.argv[sys.argv.index("--shapes") + 1].split(",")]
if "--tiers-off" in sys.argv:  # SHA-256 latency tiers off (A/B)
    lib.cg_test_sha_tiers(0, 0)
    lib.cg_test_sha_tiers_fill(0, 0)
sizes = [1 << 30, 4 << 30]
if "--sizes-gib" in sys.argv:
    sizes = [int(v) << 30 for v in sys.argv[sys.argv.index("--sizes-gib") + 1].split(",")]
res = {"workload": "synthetic NAR stream, SHA-256, 256K/1M/4M, 8 MiB pushes, 2 GiB in-flight budget",
       "hw_queues": os.environ["GPU_MAX_HW_QUEUES"], "sha_tiers": "--tiers-off" not in sys.argv, "rows": []}


def run(data, lanes, eager):
    lib.cg_test_stream_max_lanes(lanes)
    lib.cg_test_stream_eager(eager)
    st = ctypes.c_int(0)
    h = lib.cg_stream_new(256 << 10, 1 << 20, 4 << 20, 1, SL, 0, ctypes.byref(st))
    assert h, st.value
    out = np.zeros(16384, DESC_DTYPE)
    n = ctypes.c_size_t(0)
    got = []
    N = len(data)
    t0 = time.perf_counter()
    for i in range(0, N, SL):
        assert lib.cg_stream_push(h, data.ctypes.data + i, min(SL, N - i)) == 0, ca._lib.last_error()
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
    lib.cg_test_stream_max_lanes(0)
    lib.cg_test_stream_eager(0)
    return np.concatenate(got), dt


for N in sizes:
    data, _ = synth_nars([N])
    eager = ca.chunk_descriptors_array(data)
    run(data[: 64 << 20], 0, 0)  # warm
    for lanes, eager_mode in shapes:
        g, dt = run(data, lanes, eager_mode)
        assert len(g) == len(eager) and np.array_equal(g.view(np.uint8), eager.view(np.uint8)), (N, lanes, eager_mode)
        row = {"GiB": N >> 30, "lanes": lanes or "rule", "mode": eager_mode, "GiB_per_s": round(N / dt / 2**30, 3),
               "s": round(dt, 3)}
        res["rows"].append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    del data, eager
print(json.dumps(res))

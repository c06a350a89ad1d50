"""Diagnostic: where the host-to-host rate of concurrent host-entry callers goes
(bench.py `concurrent.e2e`).  Config-2 batches (256 x 4 MiB, SHA-256) in pinned host
memory; K threads; per mode the aggregate GiB/s and each call's latency (ms):

  h2d      K threads, each copying its batch to HBM on its own stream (the link alone);
  h2d_busy the same while K device-resident batches digest on other streams (the link
           under compute load);
  e2e      K threads calling cg_chunk_batch (H2D + chunk + digest + D2H).
(Round 3 also tried chaining the callers' input copies device-wide in issue order, so
they would cross the link one at a time: K8 28.2 / K16 24.4 GiB/s against 36.7 / 45.4
unchained, profiles/r03_v4_diag_e2e.json; removed.)
Prints one JSON object."""
import os
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
import argparse  # noqa: E402
import ctypes  # noqa: E402
import json  # noqa: E402
import sys  # noqa: E402
import threading  # noqa: E402
import time  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, ".")
import chunker_amd as ca  # noqa: E402
from chunker_amd.nar import synth_nars  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", default="4,8,16")
ap.add_argument("--reps", type=int, default=4)
ap.add_argument("--modes", default="h2d,h2d_busy,e2e")
args = ap.parse_args()
GIB = 1 << 30
params = (256 << 10, 1 << 20, 4 << 20)
n_per, nar = 256, 4 << 20
ks = [int(k) for k in args.k.split(",")]
host0, offs = synth_nars(np.full(n_per, nar, np.uint64))
nbytes = int(offs[-1])
cap = ca.chunking.batch_capacity(offs, params[0])
kmax = max(ks)
pins = []
for _ in range(kmax):
    t = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    t.numpy()[:] = host0
    pins.append(t)
devs = [torch.empty(nbytes + 256, dtype=torch.uint8, device="cuda") for _ in range(kmax)]
outs = [np.zeros(cap, ca.DESC_DTYPE) for _ in range(kmax)]
firsts = [np.zeros(n_per + 1, np.uint64) for _ in range(kmax)]
streams = [torch.cuda.Stream() for _ in range(kmax)]


def run(K, fn, reps):
    lat = [[] for _ in range(K)]
    bar = threading.Barrier(K + 1)
    errs = []

    def work(k):
        bar.wait()
        for _ in range(reps):
            t0 = time.perf_counter()
            try:
                fn(k)
            except Exception as e:  # noqa: BLE001
                errs.append(repr(e))
                return
            lat[k].append((time.perf_counter() - t0) * 1e3)

    th = [threading.Thread(target=work, args=(k,)) for k in range(K)]
    for x in th:
        x.start()
    bar.wait()
    t0 = time.perf_counter()
    for x in th:
        x.join()
    dt = time.perf_counter() - t0
    if errs:
        raise RuntimeError(errs[0])
    allv = [v for row in lat for v in row]
    return {"GiBps": round(K * reps * nbytes / dt / GIB, 2), "lat_ms_median": round(float(np.median(allv)), 1),
            "lat_ms_max": round(float(np.max(allv)), 1)}


def h2d(k):
    with torch.cuda.stream(streams[k]):
        devs[k][:nbytes].copy_(pins[k], non_blocking=True)
    streams[k].synchronize()


def e2e(k):
    st = ca.lib.cg_chunk_batch(ctypes.c_void_p(pins[k].data_ptr()), offs.ctypes.data, n_per, *params, 1,
                               outs[k].ctypes.data, cap, firsts[k].ctypes.data)
    if st:
        raise RuntimeError(f"status {st}: {ca._lib.last_error()}")


res = {"batch_GiB": nbytes / GIB, "reps": args.reps}
modes = args.modes.split(",")
for K in ks:
    r = {}
    if "h2d" in modes:
        run(K, h2d, 1)
        r["h2d"] = run(K, h2d, args.reps)
    if "h2d_busy" in modes:
        # K device-resident digests on other streams while K threads copy
        bsy = [torch.empty(nbytes + 256, dtype=torch.uint8, device="cuda") for _ in range(2)]
        for b in bsy:
            b[:nbytes].copy_(pins[0])
        stop = threading.Event()
        dout = [torch.empty(cap * 48, dtype=torch.uint8, device="cuda") for _ in range(2)]
        bst = [torch.cuda.Stream() for _ in range(2)]

        def busy(i):
            while not stop.is_set():
                ca.chunk_batch_device(bsy[i].data_ptr(), offs, dout[i].data_ptr(), cap, *params, hash=1,
                                      stream=bst[i].cuda_stream)

        bt = [threading.Thread(target=busy, args=(i,)) for i in range(2)]
        for x in bt:
            x.start()
        time.sleep(0.2)
        r["h2d_busy"] = run(K, h2d, args.reps)
        stop.set()
        for x in bt:
            x.join()
        del bsy, dout
    if "e2e" in modes:
        run(K, e2e, 1)
        r["e2e"] = run(K, e2e, args.reps)
    res[f"K{K}"] = r
    print(json.dumps({f"K{K}": r}), file=sys.stderr, flush=True)
print(json.dumps(res))

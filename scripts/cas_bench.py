"""Node::put on the GPU: device-resident GiB/s of
cg_node_put_batch_device (FastCDC + SHA-256 descriptors + one SHAKE-256 ContentId per
chunk + one manifest id per NAR) next to cg_chunk_batch_device alone, and the CAS
kernel by itself over the same chunk spans (cg_cas_ids_device).  Stage times come
from the library's HIP events (cg_last_stage_times; stage 6 = CAS on the side
stream).  CPU baseline: oracle.node_put (hashlib SHAKE-256 + the C FastCDC/SHA-NI
port) on a 16-thread pool over a bounded sample of NARs."""
import os
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")  # placeholder GEAR: see tables/README.md
import argparse
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import chunker_amd as ca  # noqa: E402
from chunker_amd import cas  # noqa: E402
from chunker_amd.nar import synth_nars  # noqa: E402

CFG = {"c2": (256, 4 << 20, (256 << 10, 1 << 20, 4 << 20)),
       "c4": (16, 1 << 30, (64 << 10, 256 << 10, 1 << 20))}
ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2", choices=sorted(CFG))
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--cpu-sample-nars", type=int, default=8)
args = ap.parse_args()
n, size, params = CFG[args.config]
host, offs = synth_nars(np.full(n, size, np.uint64))
d = torch.from_numpy(host).cuda()
cap = ca.chunking.batch_capacity(offs, params[0])
out = torch.zeros(cap * 48, dtype=torch.uint8, device="cuda")
ids = torch.zeros(cap * 32, dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
ca.lib.cg_set_profiling(1)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    t0, stages = time.perf_counter(), []
    for _ in range(args.steps):
        fn()
        buf = np.zeros(8)
        k = ca.lib.cg_last_stage_times(buf.ctypes.data, 8)
        stages.append(buf[:k])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / args.steps, np.mean(stages, axis=0)


res = {"workload": f"{n}x{size} NARs {params}", "bytes": int(len(host))}
dt, sg = timed(lambda: ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params, stream=st))
res["chunk_sha256"] = {"GiB_per_s": round(len(host) / dt / 2**30, 3), "ms": round(dt * 1e3, 2),
                       "stages_ms": [round(x, 3) for x in sg]}
first = None


def put():
    global first
    first, _ = cas.node_put_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, ids.data_ptr(), *params, stream=st)


dt, sg = timed(put)
res["node_put"] = {"GiB_per_s": round(len(host) / dt / 2**30, 3), "ms": round(dt * 1e3, 2),
                   "stages_ms": [round(x, 3) for x in sg], "chunks": int(first[-1])}
# CAS kernel alone over the chunk spans
descs = out.cpu().numpy().view(ca.DESC_DTYPE)[:int(first[-1])]
nar_of = np.repeat(np.arange(n), np.diff(first).astype(np.int64))
abs_off = torch.from_numpy((descs["offset"] + offs[nar_of]).astype(np.int64)).cuda()
lens = torch.from_numpy(descs["length"].astype(np.int64)).cuda()
ids2 = torch.zeros_like(ids)
m = len(descs)
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
cas.content_ids_device(d.data_ptr(), abs_off.data_ptr(), lens.data_ptr(), m, cas.ObjectKind.Chunk, ids2.data_ptr(), st)
ev0.record()
for _ in range(args.steps):
    cas.content_ids_device(d.data_ptr(), abs_off.data_ptr(), lens.data_ptr(), m, cas.ObjectKind.Chunk, ids2.data_ptr(),
                           st)
ev1.record()
torch.cuda.synchronize()
ms = ev0.elapsed_time(ev1) / args.steps
longest = int(descs["length"].max())
res["cas_only"] = {"GiB_per_s": round(len(host) / (ms / 1e3) / 2**30, 3), "ms": round(ms, 2),
                   "longest_chunk": longest, "longest_blocks": (longest + 26) // 136 + 1,
                   "ns_per_block_longest_lane": round(ms * 1e6 / ((longest + 26) // 136 + 1), 1)}
assert torch.equal(ids2[:m * 32], ids[:m * 32]), "cas-only ids differ from node_put ids"
# CPU baseline: oracle Node::put on a bounded sample
if args.cpu_sample_nars:
    from oracle import oracle as O

    k = min(args.cpu_sample_nars, n)
    sample = host[:int(offs[k])]
    t0 = time.perf_counter()
    for i in range(k):
        O.node_put(sample[offs[i]:offs[i + 1]], *params, nthreads=16)
    dt = time.perf_counter() - t0
    res["cpu_node_put"] = {"GiB_per_s": round(len(sample) / dt / 2**30, 3), "threads": 16, "nars": k,
                           "kind": "port"}
print(json.dumps(res))

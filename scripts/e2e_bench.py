"""End-to-end rate from host memory: NAR bytes start in host RAM
(pageable numpy, or pinned), cross PCIe, are chunked + digested on the GPU, and the
descriptors come back to host RAM.  Host API cg_chunk_batch (one call per batch)."""
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
from chunker_amd.nar import synth_nars  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nars", type=int, default=256)
ap.add_argument("--size", type=int, default=4 << 20)
ap.add_argument("--algo", type=int, default=1)
ap.add_argument("--steps", type=int, default=3)
args = ap.parse_args()
params = (256 << 10, 1 << 20, 4 << 20)
host, offs = synth_nars(np.full(args.nars, args.size, np.uint64))
pinned = torch.empty(len(host), dtype=torch.uint8).pin_memory()
pinned.numpy()[:] = host
res = {}
for name, buf in [("pageable", host), ("pinned", pinned.numpy())]:
    out = None
    d, first = ca.chunking.chunk_batch_flat(buf, offs, *params, hash=args.algo)  # warm-up
    t0 = time.perf_counter()
    for _ in range(args.steps):
        d, first = ca.chunking.chunk_batch_flat(buf, offs, *params, hash=args.algo, out=out)
    dt = (time.perf_counter() - t0) / args.steps
    res[name] = {"GiB_per_s": round(len(host) / dt / 2**30, 3), "ms": round(dt * 1e3, 2), "chunks": len(d)}
# H2D alone for reference
dev = torch.empty(len(host), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(args.steps):
    dev.copy_(pinned, non_blocking=True)
torch.cuda.synchronize()
res["h2d_pinned_GBps"] = round(len(host) * args.steps / (time.perf_counter() - t0) / 1e9, 2)
print(json.dumps({"workload": f"{args.nars}x{args.size} NARs algo={args.algo}", **res}))

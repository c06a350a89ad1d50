"""Digest-pipeline sweep (round 6): steady-state GiB/s of one caller's cg_pipeline over
distinct device-resident batches, per (group, lanes) setting.

Each in-flight slot owns its own input batch (synth_nars_device with first_index = slot *
nars) and output array; the pipeline is filled before the timed region, which then counts
`--steps` completions.  `--check` compares every slot's descriptors of the last pass with
cg_chunk_batch_device on the same input (the per-batch path, itself oracle-checked by
tests/test_gpu_parity.py).

usage: python scripts/pipe_bench.py --config c2 --sweep 16x2,24x2,32x1 --steps 60
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")

CONFIGS = {"c2": (256, 4 << 20, (256 << 10, 1 << 20, 4 << 20), 1),
           "c3": (256, 4 << 20, (256 << 10, 1 << 20, 4 << 20), 0),
           "c4": (16, 1 << 30, (64 << 10, 256 << 10, 1 << 20), 1),
           "c5": (16, 1 << 30, (256 << 10, 1 << 20, 4 << 20), 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--sweep", default="16x2", help="GROUPxLANES[:DEPTH],... (depth default (lanes+1)*group)")
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--slots", type=int, default=0, help="distinct input batches (0 = the largest depth)")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--profile", action="store_true", help="time each merged digest kernel (cg_set_profiling(2))")
    ap.add_argument("--sha-occ", default="", help="LATENCY,FILL workgroups per CU (cg_test_sha_occupancy)")
    ap.add_argument("--legacy", type=int, default=0, help="also time the round-5 async_after path at this depth")
    args = ap.parse_args()

    import torch

    torch.cuda.set_device(0)
    import chunker_amd as ca
    from chunker_amd.nar import synth_nars_device

    n_per, nar_bytes, params, algo = CONFIGS[args.config]
    sweep = []
    for item in args.sweep.split(","):
        gl, _, d = item.partition(":")
        g, l = (int(v) for v in gl.split("x"))
        sweep.append((g, l, int(d) if d else (l + 1) * g))
    slots = args.slots or max(d for _, _, d in sweep)
    t = time.perf_counter()
    ins, offs = [], None
    for s in range(slots):
        d, offs = synth_nars_device(np.full(n_per, nar_bytes, np.uint64), first_index=s * n_per)
        ins.append(d)
    torch.cuda.synchronize()
    synth_s = time.perf_counter() - t
    cap = ca.chunking.batch_capacity(offs, params[0])
    outs = [torch.empty(cap * 48, dtype=torch.uint8, device="cuda") for _ in range(slots)]
    total = int(offs[-1])
    res = {"config": args.config, "slots": slots, "synth_s": round(synth_s, 1),
           "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "4(default)"),
           "pipe_streams": os.environ.get("CHUNKER_AMD_PIPE_STREAMS", "high"), "runs": []}

    def run(pipe, n, t_issue, lat, firsts):
        for k in range(n):
            s = k % slots
            t_issue[k] = time.perf_counter()
            for tag, first in pipe.submit(ins[s].data_ptr(), offs, outs[s].data_ptr(), cap, tag=k):
                lat.append(time.perf_counter() - t_issue[tag])
                firsts[tag % slots] = first
        return pipe

    if args.profile:
        ca.lib.cg_set_profiling(2)
    if args.sha_occ:
        a, b = (int(v) for v in args.sha_occ.split(","))
        ca.lib.cg_test_sha_occupancy(0, a)
        ca.lib.cg_test_sha_occupancy(1, b)
        res["sha_occ"] = [a, b]
    for g, l, depth in sweep:
        if depth > slots:
            continue
        pipe = ca.BatchPipeline(depth, *params, hash=algo, group=g, lanes=l)
        t_issue, lat, firsts = {}, [], {}
        run(pipe, depth * 2, t_issue, lat, firsts)  # warm-up: every workspace sized
        lat.clear()
        # fill, untimed: depth - 1 queued (the next submit waits for the oldest)
        t_fill = time.perf_counter()
        base = depth * 2
        for k in range(depth - 1):
            s = (base + k) % slots
            t_issue[base + k] = time.perf_counter()
            pipe.submit(ins[s].data_ptr(), offs, outs[s].data_ptr(), cap, tag=base + k)
        fill_s = time.perf_counter() - t_fill
        t0 = time.perf_counter()
        done = 0
        k = base + depth - 1
        while done < args.steps:
            s = k % slots
            t_issue[k] = time.perf_counter()
            for tag, first in pipe.submit(ins[s].data_ptr(), offs, outs[s].data_ptr(), cap, tag=k):
                lat.append(time.perf_counter() - t_issue[tag])
                firsts[tag % slots] = first
                done += 1
            k += 1
        el = time.perf_counter() - t0
        t_dr = time.perf_counter()
        for tag, first in pipe.drain():
            firsts[tag % slots] = first
        drain_s = time.perf_counter() - t_dr
        st = pipe.stats()
        if st.get("timed_groups"):
            st["digest_ms_mean"] = round(st["digest_ms_sum"] / st["timed_groups"], 3)
            st["digest_GiB_mean"] = round(st["digest_bytes_sum"] / st["timed_groups"] / 2**30, 2)
        row = {"group": g, "lanes": l, "depth": depth, "GiBps": round(done * total / el / 2**30, 2),
               "steps": done, "ms": round(el * 1e3, 2), "fill_ms": round(fill_s * 1e3, 2),
               "drain_ms": round(drain_s * 1e3, 2),
               "lat_p50_ms": round(float(np.percentile(lat, 50)) * 1e3, 1),
               "lat_p99_ms": round(float(np.percentile(lat, 99)) * 1e3, 1), "stats": st}
        if args.check:
            bad = 0
            for s in range(slots):
                if s not in firsts:
                    continue
                n = int(firsts[s][-1])
                got = outs[s][: n * 48].cpu().numpy()
                ref = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
                rf = ca.chunk_batch_device(ins[s].data_ptr(), offs, ref.data_ptr(), cap, *params, hash=algo)
                torch.cuda.synchronize()
                if not (np.array_equal(rf, firsts[s]) and np.array_equal(ref[: n * 48].cpu().numpy(), got)):
                    bad += 1
            row["check"] = {"slots_checked": len(firsts), "mismatched": bad}
        pipe.close()
        res["runs"].append(row)
        print(json.dumps(row), flush=True)
    if args.legacy:
        os.environ["_"] = ""
        pipe = ca.BatchPipeline(args.legacy, *params, hash=algo, group=0)
        t_issue, lat, firsts = {}, [], {}
        run(pipe, args.legacy * 2, t_issue, lat, firsts)
        pipe.drain()
        lat.clear()
        t0 = time.perf_counter()
        run(pipe, args.steps, t_issue, lat, firsts)
        pipe.drain()
        el = time.perf_counter() - t0
        row = {"legacy_async_after_depth": args.legacy, "GiBps": round(args.steps * total / el / 2**30, 2)}
        res["runs"].append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

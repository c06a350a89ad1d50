"""bench.py -- device-resident FastCDC + per-chunk digest throughput on MI355X.

Metric (BASELINE.json): "device-resident GiB/s FastCDC+SHA-256 over synthetic NARs".
A step is one pass of the hot path (candidate scan -> cut walk -> descriptor
assembly -> per-chunk digest) over one batch of synthetic NARs already resident in
HBM, through the C ABI entry cg_chunk_batch_device.  Default workload = BASELINE
config 2: 256 x 4 MiB NARs, 256K/1M/4M, SHA-256, per GPU.

Multi-GPU (torchrun, one rank per GPU): every rank owns its own batch of NARs
(NAR indices rank*n .. rank*n+n-1: one-file-per-GPU sharding, weak scaling); after
each step the per-NAR descriptor counts and the descriptor arrays are gathered to
rank 0 over RCCL (the only exchange the path has).  value = all ranks' bytes /
max-over-ranks time.

Extra JSON keys: roofline (dominant kernel, HIP-event timed on the stream the
kernels run on), cpu_baseline (the oracle's restatement of chunk_data, rank 0),
stages_ms (per-stage device times), chunks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md
GIB = 1024 ** 3

CONFIGS = {
    # name: (n_nars, nar_bytes, (min, avg, max), algo, description)
    "c2": (256, 4 << 20, (256 << 10, 1 << 20, 4 << 20), 1,
           "256x4MiB synthetic NARs, 256K/1M/4M, SHA-256 (BASELINE config 2)"),
    "c3": (256, 4 << 20, (256 << 10, 1 << 20, 4 << 20), 0,
           "256x4MiB synthetic NARs, 256K/1M/4M, BLAKE3 (BASELINE config 3)"),
    "c4": (16, 1 << 30, (64 << 10, 256 << 10, 1 << 20), 1,
           "16x1GiB synthetic NARs, 64K/256K/1M, SHA-256 (BASELINE config 4)"),
    "c5": (16, 1 << 30, (256 << 10, 1 << 20, 4 << 20), 1,
           "16x1GiB synthetic NARs per GPU, 256K/1M/4M, SHA-256 (BASELINE config 5 shard)"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--zeros", action="store_true", help="all-zero payloads (the reference's bench data)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-nars", type=int, default=0, help="0 = whole batch (config c2/c3)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    import chunker_amd as ca
    from chunker_amd.nar import synth_nars

    n_nars, nar_bytes, params, algo, desc = CONFIGS[args.config]
    sizes = np.full(n_nars, nar_bytes, np.uint64)
    host, offs = synth_nars(sizes, zeros=args.zeros, first_index=rank * n_nars)
    total_bytes = int(offs[-1])
    d_data = torch.empty(total_bytes + 256, dtype=torch.uint8, device="cuda")
    d_data[:total_bytes].copy_(torch.from_numpy(host))
    cap = ca.chunking.batch_capacity(offs, params[0])
    d_out = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    sptr = stream.cuda_stream

    from chunker_amd.dist import gather_descriptors

    def step():
        first = ca.chunk_batch_device(d_data.data_ptr(), offs, d_out.data_ptr(), cap, *params, hash=algo,
                                      stream=sptr)
        if world > 1:  # descriptors to rank 0 over RCCL (the path's only exchange)
            gather_descriptors(d_out, int(first[-1]))
        return first

    for _ in range(args.warmup):
        first = step()
    # Per-stage device times: HIP events the library records on the stream the kernels
    # run on, live inside the timed region (each step already ends in a stream sync
    # for the NAR->chunk index, so reading them adds only host bookkeeping).
    ca.lib.cg_set_profiling(1)
    stage = np.zeros((max(args.steps, 1), 5))
    buf = (np.ctypeslib.ctypes.c_double * 5)()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        first = step()
        ca.lib.cg_last_stage_times(buf, 5)
        stage[k] = list(buf)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ca.lib.cg_set_profiling(0)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    n_chunks = int(first[-1])
    stages_ms = dict(zip(["scan", "compact", "walk", "assemble", "digest"],
                         stage[: max(args.steps, 1)].mean(axis=0).round(4)))

    # parity spot check on the last step (rank 0): descriptors cover every NAR exactly
    descs = d_out[: n_chunks * 48].cpu().numpy().view(ca.DESC_DTYPE)
    for i in range(n_nars):
        a, b = int(first[i]), int(first[i + 1])
        assert b > a and descs["offset"][a] == 0
        assert int(descs["offset"][b - 1] + descs["length"][b - 1]) == nar_bytes

    total_all = total_bytes * world
    value = total_all * args.steps / elapsed / GIB
    dig_ms = stages_ms["digest"]
    scan_ms = stages_ms["scan"]
    roofline = {
        "kernel": "k_sha256" if algo == 1 else "k_b3_groups+k_b3_top",
        "bound": "hbm",
        "achieved": round(total_bytes / (dig_ms * 1e-3) / 1e9, 2),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(total_bytes / (dig_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
        "traffic": None,
        "note": "digest stage: algorithmic bytes = every NAR byte once, / mean digest-stage duration over the "
                "timed steps; scan stage reported separately",
        "scan_kernel": {"kernel": "k_scan", "achieved": round(total_bytes / (scan_ms * 1e-3) / 1e9, 2),
                        "frac": round(total_bytes / (scan_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "traffic": None},
    }
    if algo == 1:
        roofline["latency_floor"] = sha_chain_floor(descs, n_nars, total_bytes, params, dig_ms)
    dig_kernels = ["k_sha256"] if algo == 1 else ["k_b3_groups", "k_b3_top"]
    traffic, src = pmc_traffic(args.config, dig_kernels)
    if traffic is not None:
        roofline["traffic"] = traffic
        roofline["scan_kernel"]["traffic"] = pmc_traffic(args.config, ["k_scan"])[0]
        roofline["traffic_source"] = src

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(host, offs, params, algo, args.cpu_sample_nars or n_nars)

    if rank == 0:
        line = {
            "metric": "device-resident GiB/s FastCDC+SHA-256 over synthetic NARs, 1/2/4/8 MI355X"
            if algo == 1 else "device-resident GiB/s FastCDC+BLAKE3 over synthetic NARs",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (xorshift64 NAR payloads)" if not args.zeros else "synthetic (all-zero NAR payloads)",
            "config": {"workload": desc, "nars_per_gpu": n_nars, "nar_bytes": nar_bytes,
                       "params": list(params), "parallelism": f"nar-shard x{world}"},
            "chunks": n_chunks,
            "stages_ms": stages_ms,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def sha_chain_floor(descs, n_nars, total_bytes, params, dig_ms):
    """The SHA-256 digest stage cannot end before the longest chunk's serial chain of
    64-round compressions has issued: blocks x 64 x (VALU per round x ~4.64 clocks,
    lone-wave issue cost measured by scripts/diag_sha_split.py: 41.8 quad, 46.5 pair)
    at 2.4 GHz.  The tier rule mirrors sha256_grid (quads when the expected chunk
    count leaves <= 256 x 64 chunks for one-lane workgroups)."""
    longest = int(descs["length"].max()) if len(descs) else 0
    blocks = (longest + 9 + 63) // 64
    expected = total_bytes // (params[0] + params[1]) + n_nars
    quad = expected <= 8 * 256 + 32 * 256 + 256 * 64
    cyc = 41.8 if quad else 46.5
    floor_ms = blocks * 64 * cyc / 2.4e9 * 1e3
    return {"longest_chunk_bytes": longest, "blocks": blocks, "tier": "quad" if quad else "pair",
            "cycles_per_round": cyc, "clock_GHz": 2.4, "floor_ms": round(floor_ms, 3),
            "frac": round(floor_ms / dig_ms, 4) if dig_ms else None}


def pmc_traffic(config, kernels):
    """HBM bytes per launch of `kernels` from the committed rocprofv3 --pmc summary for
    this config (profiles/*pmc_<config>.json, written by scripts/pmc_summary.py from
    scripts/gpu_pmc.sh passes): FETCH_SIZE x 2 (gfx950 correction, MI355X_MICROARCH.md
    §HBM) + WRITE_SIZE.  (None, None) when no summary has been committed."""
    files = sorted(ROOT.glob(f"profiles/*pmc_{config}.json"))
    if not files:
        return None, None
    rows = json.loads(files[-1].read_text())
    total, hit = 0.0, False
    for name, row in rows.items():
        base = name.split("::")[-1].split("<")[0]
        if base in kernels and "fetch_bytes_x2" in row:
            total += row["fetch_bytes_x2"] + row.get("write_bytes", 0.0)
            hit = True
    return (round(total), str(files[-1].relative_to(ROOT))) if hit else (None, None)


def cpu_baseline(host, offs, params, algo, sample_nars):
    """The oracle's restatement of chunk_data (one call per NAR: serial FastCDC scan,
    then per-chunk digests on a thread pool, as rayon does), timed on this host."""
    from oracle import oracle as O

    nt = min(os.cpu_count() or 1, 16)
    O.lib()
    nars = [host[int(offs[i]):int(offs[i + 1])] for i in range(min(sample_nars, len(offs) - 1))]
    O.chunk_descriptors(nars[0], *params, algo=algo, nthreads=nt)  # warm
    t0 = time.perf_counter()
    nbytes = 0
    for nar in nars:
        O.chunk_descriptors(nar, *params, algo=algo, nthreads=nt)
        nbytes += len(nar)
    dt = time.perf_counter() - t0
    return {"value": round(nbytes / dt / GIB, 4), "unit": "GiB/s", "cores": nt, "kind": "port",
            "sample": f"{len(nars)} NARs ({nbytes / GIB:.3f} GiB) of the same batch, one chunk_descriptors call "
                      f"per NAR, SHA-NI={'yes' if O.lib().or_sha256_uses_shani() else 'no'}",
            "seconds": round(dt, 3)}


if __name__ == "__main__":
    main()

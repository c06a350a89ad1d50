"""bench.py -- device-resident FastCDC + per-chunk digest throughput on MI355X.

Metric (BASELINE.json): "device-resident GiB/s FastCDC+SHA-256 over synthetic NARs,
1/2/4/8 MI355X".  A step is one pass of the hot path (candidate scan -> cut walk ->
descriptor assembly -> per-chunk digest) over one batch of synthetic NARs already
resident in HBM, through the C ABI entry cg_chunk_batch_device.  Default workload =
BASELINE config 2: 256 x 4 MiB NARs per GPU, 256K/1M/4M, SHA-256.

Multi-GPU: `--gpus N` with no torchrun environment starts N ranks itself (a child
`python -m torch.distributed.run`; this parent never touches a GPU); under the
driver's torchrun each process is one rank.  NARs are sharded one-file-per-GPU with
chunker_amd.dist.shard_nars over n_per_gpu x N NARs (weak scaling; config c5 = 16 x
1 GiB per GPU, i.e. BASELINE config 5's 128 x 1 GiB at N = 8); every step ends with
the descriptors gathered to rank 0 over RCCL, the path's only exchange.  value = all
ranks' bytes / max-over-ranks time.

Extra JSON keys: roofline (dominant kernel, HIP events around the digest on the stream
the kernels run on, in the timed steps), cpu_baseline (the oracle's restatement of
chunk_data, rank 0 at N = 1 only), stages_ms (every stage, from untimed steps after
the timed region: a timing event between two kernels delays the second by ~6 us;
digest_timed = the timed steps' digest), chunks, gear_table, and at N = 1 `concurrent`:
K independent batches in flight on K streams from K host threads (the reference's
callers are concurrent).
"""
from __future__ import annotations

import argparse
import json

import os
import re
import socket
import subprocess
import sys
import threading
import time
from collections import deque
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md
GIB = 1024 ** 3
PROFILE_STEPS = 3  # untimed steps after the timed region with every stage boundary timed
PUBLISHED_CHUNK_DATA_ZEROS = 1.055  # GiB/s, chunk_data_eager_10mb_sha256 (benchmarks/latest.md:12)

CONFIGS = {
    # name: (nars per GPU, nar_bytes, (min, avg, max), algo, description)
    "c2": (256, 4 << 20, (256 << 10, 1 << 20, 4 << 20), 1,
           "256x4MiB synthetic NARs per GPU, 256K/1M/4M, SHA-256 (BASELINE config 2)"),
    "c3": (256, 4 << 20, (256 << 10, 1 << 20, 4 << 20), 0,
           "256x4MiB synthetic NARs per GPU, 256K/1M/4M, BLAKE3 (BASELINE config 3)"),
    "c4": (16, 1 << 30, (64 << 10, 256 << 10, 1 << 20), 1,
           "16x1GiB synthetic NARs per GPU, 64K/256K/1M, SHA-256 (BASELINE config 4)"),
    "c5": (16, 1 << 30, (256 << 10, 1 << 20, 4 << 20), 1,
           "16x1GiB synthetic NARs per GPU (128x1GiB at 8 GPUs), 256K/1M/4M, SHA-256, RCCL gather "
           "(BASELINE config 5)"),
}


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--zeros", action="store_true", help="all-zero payloads (the reference's bench data)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-nars", type=int, default=0, help="0 = whole batch for c2/c3, 1 NAR for c4/c5")
    ap.add_argument("--no-concurrent", action="store_true", help="skip the K-batches-in-flight measurement")
    ap.add_argument("--concurrent", default="8,16,32", help="K values of the in-flight measurement ('' = skip it)")
    ap.add_argument("--concurrent-only", action="store_true", help="only the in-flight measurement (profiling)")
    ap.add_argument("--concurrent-reps", type=int, default=3, help="batches per thread in the in-flight measurement")
    ap.add_argument("--e2e", default="1,8,16", help="K values of the host-to-host in-flight measurement ('' = skip)")
    ap.add_argument("--drop-in", default="1,8,32",
                    help="K values of the drop-in leg: BASELINE config 1 (10 MiB, 256K/1M/4M) through the host "
                         "entry cg_chunk_descriptors from K threads, SHA-256 and BLAKE3, against the CPU port on the "
                         "same threads ('' = skip)")
    ap.add_argument("--drop-in-only", action="store_true", help="only the drop-in leg (profiling)")
    ap.add_argument("--drop-in-sizes", default="10,64,256,1024",
                    help="MiB per call of the drop-in leg's one-caller size sweep ('' = skip)")
    ap.add_argument("--hw-queues", type=int, default=0, choices=range(0, 33), metavar="0..32",
                    help="GPU_MAX_HW_QUEUES for this process (0: leave the environment's, HIP's default 4: the "
                         "digest pipeline needs no more)")
    ap.add_argument("--group", type=int, default=-1, choices=range(-1, 65), metavar="-1..64",
                    help="batches per merged SHA-256 digest launch of the digest pipeline (cg_pipeline_*; -1: "
                         "chunker_amd.default_group; 0: the round-5 per-batch-stream path, "
                         "cg_chunk_batch_device_async_after)")
    ap.add_argument("--lanes", type=int, default=0, choices=range(0, 9), metavar="0..8",
                    help="merged digests in flight (cg_pipeline_create lanes; 0: chunking.default_lanes)")
    ap.add_argument("--sha-occ", default="",
                    help="SHA-256 workgroups per CU 'LATENCY,FILL' for launches with more workgroups than CUs "
                         "(cg_test_sha_occupancy; '' = the library's)")
    ap.add_argument("--no-stage-profile", action="store_true",
                    help="skip the per-stage single steps (so a kernel trace holds only the pipeline's launches)")
    ap.add_argument("--no-clock", action="store_true", help="skip the digest clock measurement (scripts/sha_clock.py)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="queue each batch after everything on the stream (cg_chunk_batch_device_async): its "
                         "boundary stages wait for the previous batch's digest (A/B of the overlap)")
    ap.add_argument("--depth", type=int, default=0, choices=range(0, 257), metavar="0..256",
                    help="batches in flight from the one caller (each its own input batch, output array and "
                         "workspace); 1 = each batch waited for before the next is queued; 0 = auto: (lanes + 1) x "
                         "group for the digest pipeline, default_depth for --group 0")
    ap.add_argument("--split-mode", type=int, default=2, choices=(1, 2),
                    help="overlapped batches: 1 = boundary stages on the library stream, digests in stream order; "
                         "2 = the whole batch on the library stream (digests of consecutive batches overlap too)")
    ap.add_argument("--sha-tiers", default="",
                    help="SHA-256 latency tiers 'QUAD_PM,PAIR_PM[,FILL_QUAD_PM,FILL_PAIR_PM]' (cg_test_sha_tiers, "
                         "cg_test_sha_tiers_fill; quad 0 = off; '' = the library's)")
    ap.add_argument("--profile-after", action="store_true",
                    help="time the stages (PROFILE_STEPS single steps) after the timed region instead of before it")
    ap.add_argument("--no-coalesce", action="store_true",
                    help="concurrent callers digest their batches alone (cg_test_coalesce(0)); A/B of the coalescer")
    ap.add_argument("--dist-force", action="store_true",
                    help="run the N > 1 code (process group, gather to rank 0, rank-0 check) even at one rank: "
                         "rehearses the RCCL path on a one-GPU box")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1: nccl = RCCL over xGMI, one GPU per rank (the product); gloo = host-copy "
                         "gather, ranks may share a GPU (rehearses the N > 1 path on a one-GPU box)")
    return ap.parse_args()


def default_depth(algo: int, batch_bytes: int) -> int:
    """Batches the one caller keeps in flight: chunker_amd.default_depth (DESIGN.md §7
    "Batches in flight").  SHA-256 under 4 GiB a batch: 20 -- such a batch's digest is
    latency-bound, every chunk one serial chain (config 2's longest: 52,345 blocks = 53
    ms), and with the latency tiers its ~1,000 chains take ~18 workgroups, so the batches
    queued behind it fill the chip: config 2 at 22 hardware queues 318.8-320.4 GiB/s with
    twenty in flight at a per-batch p50 of 61.4-61.5 ms (55 alone; 18.1 one at a time;
    309.7 over 200 steps) (profiles/r05_v57_v58_q22.txt, r05_v24_v26_tiers_ab.txt).  From
    4 GiB: 4 (configs 4 / 5: the digest fills the chip by itself and the overlap hides the
    scan).  BLAKE3: 2 (its batches stay in stream order; the second one queued covers the
    host's per-call work).  Held to GPU_MAX_HW_QUEUES - 2: each batch in flight runs on a
    HIP stream of its own, and batches sharing a hardware queue run one after another
    (profiles/r05_v51_v52_queues_depth.txt)."""
    from chunker_amd.chunking import default_depth as rule

    return rule(algo, batch_bytes)


def timed_group(lib_default: int, steps: int) -> int:
    """The divisor of `steps` nearest the library's default group (ties: the larger), so the
    timed steps are whole merged groups: 20 steps -> 20 (library default 24)."""
    divs = [g for g in range(1, min(steps, 64) + 1) if steps % g == 0] or [1]
    return min(divs, key=lambda g: (abs(g - lib_default), -g))


def peek_hook(hook, *which) -> int:
    """The current setting of a set-and-return-previous test hook, left unchanged."""
    old = int(hook(*which, 1))
    hook(*which, old)
    return old


def launch_ranks(n: int) -> int:
    """Start n ranks as one child torchrun process (127.0.0.1 rendezvous) and return
    its exit code.  Nothing here initialises HIP: the GPUs belong to the children."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), *sys.argv[1:]]
    return subprocess.call(cmd)


def main():
    args = parse_args()
    if "WORLD_SIZE" not in os.environ and (args.gpus > 1 or args.dist_force):
        sys.exit(launch_ranks(args.gpus))
    # The installed GEAR table is the labelled placeholder (tables/README.md) and the
    # engine refuses to chunk with it unless opted in; the JSON says which table ran.
    os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")
    # The digest pipeline holds 1 + lanes streams however many batches are in flight, so
    # HIP's default 4 hardware queues suffice (round 5's per-batch streams needed 22).
    # --hw-queues N sets GPU_MAX_HW_QUEUES before anything initialises HIP (A/B only).
    if args.hw_queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    nccl = args.dist_backend == "nccl"
    multi = world > 1 or args.dist_force
    if multi and nccl:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    elif multi:
        # gloo rehearsal: ranks beyond the box's GPU count share them (RCCL would refuse
        # two ranks on one GPU); the gather runs on host copies of the descriptors.
        torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)

    import chunker_amd as ca
    from chunker_amd.dist import check_gathered_batch, gather_batch, gather_batch_async, gather_shape, shard_nars
    from chunker_amd.nar import synth_nars_device

    n_per, nar_bytes, params, algo, desc = CONFIGS[args.config]
    if args.no_coalesce:
        ca.lib.cg_test_coalesce(0)
    ca.lib.cg_test_split_mode(args.split_mode)
    if args.sha_occ:
        lat_occ, fill_occ = (int(v) for v in args.sha_occ.split(","))
        ca.lib.cg_test_sha_occupancy(0, lat_occ)
        ca.lib.cg_test_sha_occupancy(1, fill_occ)
    if args.sha_tiers:
        t = [int(v) for v in args.sha_tiers.split(",")]
        ca.lib.cg_test_sha_tiers(t[0], t[1])
        if len(t) == 4:
            ca.lib.cg_test_sha_tiers_fill(t[2], t[3])
    if args.concurrent_only:
        print(json.dumps({"concurrent": concurrent_rates(ca, torch, args, n_per, nar_bytes, params, algo)}))
        return
    if args.drop_in_only:
        print(json.dumps({"drop_in": drop_in_rates(ca, args)}))
        return
    mine = shard_nars(n_per * world, world, rank)
    sizes = np.full(len(mine), nar_bytes, np.uint64)
    batch_bytes = int(sizes.sum())
    # The product pipeline (chunker_amd.BatchPipeline): the digest pipeline with `group`
    # batches per merged SHA-256 launch and `lanes` merged launches in flight, depth (lanes +
    # 1) x group batches queued from this one caller (every lane busy while the next group
    # forms); --group 0 = the round-5 per-batch-stream path.
    # (the timed region must span whole groups: steps complete in bursts as each group's
    # members finish, so the default group is the divisor of --steps nearest the library's
    # default -- 20 for the driver's 20 steps)
    group = args.group if args.group >= 0 else timed_group(ca.chunking.default_group(algo, batch_bytes), args.steps)
    lanes = args.lanes or ca.chunking.default_lanes(algo, batch_bytes)
    depth = args.depth or (ca.chunking.pipeline_depth(algo, group, lanes) if group else default_depth(algo, batch_bytes))
    # Distinct inputs: every in-flight slot owns its own batch of NARs (global NAR indices
    # slot * n_per * world + this rank's shard, the reference's per-NAR seeds,
    # crates/node/src/lib.rs:191-203) and output array.  Slot k % depth is reused by step k
    # only after step k - depth was returned (BatchPipeline keeps at most `depth` queued).
    t_syn = time.perf_counter()
    d_ins, offs = [], None
    for slot in range(depth):
        d, offs = synth_nars_device(sizes, zeros=args.zeros, first_index=slot * n_per * world + mine.start)
        d_ins.append(d)
    torch.cuda.synchronize()
    synth_s = time.perf_counter() - t_syn
    total_bytes = int(offs[-1])
    cap = ca.chunking.batch_capacity(offs, params[0])
    # RCCL gather: fixed per-rank sizes agreed once here, so a step's gather needs no count
    # exchange and no host sync (chunker_amd.dist.gather_batch_async)
    gcap, gnars = gather_shape(cap, len(mine)) if multi and nccl else (cap, len(mine))
    d_outs = [torch.empty(gcap * 48, dtype=torch.uint8, device="cuda") for _ in range(depth)]
    # The gather of step k is queued on torch's current stream (RCCL's stream waits for that
    # one) once step k is back on the host; an event after it is the inputs-ready event of
    # step k + depth, the next writer of the same output array, so the pipeline's boundary
    # stream waits for the gather and nothing else.
    bstream = torch.cuda.Stream()
    sptr = bstream.cuda_stream
    gathered_ev = [None] * depth
    gathered = [None]
    synth_ev = torch.cuda.Event()
    synth_ev.record()

    def ready_event(k):  # the inputs-ready event of step k (its output array free again)
        ev = gathered_ev[k % depth]
        if args.no_overlap:
            if ev is not None:
                bstream.wait_event(ev)
            return 0
        return (ev or synth_ev).cuda_event

    slot_first = {}

    def after_wait(k, first):
        slot_first[k % depth] = first
        if multi and nccl:  # descriptors + NAR index to rank 0 over RCCL (the path's only exchange)
            gathered[0] = gather_batch_async(d_outs[k % depth], first, gcap, gnars)
            ev = torch.cuda.Event()
            ev.record()
            gathered_ev[k % depth] = ev
        elif multi:  # gloo rehearsal: host copies
            gathered[0] = gather_batch(d_outs[k % depth][: int(first[-1]) * 48].cpu(), first)
        return first

    pipe = ca.BatchPipeline(depth, *params, hash=algo, stream=sptr, group=group, lanes=lanes)
    t_issue = {}
    last = {"k": None, "first": None}
    nxt = [0]  # next step index

    def submit_next(on_done=None):
        k = nxt[0]
        nxt[0] += 1
        ready = ready_event(k)
        t_issue[k] = time.perf_counter()
        got = pipe.submit(d_ins[k % depth].data_ptr(), offs, d_outs[k % depth].data_ptr(), gcap,
                          inputs_ready=ready, tag=k)
        for kk, first in got:
            last["k"], last["first"] = kk, after_wait(kk, first)
            if on_done:
                on_done(kk, time.perf_counter() - t_issue[kk])
        return len(got)

    def drain(on_done=None):
        for kk, first in pipe.drain():
            last["k"], last["first"] = kk, after_wait(kk, first)
            if on_done:
                on_done(kk, time.perf_counter() - t_issue[kk])

    # warm-up: max(W, depth) + 1 steps rounded up to whole groups, so every workspace the
    # pool hands out and every lane buffer is sized before the timed region
    n_warm = max(args.warmup, depth) + 1
    if group:
        n_warm = -(-n_warm // group) * group
    for _ in range(n_warm):
        submit_next()
    drain()

    # Stage profile (every stage boundary a HIP event, cg_set_profiling(1)) on PROFILE_STEPS
    # single batches through the per-batch path (its digest is one batch's launch), then the
    # scan stage right after a 2 GiB write (the 256 MB MALL holds none of the batch): the
    # cold-HBM rate beside the warm one.  A timing event between two kernels holds the second
    # back by ~6 us, so the timed region records only the pipeline's events around each
    # merged digest (cg_set_profiling(2)).
    buf = (np.ctypeslib.ctypes.c_double * 5)()

    def single(k_slot):
        with ca.BatchPipeline(1, *params, hash=algo, stream=sptr, group=0) as one:
            one.submit(d_ins[k_slot].data_ptr(), offs, d_outs[k_slot].data_ptr(), gcap)
            one.drain()

    def profile_stages():
        ca.lib.cg_set_profiling(1)
        prof = np.zeros((PROFILE_STEPS, 5))
        for k in range(PROFILE_STEPS):
            single(k % depth)
            ca.lib.cg_last_stage_times(buf, 5)
            prof[k] = list(buf)
        cold = np.zeros(PROFILE_STEPS)
        scratch = torch.empty(2 * GIB, dtype=torch.uint8, device="cuda")
        for k in range(PROFILE_STEPS):
            scratch.fill_(k)
            torch.cuda.synchronize()
            single(k % depth)
            ca.lib.cg_last_stage_times(buf, 5)
            cold[k] = buf[0]
        del scratch
        ca.lib.cg_set_profiling(0)
        return prof, cold

    floor = None
    if args.no_stage_profile:
        prof, cold = np.full((1, 5), np.nan), np.full(1, np.nan)
    else:
        prof, cold = profile_stages()
        if algo == 1:  # the single batch's digest against its longest chunk's chain (its own launch's tiers)
            k_s = (PROFILE_STEPS - 1) % depth
            n_s = int(ca.chunking.batch_capacity(offs, params[0]))
            d_s = d_outs[k_s][: n_s * 48].cpu().numpy().view(ca.DESC_DTYPE)
            d_s = d_s[d_s["length"] > 0]
            clk = sha_clock(args) if world == 1 and not args.no_clock else None
            floor = sha_chain_floor(ca, d_s, float(np.mean(prof[:, 4])), clk)
    ca.lib.cg_set_profiling(2)
    st0 = pipe.stats()
    torch.cuda.synchronize()
    if multi:
        dist.barrier()
    # Fill (untimed): depth - 1 steps queued, the pipeline's groups forming and launching;
    # then settle (untimed): at least `depth` (and 4 x lanes groups) more steps submitted and completed one for one,
    # as in every step of a long run, ending at the completion of a whole group.  The timed
    # region then counts completions in steady state, from one group's
    # end to another's.
    t_fill = time.perf_counter()
    done0 = nxt[0]  # steps completed so far (the warm-up drained)
    while nxt[0] - done0 < depth - 1:
        submit_next()
    fill_ms = (time.perf_counter() - t_fill) * 1e3
    t_settle = time.perf_counter()
    settled = [0]

    def count(kk, waited):
        settled[0] += 1

    # (settle >= 4 x lanes groups: with four lanes the lanes' phases take a few cycles to even
    # out, profiles/r06_v37_summary.txt)
    n_settle = max(depth, 4 * lanes * group) if group else depth
    while settled[0] < n_settle or (group and (last["k"] + 1) % group):
        submit_next(count)
    settle_ms = (time.perf_counter() - t_settle) * 1e3
    # t0: the caller's own streams are idle (torch's current stream and the gather's), the
    # ranks aligned; the pipeline holds depth - 1 batches in flight, as it does at every
    # step of a long run
    torch.cuda.current_stream().synchronize()
    bstream.synchronize()
    if multi:
        dist.barrier()
    t0 = time.perf_counter()
    latency = []
    done = [0]

    def record(kk, waited):
        done[0] += 1
        latency.append(waited)

    while done[0] < args.steps:  # EXACTLY `steps` batches completed inside the timed region
        submit_next(record)
    t1 = time.perf_counter()
    elapsed = t1 - t0
    done_timed = done[0]
    # A longer steady window right after (untimed for `value`): 3 x lanes whole groups, so
    # the lanes' phase (a single group-to-group window of `steps` steps reads +-10 %) averages
    # out; reported beside `value`.
    n_long = 3 * lanes * group if group else 0
    long_rate = None
    if n_long:
        done_l = [0]

        def count_l(kk, waited):
            done_l[0] += 1

        tl = time.perf_counter()
        while done_l[0] < n_long:
            submit_next(count_l)
        long_rate = done_l[0] * total_bytes * world / (time.perf_counter() - tl) / GIB
    if multi:
        dist.barrier()
    # drain (untimed): the depth - 1 batches still in flight
    t_dr = time.perf_counter()
    drain()
    torch.cuda.synchronize()  # every stream: the batches' and the last gather
    drain_ms = (time.perf_counter() - t_dr) * 1e3
    st1 = pipe.stats()
    pipe.close()
    ca.lib.cg_set_profiling(0)
    if multi:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if nccl else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    first = last["first"]
    k_last = last["k"] % depth
    n_chunks = int(first[-1])
    stages_ms = dict(zip(["scan", "compact", "walk", "assemble", "digest"], np.nanmean(prof, axis=0).round(4)))
    # merged digest launches timed by the pipeline's events (cg_set_profiling(2)): the timed
    # region's groups and the drain's
    g_n = st1.get("timed_groups", 0) - st0.get("timed_groups", 0)
    g_ms = st1.get("digest_ms_sum", 0.0) - st0.get("digest_ms_sum", 0.0)
    g_bytes = st1.get("digest_bytes_sum", 0.0) - st0.get("digest_bytes_sum", 0.0)
    launch_ms = g_ms / g_n if g_n else float("nan")
    launch_bytes = g_bytes / g_n if g_n else float("nan")
    stages_ms["digest_launch"] = round(launch_ms, 4)

    # parity spot check on the last step: descriptors cover every NAR exactly -- this
    # rank's own batch, and at N > 1 the whole batch as gathered on rank 0 (global NAR
    # order, every NAR of every rank tiled contiguously)
    descs = d_outs[k_last][: n_chunks * 48].cpu().numpy().view(ca.DESC_DTYPE)
    check_gathered_batch(descs, first, sizes)
    gather_check = None
    if multi and rank == 0:
        g_desc, g_first = gathered[0].assemble() if nccl else gathered[0]
        g_np = g_desc.cpu().numpy().view(ca.DESC_DTYPE)
        check_gathered_batch(g_np, g_first, np.full(n_per * world, nar_bytes, np.uint64))
        gather_check = {"nars": n_per * world, "chunks": int(g_first[-1]), "backend": args.dist_backend,
                        "rank0_prefix_equal": bool(np.array_equal(g_np[:n_chunks].view(np.uint8),
                                                                  descs.view(np.uint8)))}
        assert gather_check["rank0_prefix_equal"], "rank 0's own descriptors differ inside the gathered batch"

    total_all = total_bytes * world
    value = total_all * done_timed / elapsed / GIB
    scan_ms = stages_ms["scan"]
    if group and algo == 1 and g_n:
        # dominant kernel = the merged digest: algorithmic bytes per launch = every NAR byte of
        # its `group` batches once; duration = the pipeline's HIP events around k_sha256 on
        # the lane stream it ran on
        ach = launch_bytes / (launch_ms * 1e-3) / 1e9
        kname, knote = "k_sha256", (f"merged digest launch of the digest pipeline ({group} batches per launch, {lanes} "
                                    "lanes): algorithmic bytes = every NAR byte of the launch's batches once, / the "
                                    "mean launch duration (HIP events on the lane stream around k_sha256, the timed "
                                    f"region's and the drain's {g_n} launches)")
    else:
        dig_ms = stages_ms["digest"]
        ach = total_bytes / (dig_ms * 1e-3) / 1e9
        kname = "k_sha256" if algo == 1 else "k_b3_leaves+k_b3_fold+k_b3_top"
        knote = (f"digest stage of one batch (HIP events around the digest, {PROFILE_STEPS} untimed single steps): "
                 "algorithmic bytes = every NAR byte once")
    roofline = {
        "kernel": kname,
        "bound": "hbm",
        "achieved": round(ach, 2),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(ach / HBM_PEAK_GBS, 5),
        "traffic": None,
        "note": knote,
        "launch": {"bytes": round(launch_bytes) if g_n else None, "ms": round(launch_ms, 3) if g_n else None,
                   "launches_timed": g_n},
        "scan_kernel": {"kernel": scan_kernel_name(ca, params[1], total_bytes),
                        "achieved": round(total_bytes / (scan_ms * 1e-3) / 1e9, 2),
                        "frac": round(total_bytes / (scan_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "traffic": None,
                        "cold_hbm": {"ms": round(float(np.median(cold)), 4),
                                     "achieved": round(total_bytes / (float(np.median(cold)) * 1e-3) / 1e9, 2),
                                     "frac": round(total_bytes / (float(np.median(cold)) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                     "note": "scan stage after a 2 GiB write evicted the batch from the MALL "
                                             f"(median of {PROFILE_STEPS}); the warm figure above follows the "
                                             "previous step's digest, which just read the batch"}},
    }
    roofline["aggregate"] = {"achieved": round(total_bytes * done_timed / elapsed / 1e9, 2),
                             "frac": round(total_bytes * done_timed / elapsed / 1e9 / HBM_PEAK_GBS, 5),
                             "batches_in_flight": depth,
                             "note": "this rank's algorithmic bytes of all timed steps / the timed wall time"}
    if floor is not None:
        roofline["latency_floor"] = floor
    # (the batch path assembles the leaf map, so its leaf kernel is k_b3_leaves; k_b3_groups
    # is the three-kernel form's, counted when a summary holds it instead)
    dig_kernels = ["k_sha256"] if algo == 1 else ["k_b3_leaves", "k_b3_groups", "k_b3_fold", "k_b3_top"]
    traffic, src = pmc_traffic(args.config, dig_kernels)
    if traffic is not None:
        roofline["traffic"] = traffic
        roofline["scan_kernel"]["traffic"] = pmc_traffic(args.config, [roofline["scan_kernel"]["kernel"]])[0]
        roofline["traffic_source"] = src

    # slot 0's batch (global NARs 0 .. n_per - 1 at rank 0): the e2e leg's host batch
    n0 = int(slot_first[0][-1])
    descs0 = d_outs[0][: n0 * 48].cpu().numpy().view(ca.DESC_DTYPE)
    cpu = None
    conc = None
    drop = None
    del d_ins, d_outs
    torch.cuda.empty_cache()
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, n_per, nar_bytes, params, algo)
    if world == 1 and args.drop_in:
        drop = drop_in_rates(ca, args)
    if world == 1 and not args.no_concurrent:
        conc = concurrent_rates(ca, torch, args, n_per, nar_bytes, params, algo)
        if args.e2e:
            conc["e2e"] = e2e_rates(ca, torch, args, n_per, nar_bytes, params, algo, descs0)

    if rank == 0:
        gear = "placeholder" if ca.lib.cg_gear_is_placeholder() else (
            "fastcdc-4.0.1 (selftest passed)" if ca.tables_verified() else "installed, unverified")
        lat = np.array(latency) * 1e3
        line = {
            "metric": "device-resident GiB/s FastCDC+SHA-256 over synthetic NARs, 1/2/4/8 MI355X"
            if algo == 1 else "device-resident GiB/s FastCDC+BLAKE3 over synthetic NARs",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / done_timed * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": ("synthetic (xorshift64 NAR payloads)" if not args.zeros else "synthetic (all-zero NAR payloads)"),
            "inputs": f"distinct: {depth} input batches resident in HBM, one per batch in flight",
            "timed": (f"steady: before t0 the pipeline was filled ({depth - 1} batches in flight) and settled "
                      f"({settled[0]} steps, each one submitted and one completed, ending at a group's end); exactly "
                      f"{done_timed} batches completed between t0 and t1 ({done_timed // max(group, 1)} whole groups of "
                      f"{group}; t0 after a barrier with the caller's streams idle, t1 at the last completion returned "
                      "to the host); fill, settle and drain untimed, reported"),
            "pipeline": {"kind": "digest pipeline (cg_pipeline_*)" if group else
                         "per-batch streams (cg_chunk_batch_device_async_after)",
                         "group": group, "lanes": lanes if group else None, "depth": depth,
                         "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "4 (HIP default)"),
                         "sha_wgs_per_cu": [peek_hook(ca.lib.cg_test_sha_occupancy, k) for k in (0, 1)],
                         "fill_ms": round(fill_ms, 2), "settle_steps": settled[0], "settle_ms": round(settle_ms, 2),
                         "settle_GiBps": round(settled[0] * total_bytes * world / (settle_ms * 1e-3) / GIB, 3),
                         "drain_ms": round(drain_ms, 2),
                         "steady_window": {"steps": n_long, "GiBps": round(long_rate, 3) if long_rate else None,
                                           "note": "the steps right after the timed ones, group end to group end "
                                                   "(this rank; not part of `value`)"},
                         "synth_s": round(synth_s, 1)},
            "batch_latency_ms": {"p50": round(float(np.percentile(lat, 50)), 3),
                                 "p99": round(float(np.percentile(lat, 99)), 3),
                                 "note": "submit -> results on the host, per batch, timed region"},
            "config": {"workload": desc, "nars_per_gpu": len(mine), "nar_bytes": nar_bytes,
                       "params": list(params), "parallelism": f"nar-shard x{world}",
                       **({"dist_backend": args.dist_backend} if multi else {})},
            "gear_table": gear,
            "chunks": n_chunks,
            "stages_ms": stages_ms,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "concurrent": conc,
            "drop_in": drop,
        }
        if gather_check is not None:
            line["gather_check"] = gather_check
            if not nccl:
                line["note"] = (f"gloo rehearsal of the N > 1 path: {world} ranks on "
                                f"{min(world, torch.cuda.device_count())} GPU(s), host-copy gather; "
                                "not a scaling measurement")
        print(json.dumps(line))
    if multi:
        dist.destroy_process_group()


def concurrent_rates(ca, torch, args, n_per, nar_bytes, params, algo):
    """K independent config batches in flight: K host threads, each with its own input
    batch, output array and HIP stream, calling cg_chunk_batch_device `reps` times.
    Aggregate GiB/s = K x reps x batch bytes / wall time (after one untimed round that
    sizes every workspace), and what a caller waits per call (p50 / p99 ms).  For SHA-256
    both coalescer settings run, one after the other in this process: `merged` (digests
    of more concurrent callers than per-batch launches run side by side share one launch, the
    product) and `per_batch`
    (cg_test_coalesce(0)), so the merged rate and its latency cost sit side by side; the
    coalescer's own counters (groups, members, leader wait, windows run out) are reported
    for the merged runs.  The headline `value` stays the single-batch rate."""
    import ctypes

    from chunker_amd.nar import synth_nars_device

    ks = sorted({int(k) for k in args.concurrent.split(",") if k})
    if not ks:  # --concurrent '': only the host-to-host leg (e2e)
        return {"unit": "GiB/s"}
    kmax = max(ks)
    sizes = np.full(n_per, nar_bytes, np.uint64)
    jobs = []
    for k in range(kmax):
        d, offs = synth_nars_device(sizes, zeros=args.zeros, first_index=(k + 1) * 1000 * n_per)
        cap = ca.chunking.batch_capacity(offs, params[0])
        out = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
        jobs.append((d, offs, out, cap, torch.cuda.Stream()))
    torch.cuda.synchronize()
    batch_bytes = int(jobs[0][1][-1])
    coal = bool(ca.lib.cg_test_coalesce(1))
    ca.lib.cg_test_coalesce(int(coal))
    res = {"unit": "GiB/s", "latency_unit": "ms per call", "batch": f"{n_per}x{nar_bytes >> 20}MiB",
           "reps": max(1, args.concurrent_reps), "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default (4)"),
           "digests": "coalesced (one SHA-256 launch per group once more callers are in flight than the hardware "
                      "queues less 4)"
           if coal and algo == 1 else "one launch per batch"}
    modes = [("merged", 1), ("per_batch", 0)] if coal and algo == 1 else [("per_batch", int(coal))]
    stats = (ctypes.c_uint64 * 4)()

    def measure(K, reps):
        bar = threading.Barrier(K + 1)
        errs, lat = [], [[] for _ in range(K)]

        def work(k):
            d, offs, out, cap, s = jobs[k]
            bar.wait()
            try:
                for _ in range(reps):
                    t = time.perf_counter()
                    ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params, hash=algo,
                                          stream=s.cuda_stream)
                    lat[k].append(time.perf_counter() - t)
            except Exception as e:  # noqa: BLE001
                errs.append(repr(e))

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
        ms = np.array([v for row in lat for v in row]) * 1e3
        return dt, ms

    for K in ks:
        row = {}
        for name, on in modes:
            ca.lib.cg_test_coalesce(on)
            measure(K, 1)  # untimed: sizes every workspace
            time.sleep(0.1)  # (callers that returned within 50 ms count as expected back)
            ca.lib.cg_coalesce_stats(stats)
            s0 = [int(x) for x in stats]
            dt, ms = measure(K, res["reps"])
            ca.lib.cg_coalesce_stats(stats)
            s1 = [int(x) for x in stats]
            row[name] = {"GiBps": round(K * res["reps"] * batch_bytes / dt / GIB, 3),
                         "p50": round(float(np.percentile(ms, 50)), 2), "p99": round(float(np.percentile(ms, 99)), 2)}
            if on and algo == 1:
                g = s1[0] - s0[0]
                row[name]["coalescer"] = {"groups": g, "batches": s1[1] - s0[1],
                                          "leader_wait_ms_mean": round((s1[2] - s0[2]) / 1e3 / g, 3) if g else 0.0,
                                          "windows_run_out": s1[3] - s0[3]}
        ca.lib.cg_test_coalesce(int(coal))
        res[f"K{K}"] = row[modes[0][0]]["GiBps"]
        res[f"K{K}_detail"] = row
    return res


def e2e_rates(ca, torch, args, n_per, nar_bytes, params, algo, want):
    """NAR bytes start and end in host memory (north_star: a file or socket): K host
    threads, each with its own pinned host batch and host descriptor array, call the
    host entry cg_chunk_batch `reps` times -- H2D copy, chunk + digest, descriptors D2H
    -- so one batch's copies overlap the other batches' kernels.  Aggregate GiB/s =
    K x reps x batch bytes / wall time, after one untimed round; every call's
    descriptors must equal the device-resident run's (`want`, same NARs)."""
    import ctypes

    from chunker_amd.nar import synth_nars

    ks = sorted({int(k) for k in args.e2e.split(",") if k})
    host0, offs = synth_nars(np.full(n_per, nar_bytes, np.uint64), zeros=args.zeros, first_index=0)
    nbytes = int(offs[-1])
    cap = ca.chunking.batch_capacity(offs, params[0])
    bufs = []
    for _ in range(max(ks)):
        t = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        t.numpy()[:] = host0
        bufs.append((t, np.zeros(cap, ca.DESC_DTYPE), np.zeros(n_per + 1, np.uint64)))
    del host0
    res = {"unit": "GiB/s", "batch": f"{n_per}x{nar_bytes >> 20}MiB", "reps": 4, "host_buffers": "pinned",
           "entry": "cg_chunk_batch (H2D + chunk + digest + descriptors D2H)"}
    # the host link alone: one pinned batch copied to HBM (the ceiling of every e2e rate)
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    dev.copy_(bufs[0][0], non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        dev.copy_(bufs[0][0], non_blocking=True)
    torch.cuda.synchronize()
    res["h2d_only"] = round(3 * nbytes / (time.perf_counter() - t0) / GIB, 3)
    del dev
    for K in ks:
        for timed in (False, True):
            reps = res["reps"] if timed else 1
            bar = threading.Barrier(K + 1)
            errs = []

            def work(k):
                t, out, first = bufs[k]
                bar.wait()
                for _ in range(reps):
                    st = ca.lib.cg_chunk_batch(ctypes.c_void_p(t.data_ptr()), offs.ctypes.data, n_per, *params,
                                               algo, out.ctypes.data, cap, first.ctypes.data)
                    if st:
                        errs.append(f"status {st}: {ca._lib.last_error()}")
                        return

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
        for k in range(K):
            _, out, first = bufs[k]
            n = int(first[-1])
            assert n == len(want) and np.array_equal(out[:n].view(np.uint8), want.view(np.uint8)), \
                f"e2e batch {k}: descriptors differ from the device-resident run"
        res[f"K{K}"] = round(K * reps * nbytes / dt / GIB, 3)
    if algo == 1:
        res["one_caller_overlapped"] = e2e_one_caller(ca, torch, bufs, offs, nbytes, cap, params, algo, want, args)
    return res


def e2e_one_caller(ca, torch, bufs, offs, nbytes, cap, params, algo, want, args):
    """Host to host from ONE caller thread through the product pipeline
    (chunker_amd.BatchPipeline, the digest pipeline at its default group / lanes): batch k's
    pinned H2D copy runs on a copy stream and its event is the batch's inputs-ready event,
    so the copies overlap the batches before them; the descriptors come back D2H after each
    batch is returned.  `depth` device input and output buffers are used in turn.  GiB/s =
    reps x batch bytes / wall time, fill and drain included, reps = 3 x depth."""
    host = bufs[0][0]
    group = args.group if args.group >= 0 else ca.chunking.default_group(algo, nbytes)
    lanes = args.lanes or ca.chunking.default_lanes(algo, nbytes)
    depth = args.depth or (ca.chunking.pipeline_depth(algo, group, lanes) if group else default_depth(algo, nbytes))
    reps = 3 * depth
    dins = [torch.empty(nbytes + 256, dtype=torch.uint8, device="cuda") for _ in range(depth)]
    douts = [torch.empty(cap * 48, dtype=torch.uint8, device="cuda") for _ in range(depth)]
    out = np.zeros(cap * 48, np.uint8)
    copy = torch.cuda.Stream()
    n = 0
    for timed in (False, True):
        count = reps if timed else depth
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with ca.BatchPipeline(depth, *params, hash=algo, group=group, lanes=lanes) as pipe:
            def take(done):
                nonlocal n
                for k, first in done:
                    n = int(first[-1])
                    out[: n * 48] = douts[k % depth][: n * 48].cpu().numpy()

            for k in range(count):
                j = k % depth
                with torch.cuda.stream(copy):
                    dins[j][:nbytes].copy_(host, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record()
                take(pipe.submit(dins[j].data_ptr(), offs, douts[j].data_ptr(), cap, inputs_ready=ev.cuda_event,
                                 tag=k))
            take(pipe.drain())
        dt = time.perf_counter() - t0
    assert n == len(want) and np.array_equal(out[: n * 48], want.view(np.uint8)), \
        "e2e one caller: descriptors differ from the device-resident run"
    return {"GiBps": round(reps * nbytes / dt / GIB, 3), "reps": reps, "depth": depth, "group": group,
            "shape": f"one thread, up to {depth} batches in flight: pinned H2D on a copy stream -> inputs-ready event "
                     "-> digest pipeline -> wait -> descriptors D2H (fill and drain inside the timed region)"}


def drop_in_rates(ca, args):
    """The reference's own call shape: one chunk_data call per NAR --
    Node::put per HTTP PUT (crates/node/src/lib.rs:114-116, one thread per connection,
    crates/proto/nix/src/lib.rs:153-162), the NIF per binary (src/nif.rs:188-196), and the
    published bench, 10 MiB per call (benches/throughput.rs:39-43) -- through the drop-in
    host entry cg_chunk_descriptors (pageable host bytes in, descriptors out), from K
    threads at once, each calling `reps` times on its own 10 MiB xorshift64 buffer (BASELINE
    config 1, 256K/1M/4M).  Per algorithm and K: aggregate GiB/s (K x reps x 10 MiB / wall
    time), per-call latency p50 / p99 (ms), and the CPU port (the oracle's
    chunk_descriptors: serial FastCDC + per-chunk digests on max(1, cores / K) threads, as
    K callers share rayon's pool) on the same K threads over the same buffers.  Every GPU
    call's descriptors are checked against the CPU port's."""
    import ctypes

    from chunker_amd.nar import synth_nars
    from oracle import oracle as O

    ks = sorted({int(k) for k in args.drop_in.split(",") if k})
    nt, _, _ = host_cpus()
    ten = 10 << 20
    P = (256 << 10, 1 << 20, 4 << 20)
    kmax = max(ks)
    bufs = [synth_nars([ten], first_index=7 + k)[0] for k in range(kmax)]
    cap = int(ca.lib.cg_capacity(ten, P[0]))
    outs = [np.zeros(cap, ca.DESC_DTYPE) for _ in range(kmax)]
    res = {"unit": "GiB/s", "call": "cg_chunk_descriptors, 10 MiB xorshift64 per call, 256K/1M/4M (BASELINE config 1)",
           "latency_unit": "ms per call", "cpu_threads_per_call": f"max(1, {nt} // K)",
           "digests": "one launch per call (the host entry never merges digests)"}
    for algo, name in ((1, "sha256"), (0, "blake3")):
        want = [O.chunk_descriptors(b, *P, algo=algo, nthreads=nt) for b in bufs]
        leg = {}
        for K in ks:
            reps = max(3, min(12, 96 // K))

            def run(fn):
                bar = threading.Barrier(K + 1)
                lat, errs = [[] for _ in range(K)], []

                def work(k):
                    bar.wait()
                    try:
                        for _ in range(reps):
                            t = time.perf_counter()
                            fn(k)
                            lat[k].append(time.perf_counter() - t)
                    except Exception as e:  # noqa: BLE001
                        errs.append(repr(e))

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
                ms = np.array([v for row in lat for v in row]) * 1e3
                return {"GiBps": round(K * reps * ten / dt / GIB, 3), "p50": round(float(np.percentile(ms, 50)), 3),
                        "p99": round(float(np.percentile(ms, 99)), 3)}

            n_out = [ctypes.c_size_t(0) for _ in range(K)]

            def gpu(k):
                st = ca.lib.cg_chunk_descriptors(bufs[k].ctypes.data, ten, *P, algo, outs[k].ctypes.data, cap,
                                                 ctypes.byref(n_out[k]))
                if st:
                    raise RuntimeError(f"status {st}: {ca._lib.last_error()}")

            cpu_nt = max(1, nt // K)
            run(gpu)  # untimed round: every workspace sized
            g = run(gpu)
            for k in range(K):
                n = n_out[k].value
                assert n == len(want[k]) and np.array_equal(outs[k][:n].view(np.uint8), want[k].view(np.uint8)), \
                    f"drop-in {name} K={K} caller {k}: descriptors differ from the CPU port"
            c = run(lambda k: O.chunk_descriptors(bufs[k], *P, algo=algo, nthreads=cpu_nt))
            leg[f"K{K}"] = {"gpu": g, "cpu_port": c, "reps": reps}
        res[name] = leg
    # one caller, larger inputs: where a single call starts to pay on the GPU (the SHA-256
    # chain of the longest chunk is a fixed ~50-70 ms; the CPU port's serial FastCDC ~3 GiB/s)
    sweep = {}
    for mib in sorted({int(v) for v in args.drop_in_sizes.split(",") if v}):
        nb = mib << 20
        buf = synth_nars([nb], first_index=99)[0]
        cap_s = int(ca.lib.cg_capacity(nb, P[0]))
        out = np.zeros(cap_s, ca.DESC_DTYPE)
        n = ctypes.c_size_t(0)
        row = {}
        for algo, name in ((1, "sha256"), (0, "blake3")):
            want = O.chunk_descriptors(buf, *P, algo=algo, nthreads=nt)
            reps = 3 if mib >= 256 else 6
            gt, ct = [], []
            for r in range(reps + 1):
                t = time.perf_counter()
                st = ca.lib.cg_chunk_descriptors(buf.ctypes.data, nb, *P, algo, out.ctypes.data, cap_s, ctypes.byref(n))
                if r:
                    gt.append(time.perf_counter() - t)
                assert st == 0, ca._lib.last_error()
            assert n.value == len(want) and np.array_equal(out[: n.value].view(np.uint8), want.view(np.uint8)), \
                f"drop-in sweep {name} {mib} MiB: descriptors differ from the CPU port"
            for _ in range(reps):
                t = time.perf_counter()
                O.chunk_descriptors(buf, *P, algo=algo, nthreads=nt)
                ct.append(time.perf_counter() - t)
            g, c = float(np.median(gt)), float(np.median(ct))
            row[name] = {"gpu_GiBps": round(nb / g / GIB, 3), "gpu_ms": round(g * 1e3, 2),
                         "cpu_port_GiBps": round(nb / c / GIB, 3), "cpu_port_ms": round(c * 1e3, 2)}
        sweep[f"{mib}MiB"] = row
        del buf, out
    if sweep:
        res["one_caller_sizes"] = {"note": f"K = 1, median of 3-6 calls; CPU port on {nt} threads", **sweep}
    return res


def sha_clock(args):
    """The clock the digest's longest chain ran at (scripts/sha_clock.py: the diagnostics
    build's per-workgroup shader-clock and wall-clock record of the same batch, in a child
    process so this one keeps the product library only)."""
    try:
        r = subprocess.run([sys.executable, str(ROOT / "scripts" / "sha_clock.py"), "--config", args.config],
                           capture_output=True, text=True, timeout=300)
        return json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else None
    except (subprocess.TimeoutExpired, ValueError, IndexError):
        return None


def sha_chain_floor(ca, descs, dig_ms, clk=None):
    """The SHA-256 digest stage cannot end before the longest chunk's serial chain of
    64-round compressions has issued: blocks x 64 x (VALU per round x ~4.64 clocks,
    lone-wave issue cost of the round code as built, measured by scripts/diag_sha_lone.py:
    37.95 quad, 42.2 pair, 59.4 one-lane since the round asm is 8-byte aligned -- round 3
    v39; 41.8 / 46.5 before) at 2.4 GHz.  The tier is the one the library's last digest launch
    gave the longest chunk (cg_last_sha_tiers: the length order hands the longest
    chunks to the quad workgroups first, then pairs, then one-lane workgroups)."""
    tiers = (np.ctypeslib.ctypes.c_uint32 * 4)()
    ca.lib.cg_last_sha_tiers(tiers)
    nquad, npair, nlane, pad = (int(t) for t in tiers)
    tier = "quad" if nquad else "pair" if npair else "one-lane"
    cyc = {"quad": 37.95, "pair": 42.2, "one-lane": 59.4}[tier]
    longest = int(descs["length"].max()) if len(descs) else 0
    blocks = (longest + 9 + 63) // 64
    floor_ms = blocks * 64 * cyc / 2.4e9 * 1e3
    res = {"longest_chunk_bytes": longest, "blocks": blocks, "tier": tier,
           "workgroups": {"quad": nquad, "pair": npair, "one_lane": nlane, "lds_pad": pad},
           "cycles_per_round": cyc, "clock_GHz": 2.4, "floor_ms": round(floor_ms, 3),
           "frac": round(floor_ms / dig_ms, 4) if dig_ms else None}
    if clk and clk.get("clock_GHz"):
        # the same floor at the clock the longest chain ran at (scripts/sha_clock.py)
        g = float(clk["clock_GHz"])
        f = blocks * 64 * cyc / (g * 1e9) * 1e3
        res["measured_clock"] = {"clock_GHz": g, "floor_ms": round(f, 3), "frac": round(f / dig_ms, 4) if dig_ms else None,
                                 "cycles_per_round_in_place": clk.get("cycles_per_round_wg0"),
                                 "source": "scripts/sha_clock.py (diagnostics build, same batch shape)"}
    return res


def scan_kernel_name(ca, avg, nbytes):
    """The K1 kernel launch_scan (scan.hip) picks for these params: k_scan when the
    prefilter sees fewer than 14 bits of mask_s & mask_l above bit 15, else the persistent
    k_scan_flat32p from 4 GiB (2^20 segments) on and the one-shot k_scan_flat32 below."""
    import math

    _, masks = ca.get_cdc_tables()
    bits = round(math.log2(avg))
    both = int(masks[bits + 1]) & int(masks[bits - 1])
    if bin(both >> 16).count("1") < 14:
        return "k_scan"
    return "k_scan_flat32p" if (nbytes + 4095) // 4096 >= (1 << 20) else "k_scan_flat32"


def pmc_traffic(config, kernels):
    """HBM bytes per launch of `kernels` from the committed rocprofv3 --pmc summary for
    this config (profiles/*pmc_<config>.json, written by scripts/pmc_summary.py from
    scripts/gpu_pmc.sh passes): FETCH_SIZE x 2 (gfx950 correction, MI355X_MICROARCH.md
    §HBM) + WRITE_SIZE.  (None, None) when no summary has been committed."""
    # newest = highest (round, version): natural order, so r02_v10 sorts after r02_v3
    files = sorted(ROOT.glob(f"profiles/*pmc_{config}.json"),
                   key=lambda f: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", f.name)])
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


def cpu_baseline(args, n_per, nar_bytes, params, algo):
    """The oracle's restatement of the reference's CPU path, timed on this host:

    * value: chunk_descriptors (src/chunking.rs:323-374) one call per NAR -- serial
      FastCDC scan, then per-chunk digests on a pool of `cores` threads (rayon's role)
      -- over the whole 1 GiB batch (c2/c3) or one 1 GiB NAR (c4/c5);
    * nar_parallel: the CPU upper bound, NARs spread over the same pool, one
      single-threaded chunk_descriptors per NAR, over at least one NAR per thread (for
      c4/c5: `cores` NARs of 1 GiB, not the one-NAR sample);
    * config1: BASELINE config 1 (benches/throughput.rs:39-43), chunk_data on 10 MiB
      with payload copies (:265-296), D params, SHA-256, median of 7 runs, on zeros
      (the published bench's data, 1.055 GiB/s in benchmarks/latest.md:12) and on
      xorshift64 bytes."""
    from concurrent.futures import ThreadPoolExecutor

    from chunker_amd.nar import synth_nars
    from oracle import oracle as O

    nt, affinity, quota = host_cpus()
    O.lib()
    k = args.cpu_sample_nars or (n_per if nar_bytes <= (64 << 20) else 1)
    host, offs = synth_nars(np.full(k, nar_bytes, np.uint64), zeros=args.zeros, first_index=0)
    nars = [host[int(offs[i]):int(offs[i + 1])] for i in range(k)]
    O.chunk_descriptors(nars[0][: 8 << 20], *params, algo=algo, nthreads=nt)  # warm
    reps = 5  # median of five passes over the sample (~2-5 s of CPU work in all)
    dts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        for nar in nars:
            O.chunk_descriptors(nar, *params, algo=algo, nthreads=nt)
        dts.append(time.perf_counter() - t0)
    dt = float(np.median(dts))
    nbytes = int(offs[-1])
    # the NAR-parallel bound needs at least one NAR per thread: for the 1 GiB-NAR configs
    # that is `nt` NARs of the config's size (the sample above is one)
    par = nars
    if len(par) < nt:
        extra, eoffs = synth_nars(np.full(nt - len(par), nar_bytes, np.uint64), zeros=args.zeros, first_index=k)
        par = par + [extra[int(eoffs[i]):int(eoffs[i + 1])] for i in range(nt - len(nars))]
    par_bytes = sum(len(a) for a in par)
    par_reps = reps if par_bytes <= (4 << 30) else 3
    with ThreadPoolExecutor(nt) as ex:
        dps = []
        for _ in range(par_reps):
            t1 = time.perf_counter()
            list(ex.map(lambda a: O.chunk_descriptors(a, *params, algo=algo, nthreads=1), par))
            dps.append(time.perf_counter() - t1)
        dt_par = float(np.median(dps))
    del par

    def chunk_data(buf):  # chunk_data_with_hash: descriptors + an owned payload copy per chunk
        return [(bytes(buf[int(d["offset"]):int(d["offset"] + d["length"])]), d)
                for d in O.chunk_descriptors(buf, 256 << 10, 1 << 20, 4 << 20, algo=1, nthreads=nt)]

    c1 = {}
    ten = 10 * 1024 * 1024
    for name, buf in (("zeros", np.zeros(ten, np.uint8)),
                      ("random", synth_nars([ten], first_index=7)[0])):
        chunk_data(buf)
        ts = []
        for _ in range(7):
            t = time.perf_counter()
            chunk_data(buf)
            ts.append(time.perf_counter() - t)
        c1[name] = round(ten / float(np.median(ts)) / GIB, 3)
    c1["published_zeros"] = PUBLISHED_CHUNK_DATA_ZEROS
    return {"value": round(nbytes / dt / GIB, 4), "unit": "GiB/s", "cores": nt,
            "cores_note": f"threads = the CPUs this process may use: affinity {affinity}, cgroup cpu.max quota "
                          f"{quota if quota else 'none'} (rayon's hardware_concurrency() inside the same cgroup)",
            "kind": "port",
            "sample": f"{k} NAR(s) ({nbytes / GIB:.3f} GiB) of the same workload, one chunk_descriptors call "
                      f"per NAR, median of {reps} passes, SHA-NI={'yes' if O.lib().or_sha256_uses_shani() else 'no'}",
            "seconds": round(dt, 3),
            "nar_parallel": round(par_bytes / dt_par / GIB, 4),
            "nar_parallel_sample": f"{max(k, nt)} NAR(s) of {nar_bytes >> 20} MiB, one single-threaded "
                                   f"chunk_descriptors per NAR on {nt} threads, median of {par_reps}",
            "config1_chunk_data_10MiB_D_sha256": c1,
            "cpu_model": cpu_model()}


def host_cpus():
    """(usable, affinity, quota): the CPUs this process may use -- its affinity set,
    capped by the cgroup v2 CPU quota (/sys/fs/cgroup/cpu.max) when one is set.  On the
    GPU box a one-GPU job sees the host's 256 hardware threads in its affinity mask but
    a 16-CPU quota; more threads than the quota only time-slice the same 16 CPUs."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = max(1, int(q) // int(period))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), aff, quota


def cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()

"""Multi-process (world size 2, gloo on CPU) coverage of the N>1 path: NAR
sharding and the descriptor gather to rank 0 (chunker_amd/dist.py), the same code
bench.py runs over RCCL on MI355X."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from chunker_amd.dist import DESC_BYTES, gather_descriptors, shard_nars


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_nars_partition():
    for n in [0, 1, 7, 128, 129, 1000]:
        for world in [1, 2, 3, 8]:
            got = [list(shard_nars(n, world, r)) for r in range(world)]
            assert sum(got, []) == list(range(n))
            sizes = [len(g) for g in got]
            assert max(sizes) - min(sizes) <= 1
    assert list(shard_nars(128, 8, 3)) == list(range(48, 64))  # config 5: 16 x 1 GiB per GPU


def _worker(rank, world, port, counts, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = counts[rank]
    rng = np.random.default_rng(rank)
    mine = rng.integers(0, 256, max(n, 1) * DESC_BYTES + 96, dtype=np.uint8)  # spare tail beyond n
    out = gather_descriptors(torch.from_numpy(mine), n)
    if rank == 0:
        q.put([o.numpy().tobytes() for o in out])
    dist.destroy_process_group()


@pytest.mark.parametrize("counts", [(5, 3), (0, 4), (2, 0), (0, 0)])
def test_gather_descriptors_gloo(counts):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, counts, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        rng = np.random.default_rng(r)
        want = rng.integers(0, 256, max(counts[r], 1) * DESC_BYTES + 96, dtype=np.uint8)[: counts[r] * DESC_BYTES]
        assert got[r] == want.tobytes()


def _shard_worker(rank, world, port, n_total, params, q):
    """One rank of the sharded pipeline on CPU: the oracle stands in for the GPU engine
    (same descriptor layout), the gather is the code bench.py runs over RCCL."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from chunker_amd.dist import gather_batch
    from chunker_amd.nar import synth_nars
    from oracle import oracle as O

    mine = shard_nars(n_total, world, rank)
    sizes = [200_000 + 8 * (i % 5) for i in mine]
    descs, first = [], [0]
    if len(sizes):
        data, offs = synth_nars(sizes, first_index=mine.start)
        for i in range(len(sizes)):
            d = O.chunk_descriptors(data[offs[i]:offs[i + 1]], *params, algo=1, nthreads=1)
            descs.append(d)
            first.append(first[-1] + len(d))
    flat = np.concatenate(descs) if descs else np.zeros(0, O.DESC_DTYPE)
    buf = torch.from_numpy(np.concatenate([flat.view(np.uint8), np.zeros(96, np.uint8)]))
    out = gather_batch(buf, np.array(first, np.uint64))
    if rank == 0:
        q.put((out[0].numpy().tobytes(), out[1].tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [7, 1])
def test_sharded_batch_reassembles_single_process_result(n_total):
    """shard_nars + per-rank chunking + gather_batch == one process over all NARs
    (world size 2, gloo); n_total = 1 leaves rank 1 with no NAR."""
    from chunker_amd.nar import synth_nars
    from oracle import oracle as O

    world, params = 2, (4096, 16384, 65536)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, n_total, params, q)) for r in range(world)]
    for p in procs:
        p.start()
    got_bytes, got_first = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sizes = [200_000 + 8 * (i % 5) for i in range(n_total)]
    data, offs = synth_nars(sizes, first_index=0)
    want, first = [], [0]
    for i in range(n_total):
        d = O.chunk_descriptors(data[offs[i]:offs[i + 1]], *params, algo=1, nthreads=1)
        want.append(d)
        first.append(first[-1] + len(d))
    assert got_first == first
    assert got_bytes == np.concatenate(want).tobytes()


def _gpu_shard_worker(rank, world, port, n_total, params, q):
    """One rank of bench.py's sharded step on the GPU engine: its shard synthesised in
    HBM, chunked + digested by cg_chunk_batch_device, gathered to rank 0 (gloo over host
    copies here: two ranks share the box's one GPU, where RCCL needs one GPU per rank)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import chunker_amd as ca
    from chunker_amd.dist import gather_batch
    from chunker_amd.nar import synth_nars_device

    torch.cuda.set_device(0)
    mine = shard_nars(n_total, world, rank)
    sizes = np.array([300_000 + 8 * (i % 7) for i in mine], np.uint64)
    if len(sizes):
        d, offs = synth_nars_device(sizes, first_index=mine.start)
        cap = ca.chunking.batch_capacity(offs, params[0])
        out = torch.empty(cap * DESC_BYTES, dtype=torch.uint8, device="cuda")
        first = ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params, hash=1,
                                      stream=torch.cuda.current_stream().cuda_stream)
        host = out[: int(first[-1]) * DESC_BYTES].cpu()
    else:
        first, host = np.zeros(1, np.uint64), torch.zeros(0, dtype=torch.uint8)
    res = gather_batch(torch.cat([host, torch.zeros(96, dtype=torch.uint8)]), first)
    if rank == 0:
        q.put((res[0].numpy().tobytes(), res[1].tolist()))
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("n_total", [9, 1])
def test_gpu_sharded_batch_matches_oracle(n_total):
    """Two ranks of the sharded device pipeline (shard_nars -> synth in HBM ->
    cg_chunk_batch_device -> gather_batch) reassemble exactly the oracle's descriptors
    over all NARs; n_total = 1 leaves rank 1 without a NAR."""
    from chunker_amd.nar import synth_nars
    from oracle import oracle as O

    world, params = 2, (8192, 32768, 131072)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_shard_worker, args=(r, world, port, n_total, params, q)) for r in range(world)]
    for p in procs:
        p.start()
    got_bytes, got_first = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sizes = [300_000 + 8 * (i % 7) for i in range(n_total)]
    data, offs = synth_nars(sizes, first_index=0)
    want, first = [], [0]
    for i in range(n_total):
        dsc = O.chunk_descriptors(data[offs[i]:offs[i + 1]], *params, algo=1, nthreads=1)
        want.append(dsc)
        first.append(first[-1] + len(dsc))
    assert got_first == first
    assert got_bytes == np.concatenate(want).tobytes()


def test_check_gathered_batch():
    """The rank-0 structural check bench.py runs on the gathered batch accepts a
    well-formed batch and names the NAR of every kind of defect."""
    from chunker_amd.dist import check_gathered_batch
    from oracle import oracle as O

    sizes = np.array([10, 0, 7, 5], np.uint64)
    d = np.zeros(5, O.DESC_DTYPE)
    d["offset"] = [0, 4, 0, 0, 3]
    d["length"] = [4, 6, 7, 3, 2]
    first = np.array([0, 2, 2, 3, 5], np.uint64)
    check_gathered_batch(d, first, sizes)
    check_gathered_batch(np.zeros(0, O.DESC_DTYPE), np.zeros(3, np.uint64), [0, 0])
    bad = d.copy()
    bad["offset"][1] = 5  # gap inside NAR 0
    with pytest.raises(AssertionError, match="NAR 0"):
        check_gathered_batch(bad, first, sizes)
    bad = d.copy()
    bad["length"][4] = 1  # NAR 3 ends short
    with pytest.raises(AssertionError, match="NAR 3"):
        check_gathered_batch(bad, first, sizes)
    with pytest.raises(AssertionError, match="NAR 1"):  # an empty NAR given a chunk
        check_gathered_batch(d, np.array([0, 1, 2, 3, 5], np.uint64), sizes)
    with pytest.raises(AssertionError, match="ends at"):
        check_gathered_batch(d, np.array([0, 2, 2, 3, 4], np.uint64), sizes)
    bad = d.copy()
    bad["offset"][2] = 1  # NAR 2 does not start at 0
    with pytest.raises(AssertionError, match="NAR 2"):
        check_gathered_batch(bad, first, sizes)


def test_gather_batch_async_refuses_batches_past_the_agreed_shape():
    """A rank whose batch exceeds the shapes gather_shape agreed must fail, not be truncated
    (the descriptors past max_cap would be dropped and rank 0 would mis-assemble the batch).
    The checks run before any collective, so no process group is needed."""
    from chunker_amd.dist import gather_batch_async

    desc = torch.zeros(5 * DESC_BYTES, dtype=torch.uint8)
    with pytest.raises(ValueError, match="max_cap"):
        gather_batch_async(desc, np.array([0, 5], np.uint64), max_cap=4, max_nars=1)
    with pytest.raises(ValueError, match="max_nars"):
        gather_batch_async(desc, np.array([0, 2, 5], np.uint64), max_cap=8, max_nars=1)
    with pytest.raises(ValueError, match="fewer bytes"):
        gather_batch_async(desc[:48], np.array([0, 5], np.uint64), max_cap=8, max_nars=1)

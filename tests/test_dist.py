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

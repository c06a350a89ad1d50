"""Multi-GPU plumbing: one process per GPU, NARs sharded one-file-per-GPU, chunk
descriptors gathered to rank 0.

The reference has no distributed compute: NARs are independent
(FastCDC state never crosses files), so the only exchange is collecting every
rank's descriptors on one rank.  On MI355X that is a torch.distributed gather over
RCCL/xGMI ("nccl" backend); the same code runs over gloo on CPU for tests.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

DESC_BYTES = 48


def shard_nars(n_total: int, world: int, rank: int) -> range:
    """Contiguous block of NAR indices for `rank` (balanced to within one NAR)."""
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def gather_descriptors(desc: torch.Tensor, n: int, group=None) -> list[torch.Tensor] | None:
    """Gather `n` descriptors (desc = uint8 tensor holding >= n*48 bytes) from every
    rank to rank 0.  Counts travel first (all_gather of one int64 per rank), then the
    descriptor arrays, padded to the largest count.  Returns the per-rank uint8
    tensors (n_r*48 bytes each) on rank 0, None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = desc.device
    cnt = torch.tensor([n], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    counts = [int(c.item()) for c in cnts]
    mx = max(counts)
    if mx == 0:
        return [desc[:0] for _ in range(world)] if rank == 0 else None
    buf = desc[: n * DESC_BYTES]
    if n < mx:
        buf = torch.cat([buf, torch.zeros((mx - n) * DESC_BYTES, dtype=torch.uint8, device=dev)])
    gl = [torch.empty(mx * DESC_BYTES, dtype=torch.uint8, device=dev) for _ in range(world)] if rank == 0 else None
    dist.gather(buf.contiguous(), gl, dst=0, group=group)
    if rank != 0:
        return None
    return [g[: c * DESC_BYTES] for g, c in zip(gl, counts)]


def gather_batch(desc: torch.Tensor, nar_first, group=None):
    """Gather a sharded batch to rank 0: each rank's descriptors (desc holds its
    nar_first[-1] descriptors, 48 B each) and its NAR -> first-descriptor index.
    Shards are contiguous NAR ranges in rank order (shard_nars), so rank 0 rebuilds the
    whole batch in global NAR order: returns (uint8 tensor of all descriptors on rank
    0's device, global nar_first as np.uint64[n_total + 1]) on rank 0, None elsewhere."""
    first = np.asarray(nar_first, dtype=np.uint64)
    n = int(first[-1])
    parts = gather_descriptors(desc, n, group=group)
    dev = desc.device
    # NAR indices travel as one more gather (n_nars + 1 u64 per rank, padded)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    cnt = torch.tensor([len(first)], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    lens = [int(c.item()) for c in cnts]
    mx = max(lens)
    buf = torch.zeros(mx, dtype=torch.int64, device=dev)
    buf[: len(first)] = torch.from_numpy(first.astype(np.int64)).to(dev)
    gl = [torch.empty(mx, dtype=torch.int64, device=dev) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gl, dst=0, group=group)
    if rank != 0:
        return None
    firsts, base = [np.zeros(1, np.uint64)], 0
    for g, ln in zip(gl, lens):
        f = g[:ln].cpu().numpy().astype(np.uint64)
        firsts.append(f[1:] + np.uint64(base))
        base += int(f[-1])
    return torch.cat(parts) if parts else desc[:0], np.concatenate(firsts)


def check_gathered_batch(descs: np.ndarray, first, nar_sizes) -> None:
    """Structural check of a batch gathered on rank 0 (bench.py runs it at N > 1 before
    printing): `first` (global NAR -> first-descriptor index, n_nars + 1 entries) starts
    at 0, strictly increases (every non-empty NAR has >= 1 chunk, an empty one none) and
    ends at the descriptor count; inside every NAR the descriptors tile [0, size) in
    order with no gap, overlap or empty chunk (src/chunking.rs:567-570).  Raises
    AssertionError naming the first NAR that fails."""
    first = np.asarray(first, dtype=np.int64)
    sizes = np.asarray(nar_sizes, dtype=np.int64)
    assert len(first) == len(sizes) + 1, f"nar_first has {len(first)} entries for {len(sizes)} NARs"
    assert first[0] == 0 and first[-1] == len(descs), f"nar_first ends at {first[-1]}, {len(descs)} descriptors"
    counts = np.diff(first)
    bad = np.flatnonzero((counts < 0) | ((counts == 0) != (sizes == 0)))
    assert not len(bad), f"NAR {bad[0]}: {counts[bad[0]]} chunks for {sizes[bad[0]]} bytes"
    if not len(descs):
        return
    off = descs["offset"].astype(np.int64)
    ln = descs["length"].astype(np.int64)
    assert (ln > 0).all(), f"empty chunk at descriptor {int(np.flatnonzero(ln <= 0)[0])}"
    nar_of = np.repeat(np.arange(len(sizes)), counts)
    start = first[:-1][counts > 0]
    # within a NAR: the first chunk at 0, each next one where the previous ended
    expect = np.empty_like(off)
    expect[1:] = off[:-1] + ln[:-1]
    expect[start] = 0
    gap = np.flatnonzero(off != expect)
    assert not len(gap), f"NAR {nar_of[gap[0]]}: descriptor {gap[0]} at offset {off[gap[0]]}, expected {expect[gap[0]]}"
    last = first[1:][counts > 0] - 1
    end = off[last] + ln[last]
    short = np.flatnonzero(end != sizes[counts > 0])
    assert not len(short), f"NAR {np.flatnonzero(counts > 0)[short[0]]}: chunks end at {end[short[0]]}"

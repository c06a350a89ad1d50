"""Multi-GPU plumbing: one process per GPU, NARs sharded one-file-per-GPU, chunk
descriptors gathered to rank 0.

The reference has no distributed compute: NARs are independent
(FastCDC state never crosses files), so the only exchange is collecting every
rank's descriptors on one rank.  On MI355X that is a torch.distributed gather over
RCCL/xGMI ("nccl" backend); the same code runs over gloo on CPU for tests.  The
per-step gather (gather_batch_async) has fixed sizes agreed once (gather_shape), so it
is queued without a host sync and overlaps the next batch's kernels.
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


def gather_shape(desc_cap: int, n_nars: int, group=None) -> tuple[int, int]:
    """(largest descriptor capacity, largest NAR count) over the ranks: the padded sizes
    of gather_batch_async's two per-rank buffers.  One all_gather, once per batch shape
    (bench.py calls it before the timed region), so the per-step gather needs no count
    exchange and no host sync."""
    dev = _device_for(group)
    t = torch.tensor([desc_cap, n_nars], dtype=torch.int64, device=dev)
    world = dist.get_world_size(group)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    both = torch.stack(parts).cpu()
    return int(both[:, 0].max()), int(both[:, 1].max())


def _device_for(group=None):
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")


class GatheredBatch:
    """A gather queued by gather_batch_async: on rank 0 the per-rank packed buffers
    (filled when the current stream reaches the collective); `assemble()` waits for them
    and returns (uint8 tensor of every descriptor in global NAR order, global nar_first
    as np.uint64[n_total + 1])."""

    def __init__(self, parts, meta_bytes):
        self.parts, self.meta_bytes = parts, meta_bytes

    def assemble(self):
        mb = self.meta_bytes
        metas = [p[:mb].cpu().numpy().view(np.int64) for p in self.parts]  # the one host sync, off the step's path
        descs, firsts, base = [], [np.zeros(1, np.uint64)], 0
        for m, p in zip(metas, self.parts):
            n_nars, n_desc = int(m[0]), int(m[1])
            f = m[2:3 + n_nars].astype(np.uint64)
            descs.append(p[mb: mb + n_desc * DESC_BYTES])
            firsts.append(f[1:] + np.uint64(base))
            base += n_desc
        return torch.cat(descs), np.concatenate(firsts)


def gather_batch_async(desc: torch.Tensor, nar_first, max_cap: int, max_nars: int, group=None):
    """Queue the gather of this rank's batch to rank 0 on the current stream, with no host
    sync: ONE collective of fixed size (gather_shape) over a packed per-rank buffer --
    metadata {n_nars, n_descriptors, nar_first[0..n_nars]} as int64 padded to max_nars,
    then the descriptor array padded to max_cap.  Returns a GatheredBatch on rank 0, None
    elsewhere.  The packing copies `desc` on the current stream, so once this returns
    (and the stream has reached it) the caller may overwrite `desc`."""
    first = np.asarray(nar_first, dtype=np.uint64)
    # the shapes agreed by gather_shape bound every rank's buffer: a batch past them would be
    # truncated and mis-assembled on rank 0, so it is an error, never clamped
    if len(first) - 1 > max_nars:
        raise ValueError(f"gather_batch_async: {len(first) - 1} NARs exceed the agreed max_nars {max_nars}")
    if int(first[-1]) > max_cap:
        raise ValueError(f"gather_batch_async: {int(first[-1])} descriptors exceed the agreed max_cap {max_cap}")
    if desc.numel() < int(first[-1]) * DESC_BYTES:
        raise ValueError("gather_batch_async: desc holds fewer bytes than nar_first[-1] descriptors")
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = desc.device
    meta_h = np.zeros(max_nars + 3, np.int64)
    meta_h[0], meta_h[1] = len(first) - 1, int(first[-1])
    meta_h[2:2 + len(first)] = first.astype(np.int64)
    meta = torch.from_numpy(meta_h.view(np.uint8))
    mb = meta.numel()
    want = max_cap * DESC_BYTES
    n = int(first[-1]) * DESC_BYTES
    packed = torch.zeros(mb + want, dtype=torch.uint8, device=dev)
    packed[:mb].copy_(meta.pin_memory() if dev.type == "cuda" else meta, non_blocking=True)
    packed[mb: mb + n].copy_(desc[:n], non_blocking=True)
    gd = [torch.empty(mb + want, dtype=torch.uint8, device=dev) for _ in range(world)] if rank == 0 else None
    dist.gather(packed, gd, dst=0, group=group)
    return GatheredBatch(gd, mb) if rank == 0 else None


def gather_batch(desc: torch.Tensor, nar_first, group=None):
    """Gather a sharded batch to rank 0 and wait for it: each rank's descriptors (desc
    holds its nar_first[-1] descriptors, 48 B each) and its NAR -> first-descriptor index.
    Shards are contiguous NAR ranges in rank order (shard_nars), so rank 0 rebuilds the
    whole batch in global NAR order: returns (uint8 tensor of all descriptors on rank 0's
    device, global nar_first as np.uint64[n_total + 1]) on rank 0, None elsewhere."""
    first = np.asarray(nar_first, dtype=np.uint64)
    n = int(first[-1])
    max_cap, max_nars = gather_shape(max(n, 1), len(first) - 1, group=group)
    g = gather_batch_async(desc[: n * DESC_BYTES], first, max_cap, max_nars, group=group)
    return g.assemble() if g is not None else None


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

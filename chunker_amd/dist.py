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

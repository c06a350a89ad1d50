"""Synthetic NAR batches.

A synthetic NAR is a `nix-archive-1` serialisation of one regular file: Nix
strings (u64-LE length + bytes, zero-padded to 8) `nix-archive-1 ( type regular
contents <payload> )`, 112 bytes of framing in all.  The payload is the xorshift64
stream of the reference's own deterministic test data (crates/node/src/lib.rs:192-203:
state = seed | 1; state ^= state<<13; ^= >>7; ^= <<17; emit little-endian) with
seed 0x9E3779B97F4A7C15 ^ nar_index, or all zeros (the reference's published
benches run on zeros, benches/throughput.rs:16-17).
"""
from __future__ import annotations

import numpy as np

from ._lib import lib

FRAMING = 112
SEED_BASE = 0x9E3779B97F4A7C15


def synth_nars(sizes, zeros: bool = False, first_index: int = 0, out: np.ndarray | None = None):
    """Write len(sizes) NARs back to back; returns (bytes array, offsets[n+1])."""
    sizes = np.ascontiguousarray(sizes, dtype=np.uint64)
    if np.any(sizes % 8) or np.any(sizes < FRAMING + 8):
        raise ValueError("synthetic NAR sizes must be multiples of 8 and >= 120")
    offs = np.zeros(len(sizes) + 1, np.uint64)
    np.cumsum(sizes, out=offs[1:])
    total = int(offs[-1])
    if out is None:
        out = np.empty(total, np.uint8)
    assert out.dtype == np.uint8 and out.size >= total and out.flags.c_contiguous
    lib.cg_synth_nars(out.ctypes.data, sizes.ctypes.data, len(sizes), int(zeros), first_index)
    return out[:total], offs


def synth_nars_device(sizes, zeros: bool = False, first_index: int = 0, pad: int = 256,
                      host_chunk: int = 2 << 30):
    """The same batch written straight into one device buffer (a torch uint8 CUDA
    tensor of total + pad bytes), synthesised NAR group by NAR group through a host
    buffer of at most max(host_chunk, largest NAR) bytes: 16 GiB batches (BASELINE
    configs 4 and 5) need no 16 GiB host copy.  Returns (device tensor, offsets[n+1])."""
    import torch

    sizes = np.ascontiguousarray(sizes, dtype=np.uint64)
    offs = np.zeros(len(sizes) + 1, np.uint64)
    np.cumsum(sizes, out=offs[1:])
    total = int(offs[-1])
    dev = torch.empty(total + pad, dtype=torch.uint8, device="cuda")
    cap = max(host_chunk, int(sizes.max()) if len(sizes) else 0)
    host = torch.empty(cap, dtype=torch.uint8).pin_memory()
    hnp = host.numpy()
    i = 0
    while i < len(sizes):
        j, acc = i, 0
        while j < len(sizes) and acc + int(sizes[j]) <= cap:
            acc += int(sizes[j])
            j += 1
        synth_nars(sizes[i:j], zeros=zeros, first_index=first_index + i, out=hnp)
        dev[int(offs[i]):int(offs[j])].copy_(host[:acc])  # synchronous: the host buffer is reused
        i = j
    return dev, offs


def xorshift_bytes_py(seed: int, n: int) -> bytes:
    """Pure-Python xorshift64 stream (crates/node/src/lib.rs:192-203), for tests."""
    m = (1 << 64) - 1
    s = (seed | 1) & m
    out = bytearray()
    while len(out) < n:
        s ^= (s << 13) & m
        s ^= s >> 7
        s ^= (s << 17) & m
        out += s.to_bytes(8, "little")
    return bytes(out[:n])

"""Whole-NAR hash for narinfo ``NarHash``.

``NarHash: sha256:<nix-base32>`` is SHA-256 over the whole NAR
(crates/proto/nix/src/narinfo.rs:127-157) -- one serial Merkle-Damgard chain per NAR,
so on the GPU it is the K3 SHA-256 kernel with one span per NAR (cg_hash_spans_device):
a batch of NARs runs concurrently, each NAR at one chain's speed.
``nix_base32`` restates narinfo.rs:26-55 on the host (formatting only).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import lib
from .chunking import HashAlgorithm, _check
from .hashing import sha256_hash_raw

NIX_BASE32 = "0123456789abcdfghijklmnpqrsvwxyz"  # narinfo.rs:27 (RFC 4648 minus e, o, t, u)


def nix_base32(digest: bytes) -> str:
    """narinfo.rs:34-55: little-endian, high-index-first base-32 (52 chars for 32 bytes)."""
    if not digest:
        return ""
    n_chars = (len(digest) * 8 - 1) // 5 + 1
    out = []
    for n in range(n_chars - 1, -1, -1):
        b = n * 5
        i, j = b // 8, b % 8
        c = digest[i] >> j
        if i + 1 < len(digest):
            c |= digest[i + 1] << (8 - j)
        out.append(NIX_BASE32[c & 0x1F])
    return "".join(out)


def nar_hash_field(digest: bytes) -> str:
    """The narinfo value: ``sha256:<nix-base32>`` (narinfo.rs:157)."""
    return "sha256:" + nix_base32(digest)


def nar_hash(nar) -> bytes:
    """SHA-256 of one host NAR on the GPU."""
    return sha256_hash_raw(nar)


def nar_hashes_device(d_data_ptr: int, nar_offsets: np.ndarray, d_digests_ptr: int, stream: int = 0,
                      d_offsets_ptr: int | None = None, d_lengths_ptr: int | None = None) -> None:
    """SHA-256 of every NAR of a device-resident batch (NAR i = bytes
    [off[i], off[i+1])) into d_digests (32 B each).  The span arrays must be device
    arrays; pass them, or they are made with torch on the current device."""
    offs = np.asarray(nar_offsets, dtype=np.uint64)
    n = len(offs) - 1
    keep = None
    if d_offsets_ptr is None or d_lengths_ptr is None:
        import torch

        o = torch.from_numpy(offs[:-1].astype(np.int64)).cuda()
        ln = torch.from_numpy(np.diff(offs).astype(np.int64)).cuda()
        keep = (o, ln)
        d_offsets_ptr, d_lengths_ptr = o.data_ptr(), ln.data_ptr()
    _check(lib.cg_hash_spans_device(ctypes.c_void_p(d_data_ptr), ctypes.c_void_p(d_offsets_ptr),
                                    ctypes.c_void_p(d_lengths_ptr), n, int(HashAlgorithm.Sha256),
                                    ctypes.c_void_p(d_digests_ptr), ctypes.c_void_p(stream or None)))
    del keep

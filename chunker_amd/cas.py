"""CAS content identifiers and Node::put on the engine's gfx950 kernels
(SURVEY.md §8f rows 2-3).

Mirrors ``ObjectKind`` / ``ContentId`` (crates/core/cas/src/lib.rs:31-93) and the
ingest half of ``Node::put`` (crates/node/src/lib.rs:114-132): chunk with SHA-256
``chunk_data``, one ``ContentId(Chunk, payload)`` per chunk, and the manifest id
``ContentId(Level1Manifest, concatenated chunk ids)``.  Every id is computed by the
K5 SHAKE-256 kernel (chunker_amd/csrc/cas.hip); storage, dedup bookkeeping and the
metadata DAG are the caller's (out of scope).
"""
from __future__ import annotations

import ctypes
import enum
from dataclasses import dataclass

import numpy as np

from ._lib import DESC_DTYPE, lib
from .chunking import ChunkingOptions, ChunkMetadata, _as_u8, _check, _ptr, descriptors_to_list


class ObjectKind(enum.IntEnum):
    """crates/core/cas/src/lib.rs:31-48 (same discriminants)."""
    Chunk = 0x01
    Level0Manifest = 0x02
    Level1Manifest = 0x03
    Refcount = 0x04
    Witness = 0x05
    Recipe = 0x06
    Commit = 0x07


@dataclass(frozen=True)
class ContentId:
    """32-byte content identifier (crates/core/cas/src/lib.rs:50-93)."""
    raw: bytes

    @classmethod
    def compute(cls, kind: ObjectKind, payload) -> "ContentId":
        """ContentId::compute (:59-69) on the GPU (cg_cas_id)."""
        a = _as_u8(payload)
        out = (ctypes.c_uint8 * 32)()
        _check(lib.cg_cas_id(_ptr(a), len(a), int(ObjectKind(kind)), out))
        return cls(bytes(out))

    @classmethod
    def from_bytes(cls, b: bytes) -> "ContentId":
        if len(b) != 32:
            raise ValueError("content id is 32 bytes")
        return cls(bytes(b))

    def as_bytes(self) -> bytes:
        return self.raw

    def to_hex(self) -> str:
        return self.raw.hex()


def content_ids_device(d_data_ptr: int, d_offsets_ptr: int, d_lengths_ptr: int, n: int, kind: ObjectKind,
                       d_ids_ptr: int, stream: int = 0) -> None:
    """ContentId::compute over n device-resident spans (cg_cas_ids_device); ids -> n*32 bytes."""
    _check(lib.cg_cas_ids_device(ctypes.c_void_p(d_data_ptr), ctypes.c_void_p(d_offsets_ptr),
                                 ctypes.c_void_p(d_lengths_ptr), n, int(ObjectKind(kind)),
                                 ctypes.c_void_p(d_ids_ptr), ctypes.c_void_p(stream or None)))


@dataclass
class PutResult:
    """What Node::put computes before touching storage: the manifest id it returns
    (:131), the chunks it stores (:116-122) and their ids in manifest order."""
    manifest: ContentId
    chunks: list
    chunk_ids: list


def node_put(data, min_size=None, avg_size=None, max_size=None) -> PutResult:
    """Node::put (crates/node/src/lib.rs:114-132) minus the storage writes.  Chunks are
    SHA-256 descriptors, as chunk_data always hashes with SHA-256 (src/chunking.rs:242-249)."""
    o = ChunkingOptions.resolve(min_size, avg_size, max_size)
    a = _as_u8(data)
    cap = int(lib.cg_capacity(len(a), o.min_size))
    out = np.zeros(cap, DESC_DTYPE)
    ids = np.zeros((cap, 32), np.uint8)
    man = (ctypes.c_uint8 * 32)()
    n = ctypes.c_size_t(0)
    _check(lib.cg_node_put(_ptr(a), len(a), o.min_size, o.avg_size, o.max_size, out.ctypes.data, cap,
                           ctypes.byref(n), ids.ctypes.data, man))
    descs = descriptors_to_list(out[:n.value])
    raw = bytes(a)
    chunks = [ChunkMetadata(d.hash, d.offset, d.length, raw[d.offset:d.offset + d.length]) for d in descs]
    return PutResult(ContentId(bytes(man)), chunks, [ContentId(bytes(r)) for r in ids[:n.value]])


def node_put_batch_device(d_data_ptr: int, nar_offsets: np.ndarray, d_out_ptr: int, out_cap: int,
                          d_chunk_ids_ptr: int, min_size=None, avg_size=None, max_size=None,
                          stream: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """Node::put over a device-resident batch of NARs (cg_node_put_batch_device).
    Returns (nar_first (n+1), manifest ids (n, 32))."""
    o = ChunkingOptions.resolve(min_size, avg_size, max_size)
    offs = np.ascontiguousarray(nar_offsets, dtype=np.uint64)
    n = len(offs) - 1
    first = np.zeros(n + 1, np.uint64)
    man = np.zeros((max(n, 1), 32), np.uint8)
    _check(lib.cg_node_put_batch_device(ctypes.c_void_p(d_data_ptr), offs.ctypes.data, n, o.min_size, o.avg_size,
                                        o.max_size, ctypes.c_void_p(d_out_ptr), out_cap, first.ctypes.data,
                                        ctypes.c_void_p(d_chunk_ids_ptr), man.ctypes.data,
                                        ctypes.c_void_p(stream or None)))
    return first, man[:n]


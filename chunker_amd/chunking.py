"""Host-side mirror of FlakeCache/chunker's chunking API (src/chunking.rs), backed by
the gfx950 engine through the C ABI.

Names, argument meaning and error behaviour follow the reference so its tests read
the same here:

=====================================  ======================================================
this module                            reference (src/chunking.rs)
=====================================  ======================================================
ChunkingError and subclasses           ChunkingError :33-51 (same Display strings)
HashAlgorithm                          :53-58
ChunkMetadata / ChunkDescriptor        :76-155 (equality ignores payload, :120-134)
ChunkingOptions.resolve                :157-231
chunk_data / chunk_data_with_hash      :241-297
chunk_descriptors[_with_hash]          :299-374
ChunkStream                            :382-740 (read-slice sizing :713-716, env cap :427-433),
                                       pipelined on the GPU (cg_stream_*)
PushChunker                            :742-829
ChunkStreamAsync (asyncio)             :835-1017 (feature async-stream), same handle
chunk_data_async / chunk_stream_async  :1049-1130 (buffer limit :420-445)
BlockingAsyncReadAdapter,              :1019-1047, :1090-1113
  chunk_stream_blocking_adapter
chunk_stream / chunk_stream_with_hash  :1132-1166
metrics (StreamMetrics)                :398-416 (recorded by the streaming paths only)
=====================================  ======================================================

Plus batch entry points the reference has no equivalent for (many NARs per call,
device-resident inputs): chunk_batch, chunk_batch_device.
"""
from __future__ import annotations

import asyncio
import ctypes
import enum
import os
from collections import deque
from dataclasses import dataclass, field
from typing import BinaryIO, Iterator, Sequence

import numpy as np

from . import _lib
from ._lib import DESC_DTYPE, lib

DEFAULT_MIN = 256 * 1024
DEFAULT_AVG = 1024 * 1024
DEFAULT_MAX = 4 * 1024 * 1024

# fastcdc::v2020 ranges [ext] (pinned by src/chunking.rs:1401-1415)
MINIMUM_MIN, MINIMUM_MAX = 64, 1_048_576
AVERAGE_MIN, AVERAGE_MAX = 256, 4_194_304
MAXIMUM_MIN, MAXIMUM_MAX = 1024, 16_777_216

DEFAULT_READ_SLICE_CAP = 8 * 1024 * 1024
MAX_READ_SLICE_CAP = 256 * 1024 * 1024
MIN_READ_SLICE_CAP = 4096
# ChunkStreamAsync collection cap (src/chunking.rs:420-425)
DEFAULT_ASYNC_BUFFER_LIMIT = 2 * 1024 * 1024 * 1024
MAX_ASYNC_BUFFER_LIMIT = 3 * 1024 * 1024 * 1024
MIN_ASYNC_BUFFER_LIMIT = 64 * 1024 * 1024


# ---------------------------------------------------------------------------
# errors (src/chunking.rs:33-51)
# ---------------------------------------------------------------------------
class ChunkingError(Exception):
    """Base of the ChunkingError variants."""


class BoundsError(ChunkingError):
    def __init__(self, data_len: int, offset: int, length: int):
        self.data_len, self.offset, self.length = data_len, offset, length
        super().__init__(
            f"bounds_check_failed: offset {offset} + length {length} exceeds data length {data_len}")


class IoError(ChunkingError):
    def __init__(self, msg: str):
        super().__init__(f"io_error: {msg}")


class ZeroLengthChunkError(ChunkingError):
    def __init__(self):
        super().__init__("zero_length_chunk: FastCDC returned a chunk with length 0")


class InvalidOptionsError(ChunkingError):
    def __init__(self, msg: str):
        self.detail = msg
        super().__init__(f"invalid_chunking_options: {msg}")


class BufferLimitExceededError(ChunkingError):
    def __init__(self, attempted: int, limit: int):
        self.attempted, self.limit = attempted, limit
        super().__init__(f"buffer_limit_exceeded: attempted {attempted} bytes, limit {limit} bytes")


class DeviceUnavailableError(IoError):
    """No gfx950 device: the engine has no CPU fallback (ABI status CG_E_NO_DEVICE)."""


class TablesError(IoError):
    """FastCDC tables refused (ABI status CG_E_TABLES): the placeholder GEAR is installed
    or the installed set failed the reference-fixture selftest (include/chunker_gpu.h)."""


def _raise(status: int) -> None:
    """Rebuild the reference's ChunkingError variant from the ABI status and the
    failure's fields (cg_last_error_detail), as the Rust shim does."""
    msg = _lib.last_error()
    _, a, b, c = _lib.last_error_detail()
    if status == _lib.CG_E_INVALID_OPTIONS:
        raise InvalidOptionsError(msg)
    if status == _lib.CG_E_BOUNDS:
        raise BoundsError(a, b, c)
    if status == _lib.CG_E_ZERO_LENGTH_CHUNK:
        raise ZeroLengthChunkError()
    if status == _lib.CG_E_BUFFER_LIMIT:
        raise BufferLimitExceededError(a, b)
    if status == _lib.CG_E_NO_DEVICE:
        raise DeviceUnavailableError(msg)
    if status == _lib.CG_E_TABLES:
        raise TablesError(msg)
    raise IoError(msg or f"engine status {status}")


def _check(status: int) -> None:
    if status != _lib.CG_OK:
        _raise(status)


# ---------------------------------------------------------------------------
# FastCDC tables (fastcdc 4.0.1 v2020 GEAR / MASKS): install, inspect, verify
# ---------------------------------------------------------------------------
def set_cdc_tables(gear, masks=None) -> None:
    """Install GEAR[256] (and MASKS[26], or keep the current ones) process-wide.  The
    engine runs the new set only after it reproduces the reference fixture
    (src/chunking.rs:1266-1297) on the GPU -- see selftest()."""
    g = np.ascontiguousarray(gear, dtype=np.uint64)
    if g.shape != (256,):
        raise InvalidOptionsError("GEAR must have 256 entries")
    m = None if masks is None else np.ascontiguousarray(masks, dtype=np.uint64)
    if m is not None and m.shape != (26,):
        raise InvalidOptionsError("MASKS must have 26 entries")
    _check(lib.cg_set_cdc_tables(g.ctypes.data, None if m is None else m.ctypes.data))


def get_cdc_tables() -> tuple[np.ndarray, np.ndarray]:
    g, m = np.zeros(256, np.uint64), np.zeros(26, np.uint64)
    lib.cg_get_cdc_tables(g.ctypes.data, m.ctypes.data)
    return g, m


def selftest() -> None:
    """Run the reference's golden boundary fixture through the GPU pipeline with the
    installed tables; raises TablesError (with the boundaries found) on a mismatch."""
    _check(lib.cg_selftest())


def tables_verified() -> bool:
    return bool(lib.cg_tables_verified())


# ---------------------------------------------------------------------------
# value types
# ---------------------------------------------------------------------------
class HashAlgorithm(enum.IntEnum):
    """HashAlgorithm (src/chunking.rs:53-58); values are the ABI's cg_hash_algo."""
    Blake3 = 0
    Sha256 = 1


@dataclass(frozen=True)
class ChunkDescriptor:
    """ChunkDescriptor (src/chunking.rs:100-118)."""
    hash: bytes
    offset: int
    length: int

    def hash_hex(self) -> str:
        return self.hash.hex()


@dataclass(eq=False)
class ChunkMetadata:
    """ChunkMetadata (src/chunking.rs:76-98); equality/hash ignore payload (:120-134).
    payload is bytes-like: `bytes`, or from ChunkStream a read-only memoryview into the
    slice it was read in (zero-copy, like the reference's `Bytes`)."""
    hash: bytes
    offset: int
    length: int
    payload: bytes | memoryview = field(default=b"", repr=False)

    def hash_hex(self) -> str:
        return self.hash.hex()

    def __eq__(self, other) -> bool:
        if not isinstance(other, ChunkMetadata):
            return NotImplemented
        return (self.hash, self.offset, self.length) == (other.hash, other.offset, other.length)

    def __hash__(self) -> int:
        return hash((self.hash, self.offset, self.length))


@dataclass(frozen=True)
class ChunkingOptions:
    """ChunkingOptions (src/chunking.rs:157-231)."""
    min_size: int
    avg_size: int
    max_size: int

    @classmethod
    def resolve(cls, min_size=None, avg_size=None, max_size=None) -> "ChunkingOptions":
        o = cls(DEFAULT_MIN if min_size is None else int(min_size),
                DEFAULT_AVG if avg_size is None else int(avg_size),
                DEFAULT_MAX if max_size is None else int(max_size))
        o.validate()
        return o

    def validate(self) -> None:
        """src/chunking.rs:190-231, same order and messages (the ABI re-checks)."""
        for name, v, lo, hi in (("min_size", self.min_size, MINIMUM_MIN, MINIMUM_MAX),
                                ("avg_size", self.avg_size, AVERAGE_MIN, AVERAGE_MAX),
                                ("max_size", self.max_size, MAXIMUM_MIN, MAXIMUM_MAX)):
            if not lo <= v <= hi:
                raise InvalidOptionsError(f"{name} must be in {lo}..={hi}, got {v}")
        if self.min_size > self.avg_size:
            raise InvalidOptionsError("min_size must be <= avg_size")
        if self.avg_size > self.max_size:
            raise InvalidOptionsError("avg_size must be <= max_size")


# ---------------------------------------------------------------------------
# helpers
# ---------------------------------------------------------------------------
def _as_u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        a = data.reshape(-1)
        if a.dtype != np.uint8:
            a = a.view(np.uint8)
        return np.ascontiguousarray(a)
    return np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)


def _ptr(a: np.ndarray):
    return a.ctypes.data if a.size else None


def descriptors_to_list(arr: np.ndarray) -> list[ChunkDescriptor]:
    return [ChunkDescriptor(bytes(r["hash"]), int(r["offset"]), int(r["length"])) for r in arr]


# ---------------------------------------------------------------------------
# eager API
# ---------------------------------------------------------------------------
def chunk_descriptors_array(data, min_size=None, avg_size=None, max_size=None,
                            hash: HashAlgorithm = HashAlgorithm.Sha256) -> np.ndarray:
    """chunk_descriptors_with_hash as a structured numpy array (DESC_DTYPE)."""
    o = ChunkingOptions.resolve(min_size, avg_size, max_size)
    a = _as_u8(data)
    cap = max(lib.cg_capacity(len(a), o.min_size), 1)
    out = np.zeros(cap, DESC_DTYPE)
    n = ctypes.c_size_t(0)
    _check(lib.cg_chunk_descriptors(_ptr(a), len(a), o.min_size, o.avg_size, o.max_size, int(hash),
                                    out.ctypes.data, cap, ctypes.byref(n)))
    return out[: n.value]


def chunk_descriptors_with_hash(data, min_size=None, avg_size=None, max_size=None,
                                hash: HashAlgorithm = HashAlgorithm.Sha256) -> list[ChunkDescriptor]:
    """src/chunking.rs:323-374."""
    return descriptors_to_list(chunk_descriptors_array(data, min_size, avg_size, max_size, hash))


def chunk_descriptors(data, min_size=None, avg_size=None, max_size=None) -> list[ChunkDescriptor]:
    """src/chunking.rs:308-315 (SHA-256)."""
    return chunk_descriptors_with_hash(data, min_size, avg_size, max_size, HashAlgorithm.Sha256)


def chunk_data_with_hash(data, min_size=None, avg_size=None, max_size=None,
                         hash: HashAlgorithm = HashAlgorithm.Sha256) -> list[ChunkMetadata]:
    """src/chunking.rs:256-297: descriptors plus an owned payload copy per chunk."""
    a = _as_u8(data)
    out = []
    for d in chunk_descriptors_array(a, min_size, avg_size, max_size, hash):
        off, ln = int(d["offset"]), int(d["length"])
        if off + ln > len(a):  # bounds check (:268-287)
            raise BoundsError(len(a), off, ln)
        out.append(ChunkMetadata(bytes(d["hash"]), off, ln, a[off:off + ln].tobytes()))
    return out


def chunk_data(data, min_size=None, avg_size=None, max_size=None) -> list[ChunkMetadata]:
    """src/chunking.rs:241-249 (SHA-256)."""
    return chunk_data_with_hash(data, min_size, avg_size, max_size, HashAlgorithm.Sha256)


# ---------------------------------------------------------------------------
# batch API (one engine call for many independent NARs)
# ---------------------------------------------------------------------------
def chunk_batch(nars: Sequence, min_size=None, avg_size=None, max_size=None,
                hash: HashAlgorithm = HashAlgorithm.Sha256) -> list[np.ndarray]:
    """Chunk every NAR of `nars` independently (== one chunk_descriptors_with_hash
    per NAR) in a single device pass; returns one descriptor array per NAR."""
    o = ChunkingOptions.resolve(min_size, avg_size, max_size)
    arrs = [_as_u8(x) for x in nars]
    offs = np.zeros(len(arrs) + 1, np.uint64)
    np.cumsum([len(x) for x in arrs], out=offs[1:])
    flat = np.concatenate(arrs) if arrs else np.zeros(0, np.uint8)
    cap = max(sum(lib.cg_capacity(len(x), o.min_size) for x in arrs), 1)
    out = np.zeros(cap, DESC_DTYPE)
    first = np.zeros(len(arrs) + 1, np.uint64)
    _check(lib.cg_chunk_batch(_ptr(flat), offs.ctypes.data, len(arrs), o.min_size, o.avg_size, o.max_size,
                              int(hash), out.ctypes.data, cap, first.ctypes.data))
    return [out[int(first[i]):int(first[i + 1])] for i in range(len(arrs))]


def chunk_batch_flat(flat, nar_offsets, min_size=None, avg_size=None, max_size=None,
                     hash: HashAlgorithm = HashAlgorithm.Sha256, out: np.ndarray | None = None):
    """Host-resident batch without re-packing: `flat` holds the NARs back to back,
    NAR i = flat[nar_offsets[i]:nar_offsets[i+1]].  Returns (descriptors, nar_first)."""
    o = ChunkingOptions.resolve(min_size, avg_size, max_size)
    a = _as_u8(flat)
    offs = np.ascontiguousarray(nar_offsets, dtype=np.uint64)
    n = len(offs) - 1
    cap = max(batch_capacity(offs, o.min_size), 1)
    if out is None or len(out) < cap:
        out = np.zeros(cap, DESC_DTYPE)
    first = np.zeros(n + 1, np.uint64)
    _check(lib.cg_chunk_batch(_ptr(a), offs.ctypes.data, n, o.min_size, o.avg_size, o.max_size, int(hash),
                              out.ctypes.data, len(out), first.ctypes.data))
    return out[: int(first[-1])], first


def chunk_batch_device(d_data_ptr: int, nar_offsets: np.ndarray, d_out_ptr: int, out_cap: int,
                       min_size=None, avg_size=None, max_size=None,
                       hash: HashAlgorithm = HashAlgorithm.Sha256, stream: int = 0) -> np.ndarray:
    """Device-resident batch: pointers are HIP device addresses (e.g. torch
    tensor.data_ptr()); returns nar_first (n+1) with the per-NAR descriptor starts."""
    o = ChunkingOptions.resolve(min_size, avg_size, max_size)
    offs = np.ascontiguousarray(nar_offsets, dtype=np.uint64)
    n = len(offs) - 1
    first = np.zeros(n + 1, np.uint64)
    _check(lib.cg_chunk_batch_device(ctypes.c_void_p(d_data_ptr), offs.ctypes.data, n, o.min_size,
                                     o.avg_size, o.max_size, int(hash), ctypes.c_void_p(d_out_ptr), out_cap,
                                     first.ctypes.data, ctypes.c_void_p(stream or None)))
    return first


class BatchInFlight:
    """A device batch queued by chunk_batch_device_async: wait() blocks until it is done,
    raises its error (if any) and returns nar_first.  An unwaited batch is waited for when
    collected, so its workspace always goes back to the engine's pool."""

    def __init__(self, handle: int, n_nars: int):
        self._h = handle
        self._n = n_nars

    def wait(self) -> np.ndarray:
        if self._h is None:
            raise IoError("batch already waited for")
        first = np.zeros(self._n + 1, np.uint64)
        h, self._h = self._h, None
        _check(lib.cg_batch_wait(ctypes.c_void_p(h), first.ctypes.data))
        return first

    def __del__(self):
        if getattr(self, "_h", None) is not None:
            lib.cg_batch_wait(ctypes.c_void_p(self._h), None)
            self._h = None


def chunk_batch_device_async(d_data_ptr: int, nar_offsets: np.ndarray, d_out_ptr: int, out_cap: int,
                             min_size=None, avg_size=None, max_size=None,
                             hash: HashAlgorithm = HashAlgorithm.Sha256, stream: int = 0,
                             inputs_ready: int = 0) -> BatchInFlight:
    """chunk_batch_device without the wait (cg_chunk_batch_device_async): the pipeline is
    queued on `stream` and the call returns; BatchInFlight.wait() gives nar_first.  Keeping
    the next batch queued while waiting for the current one hides the host side of every
    call behind the GPU's work.  `inputs_ready` (a hipEvent_t handle, e.g.
    torch.cuda.Event().cuda_event, recorded after the last write to the input and the last
    use of the output array) orders the batch after that event only
    (cg_chunk_batch_device_async_after): it runs on a library stream beside the batch queued
    before it, and `stream` waits for its end; 0 = after everything queued on `stream`."""
    o = ChunkingOptions.resolve(min_size, avg_size, max_size)
    offs = np.ascontiguousarray(nar_offsets, dtype=np.uint64)
    n = len(offs) - 1
    h = ctypes.c_void_p()
    _check(lib.cg_chunk_batch_device_async_after(ctypes.c_void_p(d_data_ptr), offs.ctypes.data, n, o.min_size,
                                                 o.avg_size, o.max_size, int(hash), ctypes.c_void_p(d_out_ptr),
                                                 out_cap, ctypes.c_void_p(stream or None),
                                                 ctypes.c_void_p(inputs_ready or None), ctypes.byref(h)))
    return BatchInFlight(h.value, n)


def default_depth(hash: HashAlgorithm, batch_bytes: int, hw_queues: int | None = None) -> int:
    """Batches one caller keeps in flight through the per-batch-stream path
    (BatchPipeline(group=0), cg_chunk_batch_device_async_after): SHA-256
    under 4 GiB a batch 20, from 4 GiB 4, BLAKE3 2 -- held to the hardware queues less 2
    (`hw_queues` None = the GPU_MAX_HW_QUEUES the library saw when it was loaded, which is
    what HIP applies), since every batch in flight holds a HIP stream and batches sharing a
    hardware queue run one after another.  The digest pipeline (the default) needs no such
    limit: default_group."""
    if HashAlgorithm(hash) != HashAlgorithm.Sha256:
        return 2
    hwq = int(lib.cg_hw_queues()) if hw_queues is None else int(hw_queues)
    return max(2, min(20 if batch_bytes < (4 << 30) else 4, hwq - 2))


def pipeline_create(device: int, group: int, lanes: int) -> int:
    """cg_pipeline_create: a digest pipeline handle."""
    h = ctypes.c_void_p()
    _check(lib.cg_pipeline_create(device, group, lanes, ctypes.byref(h)))
    return h.value


def pipeline_submit(p: int, d_data_ptr: int, offs: np.ndarray, d_out_ptr: int, out_cap: int, o: "ChunkingOptions",
                    hash: HashAlgorithm, inputs_ready: int = 0) -> BatchInFlight:
    """cg_pipeline_submit: one device batch into the pipeline `p`."""
    n = len(offs) - 1
    h = ctypes.c_void_p()
    _check(lib.cg_pipeline_submit(ctypes.c_void_p(p), ctypes.c_void_p(d_data_ptr), offs.ctypes.data, n, o.min_size,
                                  o.avg_size, o.max_size, int(hash), ctypes.c_void_p(d_out_ptr), out_cap,
                                  ctypes.c_void_p(inputs_ready or None), ctypes.byref(h)))
    return BatchInFlight(h.value, n)


def pipeline_flush(p: int) -> None:
    _check(lib.cg_pipeline_flush(ctypes.c_void_p(p)))


def pipeline_destroy(p: int) -> None:
    lib.cg_pipeline_destroy(ctypes.c_void_p(p))


PIPE_GROUP_BYTES = 24 << 30  # bytes of batches one merged SHA-256 digest launch takes (default_group)
PIPE_LANES = 3               # merged digests in flight (cg_pipeline_create lanes; default_lanes)


def pipeline_depth(hash: HashAlgorithm, group: int, lanes: int) -> int:
    """Batches in flight for the digest pipeline: (lanes + 1) x group for SHA-256 (every lane
    busy while the next group forms); 8 for BLAKE3, whose batches run whole on the
    pipeline's three boundary streams (profiles/r06_v42_summary.txt)."""
    if HashAlgorithm(hash) != HashAlgorithm.Sha256:
        return 8
    return (lanes + 1) * group


def default_lanes(hash: HashAlgorithm, batch_bytes: int) -> int:
    """Merged digest launches in flight: three.  (Four with two boundary streams raise config
    2's steady rate ~7 %, but their phases drift and a 20-batch window reads 0.7-1.1x of it,
    profiles/r06_v38_summary.txt; lanes= and CHUNKER_AMD_PIPE_BSTREAMS select that form.)"""
    del hash, batch_bytes
    return PIPE_LANES


def default_group(hash: HashAlgorithm, batch_bytes: int) -> int:
    """Batches per merged SHA-256 digest launch of the digest pipeline (cg_pipeline_create):
    enough 1 GiB batches to fill the chip with their chains (a config-2 batch's digest is its
    longest chunk's ~55 ms chain on ~18 workgroups), one for batches that fill it alone.
    BLAKE3: 1 (not merged)."""
    if HashAlgorithm(hash) != HashAlgorithm.Sha256:
        return 1
    b = max(int(batch_bytes), 1)
    return int(max(1, min(64, (PIPE_GROUP_BYTES + b // 2) // b)))


class BatchPipeline:
    """Device batches in flight from one thread (an ingest worker draining NAR batches):
    submit() queues a batch after its inputs-ready event only and, once `depth` are queued,
    waits for the oldest and returns it; drain() waits for the rest.  Results come back in
    submission order as (tag, nar_first).  The caller owns the buffers: a batch's input and
    output arrays must stay untouched until its result has been returned (one output array
    per batch in flight).

    The product form is the digest pipeline (cg_pipeline_*): every batch's boundary stages
    on one library stream, the SHA-256 digests of `group` consecutive batches merged into one
    launch on one of `lanes` digest streams, each batch completing when its own chunks are
    digested -- so the batches in flight need no hardware queue each.  depth None = (lanes +
    1) x group, which keeps every lane busy while the next group forms.  group None =
    default_group for the first batch's size; group=0 selects the round-5 per-batch-stream
    path (cg_chunk_batch_device_async_after on `stream`, depth default_depth)."""

    def __init__(self, depth: int | None = None, min_size=None, avg_size=None, max_size=None,
                 hash: HashAlgorithm = HashAlgorithm.Sha256, stream: int = 0, group: int | None = None,
                 lanes: int | None = None, device: int = -1):
        if depth is not None and depth < 1:
            raise InvalidOptionsError(f"pipeline depth must be at least 1, got {depth}")
        if group is not None and not 0 <= group <= 64:
            raise InvalidOptionsError(f"pipeline group must be in 0..=64, got {group}")
        self.depth = depth
        self.options = ChunkingOptions.resolve(min_size, avg_size, max_size)
        self.hash = HashAlgorithm(hash)
        self.stream = stream
        self.group = group
        self._lanes = lanes
        self.lanes = lanes or PIPE_LANES
        self.device = device
        self._p = None
        self._opened = False
        self._q: deque = deque()

    def _open(self, batch_bytes: int) -> None:
        self._opened = True
        if self.group is None:
            self.group = default_group(self.hash, batch_bytes)
        if not self._lanes:
            self.lanes = default_lanes(self.hash, batch_bytes)
        if self.group:
            self._p = pipeline_create(self.device, self.group, self.lanes)
            if self.depth is None:
                self.depth = pipeline_depth(self.hash, self.group, self.lanes)
        elif self.depth is None:
            self.depth = default_depth(self.hash, batch_bytes)

    def submit(self, d_data_ptr: int, nar_offsets: np.ndarray, d_out_ptr: int, out_cap: int,
               inputs_ready: int = 0, tag=None) -> list:
        offs = np.ascontiguousarray(nar_offsets, dtype=np.uint64)
        if not self._opened:
            self._open(int(offs[-1]) if len(offs) else 0)
        o = self.options
        if self._p is not None:
            b = pipeline_submit(self._p, d_data_ptr, offs, d_out_ptr, out_cap, o, self.hash, inputs_ready)
        else:
            b = chunk_batch_device_async(d_data_ptr, offs, d_out_ptr, out_cap, o.min_size, o.avg_size, o.max_size,
                                         hash=self.hash, stream=self.stream, inputs_ready=inputs_ready)
        self._q.append((tag, b))
        done = []
        while len(self._q) >= self.depth:
            t, oldest = self._q.popleft()
            done.append((t, oldest.wait()))
        return done

    def flush(self) -> None:
        """Launch the digest of the batches queued since the last group (cg_pipeline_flush)."""
        if self._p is not None:
            pipeline_flush(self._p)

    def drain(self) -> list:
        done = []
        self.flush()
        while self._q:
            t, b = self._q.popleft()
            done.append((t, b.wait()))
        return done

    def stats(self) -> dict:
        """Digest-pipeline counters (cg_pipeline_stats): merged groups and their batches, and
        -- for groups launched while cg_set_profiling was on -- the digest kernel's time."""
        if self._p is None:
            return {}
        out = (ctypes.c_double * 6)()
        _check(lib.cg_pipeline_stats(ctypes.c_void_p(self._p), out))
        return {"groups": int(out[0]), "batches": int(out[1]), "timed_groups": int(out[2]),
                "digest_ms_sum": out[3], "digest_bytes_sum": out[4], "last_digest_ms": out[5]}

    def close(self) -> None:
        """Wait for everything queued, then free the pipeline's streams."""
        try:
            while self._q:
                _, b = self._q.popleft()
                b.wait()
        finally:
            if self._p is not None:
                pipeline_destroy(self._p)
                self._p = None

    def __len__(self) -> int:
        return len(self._q)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        # wait for everything queued, whatever happened (the workspaces go back to the pool)
        try:
            self.flush()
        except ChunkingError:
            pass
        while self._q:
            _, b = self._q.popleft()
            try:
                b.wait()
            except ChunkingError:
                if exc[0] is None:
                    raise
        if self._p is not None:
            pipeline_destroy(self._p)
            self._p = None
        return False

    def __del__(self):
        if getattr(self, "_p", None) is not None:
            self._q.clear()  # (each BatchInFlight waits for itself when collected)
            pipeline_destroy(self._p)
            self._p = None


class MultiDevicePipeline:
    """One host process driving several GPUs (cg_multi_*): each step is a batch of NARs
    sharded one-file-per-GPU -- shard k already in device k's HBM -- and chunked by device
    k's digest pipeline; the descriptors are gathered into one array on devices[0] over xGMI
    peer copies, with the global NAR index on the host (north_star's 8-GPU split for the
    reference's single node-bin process).  submit()/drain() behave as BatchPipeline's: up to
    `depth` steps in flight, results (tag, nar_first) in submission order.  A device may be
    listed more than once (a rehearsal of the split on one GPU)."""

    def __init__(self, devices, min_size=None, avg_size=None, max_size=None,
                 hash: HashAlgorithm = HashAlgorithm.Sha256, group: int | None = None, lanes: int | None = None,
                 depth: int | None = None):
        if depth is not None and depth < 1:
            raise InvalidOptionsError(f"pipeline depth must be at least 1, got {depth}")
        self.devices = [int(d) for d in devices]
        self.options = ChunkingOptions.resolve(min_size, avg_size, max_size)
        self.hash = HashAlgorithm(hash)
        self.group, self.lanes, self.depth = group, lanes or PIPE_LANES, depth
        self._m = None
        self._q: deque = deque()

    def _open(self, shard_bytes: int) -> None:
        if self.group is None:
            self.group = default_group(self.hash, shard_bytes)
        if self.depth is None:
            self.depth = (self.lanes + 1) * max(self.group, 1)
        devs = (ctypes.c_int * len(self.devices))(*self.devices)
        h = ctypes.c_void_p()
        _check(lib.cg_multi_create(devs, len(self.devices), max(self.group, 1), self.lanes, ctypes.byref(h)))
        self._m = h.value

    def submit(self, shards, d_out_ptr: int, out_cap: int, inputs_ready=None, tag=None) -> list:
        """shards: one (device pointer, nar_offsets starting at 0) per device, in NAR order."""
        if len(shards) != len(self.devices):
            raise InvalidOptionsError(f"{len(shards)} shards for {len(self.devices)} devices")
        offs = [np.ascontiguousarray(o, dtype=np.uint64) for _, o in shards]
        if self._m is None:
            self._open(max(int(o[-1]) if len(o) else 0 for o in offs))
        nd = len(shards)
        d = (ctypes.c_void_p * nd)(*[ctypes.c_void_p(p) for p, _ in shards])
        op = (ctypes.c_void_p * nd)(*[ctypes.c_void_p(o.ctypes.data) for o in offs])
        nn = (ctypes.c_size_t * nd)(*[len(o) - 1 for o in offs])
        ev = (ctypes.c_void_p * nd)(*[ctypes.c_void_p(e or None) for e in (inputs_ready or [0] * nd)])
        o = self.options
        h = ctypes.c_void_p()
        _check(lib.cg_multi_submit(ctypes.c_void_p(self._m), d, op, nn, o.min_size, o.avg_size, o.max_size,
                                   int(self.hash), ctypes.c_void_p(d_out_ptr), out_cap, ev, ctypes.byref(h)))
        self._q.append((tag, h.value, sum(len(x) - 1 for x in offs), offs))
        done = []
        while len(self._q) >= self.depth:
            done.append(self._wait_oldest())
        return done

    def _wait_oldest(self):
        t, h, n, _ = self._q.popleft()
        first = np.zeros(n + 1, np.uint64)
        _check(lib.cg_multi_wait(ctypes.c_void_p(h), first.ctypes.data))
        return t, first

    def drain(self) -> list:
        if self._m is not None:
            _check(lib.cg_multi_flush(ctypes.c_void_p(self._m)))
        done = []
        while self._q:
            done.append(self._wait_oldest())
        return done

    def close(self) -> None:
        try:
            while self._q:
                _, h, _, _ = self._q.popleft()
                lib.cg_multi_wait(ctypes.c_void_p(h), None)
        finally:
            if self._m is not None:
                lib.cg_multi_destroy(ctypes.c_void_p(self._m))
                self._m = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __del__(self):
        if getattr(self, "_m", None) is not None:
            self.close()


def batch_capacity(nar_offsets: np.ndarray, min_size=None) -> int:
    m = DEFAULT_MIN if min_size is None else int(min_size)
    lens = np.diff(np.asarray(nar_offsets, dtype=np.uint64))
    return int(sum(lib.cg_capacity(int(x), m) for x in lens))


# ---------------------------------------------------------------------------
# streaming
# ---------------------------------------------------------------------------
class PushChunker:
    """PushChunker (src/chunking.rs:753-829): feed slices, get the chunks whose
    content-defined boundaries are now final (with payloads)."""

    def __init__(self, min_size=None, avg_size=None, max_size=None,
                 hash: HashAlgorithm = HashAlgorithm.Sha256):
        self.options = ChunkingOptions.resolve(min_size, avg_size, max_size)
        self.hash = HashAlgorithm(hash)
        st = ctypes.c_int(0)
        o = self.options
        self._h = lib.cg_push_new(o.min_size, o.avg_size, o.max_size, int(self.hash), ctypes.byref(st))
        if not self._h:
            _raise(st.value)
        # payload bookkeeping (the engine returns descriptors; payloads are sliced here
        # from the pushed slices, which are kept by reference: one copy per payload byte)
        self._segs: list[tuple[int, memoryview]] = []  # (stream offset, bytes) not yet emitted
        self._pushed = 0

    def _payload(self, off: int, ln: int) -> bytes:
        parts = []
        for start, mv in self._segs:
            lo, hi = max(off, start), min(off + ln, start + len(mv))
            if lo < hi:
                parts.append(mv[lo - start:hi - start])
        return b"".join(parts)

    def _collect(self, arr: np.ndarray) -> list[ChunkMetadata]:
        out = [ChunkMetadata(bytes(d["hash"]), int(d["offset"]), int(d["length"]),
                             self._payload(int(d["offset"]), int(d["length"]))) for d in arr]
        for c in out:  # drain_finalized_chunks records per emitted chunk (:613-616, :655-658)
            metrics.record(c.length)
        if len(arr):
            end = int(arr[-1]["offset"] + arr[-1]["length"])
            self._segs = [(st, mv) for st, mv in self._segs if st + len(mv) > end]
        return out

    def push(self, data) -> list[ChunkMetadata]:
        a = _as_u8(data)
        cap = lib.cg_push_out_capacity(self._h, len(a))
        out = np.zeros(max(cap, 1), DESC_DTYPE)
        n = ctypes.c_size_t(0)
        st = lib.cg_push_push(self._h, _ptr(a), len(a), out.ctypes.data, len(out), ctypes.byref(n))
        _check(st)
        # immutable input is kept by reference, anything else is copied once
        keep = data if isinstance(data, bytes) else a.tobytes()
        if len(keep):
            self._segs.append((self._pushed, memoryview(keep)))
            self._pushed += len(keep)
        return self._collect(out[: n.value])

    def finish(self) -> list[ChunkMetadata]:
        cap = lib.cg_push_out_capacity(self._h, 0)
        out = np.zeros(max(cap, 1), DESC_DTYPE)
        n = ctypes.c_size_t(0)
        _check(lib.cg_push_finish(self._h, out.ctypes.data, len(out), ctypes.byref(n)))
        return self._collect(out[: n.value])

    def bytes_consumed(self) -> int:
        return int(lib.cg_push_bytes_consumed(self._h))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.cg_push_free(h)
            self._h = None


_USIZE_MAX = 2 ** 64 - 1


def _parse_usize(s: str | None) -> int | None:
    """Rust's `s.parse::<usize>().ok()`: ASCII decimal digits with an optional leading '+',
    no whitespace, no '-', no '_', at most usize::MAX; anything else is None."""
    if not s:
        return None
    body = s[1:] if s[0] == "+" else s
    if not body or not all("0" <= ch <= "9" for ch in body):
        return None
    v = int(body)
    return v if v <= _USIZE_MAX else None


def effective_read_slice_cap() -> int:
    """src/chunking.rs:427-433."""
    v = _parse_usize(os.environ.get("CHUNKER_READ_SLICE_CAP_BYTES"))
    if v is not None and MIN_READ_SLICE_CAP <= v <= MAX_READ_SLICE_CAP:
        return v
    return DEFAULT_READ_SLICE_CAP


def stream_read_size(max_size: int) -> int:
    """Read size per refill, src/chunking.rs:713-716:
    max(min(max(max_size * 8, 4 MiB), cap), 4096), cap = CHUNKER_READ_SLICE_CAP_BYTES
    (default 8 MiB)."""
    target = max(max_size * 8, 4 * 1024 * 1024)
    return max(min(target, effective_read_slice_cap()), MIN_READ_SLICE_CAP)


DEFAULT_STREAM_INFLIGHT = 2048 * 1024 * 1024


def stream_inflight_bytes() -> int:
    """HBM the engine may hold for one ChunkStream's slices in flight (cg_stream_new):
    CHUNKER_AMD_STREAM_INFLIGHT_BYTES, default 2 GiB (the engine's own default).  The
    host keeps the same slices alive until their chunks are emitted (payloads are
    slices of them)."""
    v = _parse_usize(os.environ.get("CHUNKER_AMD_STREAM_INFLIGHT_BYTES"))
    return v if v else DEFAULT_STREAM_INFLIGHT


class StreamMetrics:
    """The reference's streaming metrics (src/chunking.rs:398-416): counters
    `chunker.chunks_emitted` and `chunker.bytes_processed` and histogram
    `chunker.chunk_size`, recorded per chunk handed out by the streaming paths --
    PushChunker / ChunkStream (:613-616, :655-658) and ChunkStreamAsync (:926-929,
    :962-965) -- and not by chunk_data, as in the reference.  The histogram keeps count,
    sum, min and max.  `snapshot()` returns them by the reference's metric names."""

    def __init__(self):
        import threading

        self._mu = threading.Lock()
        self.reset()

    def reset(self) -> None:
        self.chunks_emitted = 0
        self.bytes_processed = 0
        self._hist = [0, 0, None, None]  # count, sum, min, max

    def record(self, length: int) -> None:
        with self._mu:
            self.chunks_emitted += 1
            self.bytes_processed += length
            h = self._hist
            h[0] += 1
            h[1] += length
            h[2] = length if h[2] is None else min(h[2], length)
            h[3] = length if h[3] is None else max(h[3], length)

    def snapshot(self) -> dict:
        with self._mu:
            c, sm, lo, hi = self._hist
            return {"chunker.chunks_emitted": self.chunks_emitted, "chunker.bytes_processed": self.bytes_processed,
                    "chunker.chunk_size": {"count": c, "sum": sm, "min": lo, "max": hi}}


metrics = StreamMetrics()


class _StreamCore:
    """What ChunkStream and ChunkStreamAsync share: the engine's pipelined stream handle
    (cg_stream_*), the read slices kept for payloads, and the failure rule -- the first
    engine error poisons the handle (the C side repeats it on every later call) and the
    stream ends, so no chunk after a lost slice is ever handed out.

    Payloads are read-only memoryviews (the reference's `Bytes`): a view into the slice
    the chunk was read in, or, for a chunk spanning slices, into one joined copy.  A view
    keeps its slice alive (at most one read size); bytes(payload) makes an owned copy."""

    def _open(self, read_size: int) -> None:
        st = ctypes.c_int(0)
        o = self.options
        self._h = lib.cg_stream_new(o.min_size, o.avg_size, o.max_size, int(self.hash), read_size,
                                    stream_inflight_bytes(), ctypes.byref(st))
        if not self._h:
            _raise(st.value)
        self._segs: deque = deque()  # (stream offset, read-only memoryview) not yet fully emitted
        self._pushed = 0
        self._pending: deque = deque()
        self._eof = False
        self._done = False
        self._out = np.zeros(4096, DESC_DTYPE)

    def _engine(self, status: int) -> None:
        """_check for engine calls: on failure the stream is over (handle freed)."""
        if status != _lib.CG_OK:
            try:
                _raise(status)
            finally:
                self._done = True
                self._release()

    def _take(self, wait: bool) -> int:
        n = ctypes.c_size_t(0)
        self._engine(lib.cg_stream_take(self._h, self._out.ctypes.data, len(self._out), ctypes.byref(n), int(wait)))
        for d in self._out[: n.value]:
            off, ln = int(d["offset"]), int(d["length"])
            self._pending.append(ChunkMetadata(bytes(d["hash"]), off, ln, self._payload(off, ln)))
        if n.value:  # drop slices wholly before the last emitted byte
            end = self._pending[-1].offset + self._pending[-1].length
            while self._segs and self._segs[0][0] + len(self._segs[0][1]) <= end:
                self._segs.popleft()
        return n.value

    def _push(self, buf) -> None:
        a = _as_u8(buf)
        self._engine(lib.cg_stream_push(self._h, _ptr(a), len(a)))
        # payloads are views of what was read: keep immutable buffers as they are
        # (bytes, read-only views), copy anything the reader might reuse
        keep = buf if isinstance(buf, bytes) or (isinstance(buf, memoryview) and buf.readonly) else a.tobytes()
        mv = memoryview(keep).cast("B")
        self._segs.append((self._pushed, mv.toreadonly()))
        self._pushed += len(mv)

    def _finish(self) -> None:
        self._engine(lib.cg_stream_finish(self._h))
        self._eof = True

    def _drained(self) -> bool:
        """At EOF: nothing left in the engine -> the stream is done (handle freed now,
        not at garbage collection)."""
        if lib.cg_stream_pending(self._h) == 0:
            self._done = True
            self._release()
            return True
        return False

    def _payload(self, off: int, ln: int) -> memoryview:
        parts = []
        for start, mv in self._segs:
            if start >= off + ln:
                break
            lo, hi = max(off, start), min(off + ln, start + len(mv))
            if lo < hi:
                parts.append(mv[lo - start:hi - start])
        # one slice: a zero-copy view of the bytes read (the reference's Bytes::split_to,
        # src/chunking.rs:592); a chunk spanning slices is joined once
        return parts[0] if len(parts) == 1 else memoryview(b"".join(parts))

    def _emit(self) -> ChunkMetadata:
        c = self._pending.popleft()
        metrics.record(c.length)
        return c

    def bytes_consumed(self) -> int:
        return self._pushed

    def _release(self) -> None:
        h = getattr(self, "_h", None)
        if h:
            lib.cg_stream_free(h)
            self._h = None


class ChunkStream(_StreamCore):
    """ChunkStream (src/chunking.rs:382-740): pull chunks from a binary reader.

    Reads slices of the reference's size (stream_read_size) and pushes them into the
    engine's pipelined stream handle (cg_stream_*): cut points are found per slice, the
    digests of many slices run concurrently on the GPU, and chunks come back strictly in
    stream order with the reference's (offset, length, hash).  One slice is read ahead
    on a helper thread while the engine works (the ctypes calls release the GIL).  A
    reader error raises IoError and the next call reads again (as the reference's
    ChunkStream::next does); an engine error ends the stream."""

    def __init__(self, reader: BinaryIO, min_size=None, avg_size=None, max_size=None,
                 hash: HashAlgorithm = HashAlgorithm.Sha256):
        self._reader = reader
        self.options = ChunkingOptions.resolve(min_size, avg_size, max_size)
        self.hash = HashAlgorithm(hash)
        self._slice = stream_read_size(self.options.max_size)
        self._pool = None
        self._next = None
        self._open(self._slice)

    @classmethod
    def new_with_hash(cls, reader, min_size, avg_size, max_size, hash):
        return cls(reader, min_size, avg_size, max_size, hash)

    def _read_async(self):
        from concurrent.futures import ThreadPoolExecutor

        if self._pool is None:
            self._pool = ThreadPoolExecutor(1, thread_name_prefix="chunk-stream-read")
        self._next = self._pool.submit(self._reader.read, self._slice)

    def _close_pool(self):
        if self._pool is not None:
            self._pool.shutdown(wait=True)
            self._pool = None

    def _release(self) -> None:
        super()._release()
        pool = getattr(self, "_pool", None)
        if pool is not None:
            pool.shutdown(wait=False)
            self._pool = None

    def __iter__(self) -> Iterator[ChunkMetadata]:
        return self

    def __next__(self) -> ChunkMetadata:
        while True:
            if self._pending:
                return self._emit()
            if self._done:
                raise StopIteration
            if self._eof:
                if self._take(True) == 0:
                    self._drained()
                continue
            if self._take(False):
                continue
            if self._next is None:
                self._read_async()
            try:
                buf = self._next.result()
            except OSError as e:
                # the failed read is consumed: a later next() reads again (as the
                # reference's ChunkStream::next does after an Io error)
                self._next = None
                raise IoError(str(e)) from e
            if not buf:
                self._next = None
                self._close_pool()
                self._finish()
                continue
            self._read_async()
            self._push(buf)

    def __del__(self):
        self._release()


def effective_async_buffer_limit() -> int:
    """src/chunking.rs:435-445: CHUNKER_ASYNC_BUFFER_LIMIT_BYTES (default 2 GiB), clamped
    to 64 MiB..3 GiB; a value usize's parser rejects ('-1', ' 5 ', '1_000') means the default."""
    v = _parse_usize(os.environ.get("CHUNKER_ASYNC_BUFFER_LIMIT_BYTES"))
    if v is None:
        v = DEFAULT_ASYNC_BUFFER_LIMIT
    return min(max(v, MIN_ASYNC_BUFFER_LIMIT), MAX_ASYNC_BUFFER_LIMIT)


class ChunkStreamAsync(_StreamCore):
    """ChunkStreamAsync (src/chunking.rs:835-1017, feature `async-stream`) for asyncio:

        async for chunk in ChunkStreamAsync(reader, min_size, avg_size, max_size): ...

    `reader` is any object with a coroutine `read(n)` (asyncio.StreamReader, an async
    file).  It reads max(min(max_size, CHUNKER_READ_SLICE_CAP_BYTES), 4096) bytes per
    refill (:981-986) and yields the chunks the reference's try_stream! yields -- its
    rule of emitting the buffer's first FastCDC chunk when `len != buffer.len() || eof ||
    len >= max_size` (:923) gives exactly the eager chunk sequence, which is what the
    engine's stream handle produces (retain rule :579-584 + EOF remainder).  The
    reference digests each chunk inline (:931); here the slices' digests run on the GPU
    while the event loop keeps reading: engine calls (which wait for the device) run on
    one helper thread per stream, in call order, off the loop.  Metrics are recorded per
    chunk as at :926-929 / :962-965.  As in try_stream!, the first error (reader or
    engine) is raised once and ends the stream."""

    def __init__(self, reader, min_size=None, avg_size=None, max_size=None,
                 hash: HashAlgorithm = HashAlgorithm.Sha256):
        self._reader = reader
        self.options = ChunkingOptions.resolve(min_size, avg_size, max_size)
        self.hash = HashAlgorithm(hash)
        self._read_size = max(min(self.options.max_size, effective_read_slice_cap()), MIN_READ_SLICE_CAP)
        self._exec = None
        self._open(self._read_size)

    @classmethod
    def new_with_hash(cls, reader, min_size, avg_size, max_size, hash):
        return cls(reader, min_size, avg_size, max_size, hash)

    async def _call(self, fn, *args):
        import asyncio
        from concurrent.futures import ThreadPoolExecutor

        if self._exec is None:
            self._exec = ThreadPoolExecutor(1, thread_name_prefix="chunk-stream-async")
        return await asyncio.get_running_loop().run_in_executor(self._exec, fn, *args)

    def _release(self) -> None:
        super()._release()
        ex = getattr(self, "_exec", None)
        if ex is not None:
            ex.shutdown(wait=False)
            self._exec = None

    def __aiter__(self):
        return self

    async def __anext__(self) -> ChunkMetadata:
        while True:
            if self._pending:
                return self._emit()
            if self._done:
                raise StopAsyncIteration
            if self._eof:
                if await self._call(self._take, True) == 0:
                    self._drained()
                continue
            if await self._call(self._take, False):
                continue
            try:
                buf = await self._reader.read(self._read_size)
            except asyncio.CancelledError:
                raise  # cancellation is not a stream error: the stream stays usable
            except Exception as e:  # noqa: BLE001 -- the first reader error ends the stream (try_stream!)
                self._done = True
                self._release()
                if isinstance(e, OSError):
                    raise IoError(str(e)) from e
                raise
            if not buf:
                await self._call(self._finish)
                continue
            await self._call(self._push, buf)

    def __del__(self):
        self._release()


async def chunk_data_async(reader, min_size=None, avg_size=None, max_size=None) -> list[ChunkMetadata]:
    """chunk_data_async (src/chunking.rs:1061-1088): collect a ChunkStreamAsync's chunks,
    raising BufferLimitExceededError once their total length passes
    effective_async_buffer_limit()."""
    limit = effective_async_buffer_limit()
    chunks, total = [], 0
    async for c in ChunkStreamAsync(reader, min_size, avg_size, max_size):
        total += c.length
        if total > limit:
            raise BufferLimitExceededError(total, limit)
        chunks.append(c)
    return chunks


async def chunk_stream_async(reader, min_size=None, avg_size=None, max_size=None) -> list[ChunkMetadata]:
    """chunk_stream_async (src/chunking.rs:1122-1130) = chunk_data_async."""
    return await chunk_data_async(reader, min_size, avg_size, max_size)


class BlockingAsyncReadAdapter:
    """BlockingAsyncReadAdapter (src/chunking.rs:1028-1047): a blocking `read(n)` over an
    async reader -- on `loop` from another thread (run_coroutine_threadsafe), or on a
    private event loop when none is given.  Blocks the calling thread, as the
    reference warns."""

    def __init__(self, inner, loop=None):
        self._inner, self._loop, self._own = inner, loop, None

    def read(self, n: int = -1) -> bytes:
        import asyncio

        if self._loop is not None:
            return asyncio.run_coroutine_threadsafe(self._inner.read(n), self._loop).result()
        if self._own is None:
            self._own = asyncio.new_event_loop()
        return self._own.run_until_complete(self._inner.read(n))


def chunk_stream_blocking_adapter(reader, min_size=None, avg_size=None, max_size=None,
                                  loop=None) -> list[ChunkMetadata]:
    """chunk_stream_blocking_adapter (src/chunking.rs:1104-1113)."""
    return chunk_stream(BlockingAsyncReadAdapter(reader, loop), min_size, avg_size, max_size)


def chunk_stream_with_hash(reader, min_size=None, avg_size=None, max_size=None,
                           hash: HashAlgorithm = HashAlgorithm.Sha256) -> list[ChunkMetadata]:
    """src/chunking.rs:1153-1166."""
    return list(ChunkStream(reader, min_size, avg_size, max_size, hash))


def chunk_stream(reader, min_size=None, avg_size=None, max_size=None) -> list[ChunkMetadata]:
    """src/chunking.rs:1139-1146."""
    return chunk_stream_with_hash(reader, min_size, avg_size, max_size, HashAlgorithm.Sha256)

"""GPU streaming paths beyond tests/streaming_chunking.rs: ChunkStreamAsync and its
helpers (src/chunking.rs:835-1130, feature async-stream) against the oracle's eager
result, the streaming metrics (:398-416, :613-616, :926-929), the payload type, and
the stream handle's failure rule (the first engine error poisons cg_stream_*; ADVICE
r2) and lazy device resources.
"""
import asyncio
import ctypes
import io

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHA, B3 = 1, 0
P = (16_384, 65_536, 262_144)


@pytest.fixture(scope="module")
def ca(gpu):
    import chunker_amd

    return chunker_amd


@pytest.fixture(scope="module")
def O():
    from oracle import oracle

    return oracle


def rand_bytes(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


class AsyncBytesReader:
    """An async reader (`await read(n)`) over bytes that returns short reads of uneven
    sizes and yields to the event loop between them, like a socket."""

    def __init__(self, data: bytes, steps=(1, 4096, 70_000, 333, 1 << 20)):
        self._d, self._pos, self._steps, self._k = data, 0, steps, 0
        self.reads = 0

    async def read(self, n=-1):
        await asyncio.sleep(0)
        step = self._steps[self._k % len(self._steps)]
        self._k += 1
        self.reads += 1
        take = len(self._d) - self._pos if n < 0 else min(n, step, len(self._d) - self._pos)
        out = self._d[self._pos:self._pos + take]
        self._pos += take
        return out


def triples(chunks):
    return [(c.offset, c.length, c.hash) for c in chunks]


def oracle_triples(O, data, params, algo):
    return [(int(r["offset"]), int(r["length"]), bytes(r["hash"]))
            for r in O.chunk_descriptors(data, *params, algo=algo, nthreads=8)]


@pytest.mark.parametrize("algo", [SHA, B3], ids=["sha256", "blake3"])
@pytest.mark.parametrize("n,params", [(3_000_017, P), (0, P), (100, P), (9_000_000, (None, None, None))],
                         ids=["ragged", "empty", "tiny", "default"])
def test_chunk_stream_async_matches_eager(ca, O, algo, n, params):
    """ChunkStreamAsync over an uneven async reader == the eager chunk sequence (the
    reference's :923 emit rule reproduces chunk_data exactly), payloads reassemble the
    input, offsets are contiguous (fuzz_targets/chunking.rs invariants)."""
    data = rand_bytes(n, 31 + n % 7)

    async def run():
        return [c async for c in ca.ChunkStreamAsync(AsyncBytesReader(data), *params, hash=algo)]

    got = asyncio.run(run())
    o = ca.ChunkingOptions.resolve(*params)
    assert triples(got) == oracle_triples(O, data, (o.min_size, o.avg_size, o.max_size), algo)
    assert b"".join(c.payload for c in got) == data
    pos = 0
    for c in got:
        assert c.offset == pos and len(c.payload) == c.length
        pos += c.length


def test_chunk_data_async_and_helpers(ca, O, monkeypatch):
    """chunk_data_async / chunk_stream_async (src/chunking.rs:1061-1130) collect the same
    chunks; the buffer limit (:1077-1082, clamp :435-445) raises BufferLimitExceeded
    with the running total; chunk_stream_blocking_adapter (:1104-1113) drives an async
    reader from blocking code."""
    data = rand_bytes(2_500_000, 5)
    want = oracle_triples(O, data, P, SHA)
    assert triples(asyncio.run(ca.chunk_data_async(AsyncBytesReader(data), *P))) == want
    assert triples(asyncio.run(ca.chunk_stream_async(AsyncBytesReader(data), *P))) == want
    assert triples(ca.chunk_stream_blocking_adapter(AsyncBytesReader(data), *P)) == want
    # 64 MiB is the clamp floor: 70 MiB of input passes it part-way
    big = rand_bytes(70 << 20, 6)
    monkeypatch.setenv("CHUNKER_ASYNC_BUFFER_LIMIT_BYTES", "1")
    with pytest.raises(ca.BufferLimitExceededError) as ei:
        asyncio.run(ca.chunk_data_async(AsyncBytesReader(big, steps=(8 << 20,)), *P))
    assert ei.value.limit == 64 << 20 and ei.value.attempted > ei.value.limit


class FailingAsyncReader(AsyncBytesReader):
    """Reads `ok` bytes, then raises `exc` on every later read."""

    def __init__(self, data, ok, exc):
        super().__init__(data, steps=(65536,))
        self._ok, self._exc = ok, exc

    async def read(self, n=-1):
        if self._pos >= self._ok:
            self.reads += 1
            raise self._exc
        return await super().read(min(n, self._ok - self._pos) if n >= 0 else self._ok - self._pos)


@pytest.mark.parametrize("exc,want", [(ConnectionResetError("peer reset"), "IoError"),
                                      (asyncio.IncompleteReadError(b"", 10), "IncompleteReadError"),
                                      (ValueError("bad frame"), "ValueError")],
                         ids=["oserror", "incomplete_read", "valueerror"])
def test_chunk_stream_async_first_reader_error_ends_stream(ca, exc, want):
    """the first reader error of any kind ends ChunkStreamAsync (try_stream!
    stops at the first Err, src/chunking.rs:987-998): an OSError surfaces as IoError, any
    other exception as itself; the next iteration ends the stream instead of reading again."""
    data = rand_bytes(1_000_000, 44)
    rd = FailingAsyncReader(data, 300_000, exc)

    async def run():
        s = ca.ChunkStreamAsync(rd, *P)
        got = []
        with pytest.raises(Exception) as ei:
            async for c in s:
                got.append(c)
        reads = rd.reads
        rest = [c async for c in s]
        return ei.value, got, rest, reads

    err, got, rest, reads = asyncio.run(run())
    assert type(err).__name__ == want
    assert rest == [] and rd.reads == reads  # ended: no further read
    assert sum(c.length for c in got) <= 300_000


def test_stream_metrics_recorded_by_streaming_paths_only(ca):
    """chunker.chunks_emitted / bytes_processed / chunk_size are recorded per chunk by
    PushChunker, ChunkStream and ChunkStreamAsync, and not by chunk_data (as in the
    reference: :613-616, :655-658, :926-929, :962-965 only)."""
    data = rand_bytes(1_200_000, 8)
    m = ca.metrics
    m.reset()
    ref = ca.chunk_data(data, *P)
    assert m.snapshot()["chunker.chunks_emitted"] == 0
    list(ca.ChunkStream(io.BytesIO(data), *P))
    pc = ca.PushChunker(*P)
    pc.push(data)
    pc.finish()

    async def run():
        return [c async for c in ca.ChunkStreamAsync(AsyncBytesReader(data), *P)]

    asyncio.run(run())
    snap = m.snapshot()
    assert snap["chunker.chunks_emitted"] == 3 * len(ref)
    assert snap["chunker.bytes_processed"] == 3 * len(data)
    h = snap["chunker.chunk_size"]
    assert h["count"] == 3 * len(ref) and h["max"] == max(c.length for c in ref)


def test_stream_payloads_are_readonly_views(ca):
    """ChunkStream payloads have one type: a read-only memoryview, whether
    the chunk lies in one read slice or spans two."""
    data = rand_bytes(9_000_000, 12)  # three read slices of stream_read_size(256 KiB) = 4 MiB
    got = list(ca.ChunkStream(io.BytesIO(data), *P))
    slice_size = ca.chunking.stream_read_size(P[2])
    spans = [c for c in got if c.offset // slice_size != (c.offset + c.length - 1) // slice_size]
    inside = [c for c in got if c not in spans]
    assert spans and inside
    for c in got:
        assert isinstance(c.payload, memoryview) and c.payload.readonly
        assert c.payload == data[c.offset:c.offset + c.length]


def test_stream_engine_error_poisons_handle(ca):
    """after the first engine error (here the SHA-256 spin guard, forced) the
    stream handle repeats that failure on every later push / finish / take, even with
    the cause gone, instead of continuing with a slice missing; the Python ChunkStream
    raises once and then ends."""
    data = rand_bytes(4_000_000, 3)
    st = ctypes.c_int(0)
    h = ca.lib.cg_stream_new(*P, SHA, 1 << 20, 16 << 20, ctypes.byref(st))
    assert h and st.value == 0
    out = np.zeros(4096, ca.DESC_DTYPE)
    n = ctypes.c_size_t(0)
    a = np.frombuffer(data, np.uint8)
    old = ca.lib.cg_test_sha_spin_limit(0)
    try:
        rc = 0
        for k in range(0, len(a), 1 << 20):
            rc = rc or ca.lib.cg_stream_push(h, a[k:].ctypes.data, min(1 << 20, len(a) - k))
        rc = rc or ca.lib.cg_stream_finish(h)
        rc = rc or ca.lib.cg_stream_take(h, out.ctypes.data, len(out), ctypes.byref(n), 1)
        assert rc == 2, rc  # CG_E_IO: a digest group hit the spin guard
    finally:
        ca.lib.cg_test_sha_spin_limit(old)
    for call in (lambda: ca.lib.cg_stream_push(h, a.ctypes.data, 1000),
                 lambda: ca.lib.cg_stream_finish(h),
                 lambda: ca.lib.cg_stream_take(h, out.ctypes.data, len(out), ctypes.byref(n), 1)):
        assert call() == 2
        assert "stream failed earlier" in ca._lib.last_error()
    ca.lib.cg_stream_free(h)

    s = ca.ChunkStream(io.BytesIO(data), *P)
    old = ca.lib.cg_test_sha_spin_limit(0)
    try:
        with pytest.raises(ca.IoError):
            list(s)
    finally:
        ca.lib.cg_test_sha_spin_limit(old)
    assert list(s) == []  # ended, not resumed with a hole


def test_stream_failed_arena_allocation_poisons_handle(ca):
    """The arena is allocated at the first push (lazily, two slots): when that
    allocation fails the push reports BufferLimitExceeded, and so does every later call
    on the handle."""
    st = ctypes.c_int(0)
    h = ca.lib.cg_stream_new(*P, SHA, 1 << 20, 64 << 20, ctypes.byref(st))
    assert h and st.value == 0
    a = np.frombuffer(rand_bytes(300_000, 4), np.uint8)
    ca.lib.cg_test_fail_alloc(1)
    try:
        assert ca.lib.cg_stream_push(h, a.ctypes.data, len(a)) == 5
    finally:
        ca.lib.cg_test_fail_alloc(0)
    stt, attempted, limit, _ = ca._lib.last_error_detail()
    assert stt == 5 and attempted > 0
    assert ca.lib.cg_stream_push(h, a.ctypes.data, len(a)) == 5
    assert ca._lib.last_error_detail()[1:3] == (attempted, limit)
    assert ca.lib.cg_stream_finish(h) == 5
    ca.lib.cg_stream_free(h)


def test_short_stream_takes_little_device_memory(ca, O):
    """a 1 KB stream no longer reserves the whole in-flight budget (2 GiB by
    default) -- its arena is two slots -- and a long stream still grows to the budget
    and stays exact."""
    import torch

    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    streams = [ca.ChunkStream(io.BytesIO(rand_bytes(1000, k)), *P) for k in range(4)]
    firsts = [next(s) for s in streams]
    free1, _ = torch.cuda.mem_get_info()
    assert free0 - free1 < 4 * (64 << 20), (free0 - free1) >> 20
    assert all(f.length == 1000 for f in firsts)
    del streams
    data = rand_bytes(40_000_000, 9)
    got = list(ca.ChunkStream(io.BytesIO(data), *P))
    assert triples(got) == oracle_triples(O, data, P, SHA)


@pytest.mark.parametrize("algo", [SHA, B3], ids=["sha256", "blake3"])
@pytest.mark.parametrize("shape", [(0, 1, 0), (1, 2, 0), (1, 0, 1), (0, 0, 0)],
                         ids=["one-lane", "two-lanes-small-groups", "eager", "built-in"])
def test_stream_shapes_match_eager(ca, O, monkeypatch, algo, shape):
    """The stream handle's pipeline shape (group size cap, digest lanes, launching a group
    whenever a lane is idle; test hooks) changes only timing: with a 24 MiB budget the
    arena grows, slots are reused and lanes wait for each other, and the chunks stay the
    eager sequence."""
    small_groups, lanes, eager = shape
    monkeypatch.setenv("CHUNKER_AMD_STREAM_INFLIGHT_BYTES", str(24 << 20))
    data = rand_bytes(40_000_003, 17 + algo)
    old = (ca.lib.cg_test_stream_group_cap(1 if small_groups else 0), ca.lib.cg_test_stream_max_lanes(lanes),
           ca.lib.cg_test_stream_eager(eager))
    try:
        got = list(ca.ChunkStream(io.BytesIO(data), *P, hash=algo))
    finally:
        ca.lib.cg_test_stream_group_cap(old[0])
        ca.lib.cg_test_stream_max_lanes(old[1])
        ca.lib.cg_test_stream_eager(old[2])
    assert triples(got) == oracle_triples(O, data, P, algo)

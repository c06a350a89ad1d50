"""Host-side mirror logic that needs no GPU: the async-stream configuration
(src/chunking.rs:417-445), the streaming metrics (:398-416), and the async adapters'
plumbing (errors surface before any engine call)."""
import asyncio

import pytest

import chunker_amd as ca
from chunker_amd import chunking


def test_async_buffer_limit_clamp(monkeypatch):
    """effective_async_buffer_limit (src/chunking.rs:435-445): default 2 GiB, clamped to
    64 MiB..3 GiB, unparsable -> default."""
    monkeypatch.delenv("CHUNKER_ASYNC_BUFFER_LIMIT_BYTES", raising=False)
    assert chunking.effective_async_buffer_limit() == 2 << 30
    for v, want in (("1", 64 << 20), (str(100 << 20), 100 << 20), (str(1 << 40), 3 << 30), ("x", 2 << 30),
                    # usize's parser: '+' accepted; '-', whitespace, '_' and overflow rejected -> default
                    ("+100000000", 100000000), ("-1", 2 << 30), (" 5 ", 2 << 30), ("1_000", 2 << 30),
                    (str(1 << 64), 2 << 30), ("\u0665", 2 << 30)):
        monkeypatch.setenv("CHUNKER_ASYNC_BUFFER_LIMIT_BYTES", v)
        assert chunking.effective_async_buffer_limit() == want, v


def test_read_sizes(monkeypatch):
    """ChunkStream reads max(min(max(max*8, 4 MiB), cap), 4096) (:713-716);
    ChunkStreamAsync max(min(max, cap), 4096) (:982-983); cap from
    CHUNKER_READ_SLICE_CAP_BYTES in 4 KiB..256 MiB, else 8 MiB (:427-433)."""
    monkeypatch.delenv("CHUNKER_READ_SLICE_CAP_BYTES", raising=False)
    assert chunking.stream_read_size(4 << 20) == 8 << 20
    assert chunking.stream_read_size(1024) == 4 << 20
    monkeypatch.setenv("CHUNKER_READ_SLICE_CAP_BYTES", "65536")
    assert chunking.stream_read_size(4 << 20) == 65536
    monkeypatch.setenv("CHUNKER_READ_SLICE_CAP_BYTES", "100")  # out of range -> default
    assert chunking.effective_read_slice_cap() == 8 << 20


def test_stream_metrics_counters():
    m = chunking.StreamMetrics()
    assert m.snapshot()["chunker.chunk_size"]["count"] == 0
    for n in (5, 1, 9):
        m.record(n)
    s = m.snapshot()
    assert s["chunker.chunks_emitted"] == 3 and s["chunker.bytes_processed"] == 15
    assert s["chunker.chunk_size"] == {"count": 3, "sum": 15, "min": 1, "max": 9}
    m.reset()
    assert m.snapshot()["chunker.chunks_emitted"] == 0


def test_async_invalid_options_raise_before_the_engine():
    """ChunkStreamAsync::new_with_hash resolves the options first (:880): bad sizes raise
    InvalidOptions with the reference's message, no device needed."""
    class R:
        async def read(self, n):
            return b""

    with pytest.raises(ca.InvalidOptionsError, match="min_size must be in 64..=1048576, got 32"):
        ca.ChunkStreamAsync(R(), 32, 256, 1024)
    with pytest.raises(ca.InvalidOptionsError):
        asyncio.run(ca.chunk_data_async(R(), 1024, 512, 4096))


def test_blocking_adapter_reads_through_private_loop():
    class R:
        def __init__(self):
            self.n = 0

        async def read(self, n):
            await asyncio.sleep(0)
            self.n += 1
            return b"ab"[: n]

    r = R()
    a = chunking.BlockingAsyncReadAdapter(r)
    assert a.read(1) == b"a" and a.read(5) == b"ab" and r.n == 2


def test_bench_cli_contract():
    """bench.py's command line (the driver's `--gpus N --steps K --warmup W`, the A/B flags
    the round-5 measurements use) parses without touching a GPU, and the help lists them."""
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--help"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    for flag in ("--gpus", "--steps", "--warmup", "--config", "--no-overlap", "--split-mode", "--drop-in",
                 "--drop-in-sizes", "--no-coalesce", "--dist-force", "--depth"):
        assert flag in r.stdout, flag


def test_bench_timed_group():
    """bench.py's group: the divisor of --steps nearest the library default, so the timed
    steps are whole merged groups."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import bench

    assert bench.timed_group(24, 20) == 20 and bench.timed_group(24, 48) == 24 and bench.timed_group(24, 5) == 5
    assert bench.timed_group(1, 20) == 1 and bench.timed_group(24, 96) == 24 and bench.timed_group(16, 20) == 20


def test_default_depth_and_group():
    """Per-batch-stream path (group=0): 20 batches in flight for sub-4-GiB SHA-256 batches,
    4 from 4 GiB, 2 for BLAKE3, never more than the hardware queues less 2 (each batch in
    flight holds a stream of its own); the queue count defaults to what the library saw at
    load (cg_hw_queues), not the environment's current value.  Digest pipeline: 16 GiB of
    batches per merged SHA-256 launch (1 GiB -> 24, 16 GiB -> 2), BLAKE3 unmerged."""
    G = 1 << 30
    dd = chunking.default_depth
    assert dd(1, G, 22) == 20 and dd(1, G, 32) == 20 and dd(1, G, 16) == 14
    assert dd(1, 16 * G, 16) == 4 and dd(0, G, 16) == 2 and dd(1, G, 8) == 6
    assert dd(1, G, 4) == 2 and dd(1, 16 * G, 4) == 2
    assert dd(1, G) == dd(1, G, ca.lib.cg_hw_queues())
    dg = chunking.default_group
    assert dg(1, G) == 24 and dg(1, 4 * G) == 6 and dg(1, 16 * G) == 2 and dg(1, 64 << 20) == 64
    assert dg(1, 32 * G) == 1
    assert dg(0, G) == 1
    # lanes: three (four with two boundary streams only as an A/B)
    dl = chunking.default_lanes
    assert dl(1, G) == 3 and dl(1, 16 * G) == 3 and dl(0, G) == 3


def test_batch_pipeline_order_depth_and_drain(monkeypatch):
    """BatchPipeline's host logic with the engine call replaced: at most `depth` batches
    queued, results in submission order, drain() empties it, the context exit waits for
    whatever is left (and re-raises a batch's error only when nothing else is raising),
    and the default depth follows default_depth for the first batch's size."""
    import numpy as np

    log = []

    class FakeBatch:
        def __init__(self, k, fail=False):
            self.k, self.fail = k, fail

        def wait(self):
            log.append(("wait", self.k))
            if self.fail:
                raise ca.IoError("boom")
            return np.array([0, self.k], np.uint64)

    issued = []

    def fake_async(d_data, offs, d_out, cap, mn, avg, mx, hash=None, stream=0, inputs_ready=0):
        k = len(issued)
        issued.append((d_data, inputs_ready))
        log.append(("issue", k))
        return FakeBatch(k, fail=(d_data == 666))

    monkeypatch.setattr(chunking, "chunk_batch_device_async", fake_async)
    offs = np.array([0, 1 << 20], np.uint64)
    with chunking.BatchPipeline(3, group=0) as p:
        got = []
        for k in range(7):
            got += p.submit(1, offs, 2, 3, inputs_ready=9, tag=f"b{k}")
            assert len(p) <= 2
        got += p.drain()
        assert len(p) == 0
    assert [t for t, _ in got] == [f"b{k}" for k in range(7)]
    assert [int(f[1]) for _, f in got] == list(range(7))
    # batch k is waited for only after batch k + 2 was issued (depth 3)
    assert log.index(("wait", 0)) > log.index(("issue", 2))
    assert all(r == 9 for _, r in issued)
    # a failing batch raises from submit/drain; leaving the context waits for the rest
    issued.clear()
    log.clear()
    with pytest.raises(ca.IoError):
        with chunking.BatchPipeline(2, group=0) as p:
            p.submit(666, offs, 2, 3)
            p.submit(1, offs, 2, 3)  # waits for the failing first batch -> raises
    assert ("wait", 1) in log  # the context exit still waited for the second one
    monkeypatch.setattr(chunking.lib, "cg_hw_queues", lambda: 22)
    p = chunking.BatchPipeline(group=0)
    p.submit(1, offs, 2, 3)
    assert p.depth == 20
    p.drain()
    with pytest.raises(ca.InvalidOptionsError):
        chunking.BatchPipeline(0)
    with pytest.raises(ca.InvalidOptionsError):
        chunking.BatchPipeline(group=65)


def test_batch_pipeline_digest_pipeline_host_logic(monkeypatch):
    """BatchPipeline over the digest pipeline (cg_pipeline_*) with the engine calls
    replaced: one pipeline created at the first submit with default_group / the lanes,
    depth (lanes + 1) x group by default, every batch submitted to it in order with its
    inputs-ready event, results in submission order, drain() flushes the open group before
    waiting, and leaving the context destroys the pipeline after every wait."""
    import numpy as np

    log = []

    class FakeBatch:
        def __init__(self, k):
            self.k = k

        def wait(self):
            log.append(("wait", self.k))
            return np.array([0, self.k], np.uint64)

    monkeypatch.setattr(chunking, "pipeline_create", lambda dev, g, l: log.append(("create", dev, g, l)) or 77)
    monkeypatch.setattr(chunking, "pipeline_flush", lambda p: log.append(("flush", p)))
    monkeypatch.setattr(chunking, "pipeline_destroy", lambda p: log.append(("destroy", p)))
    sub = []

    def fake_submit(p, d, offs, o, cap, opts, hash, ready=0):
        assert p == 77
        sub.append((d, ready))
        log.append(("submit", len(sub) - 1))
        return FakeBatch(len(sub) - 1)

    monkeypatch.setattr(chunking, "pipeline_submit", fake_submit)
    offs = np.array([0, 1 << 30], np.uint64)  # 1 GiB batches: default group 24
    with chunking.BatchPipeline(lanes=2) as p:
        got = []
        for k in range(80):
            got += p.submit(k, offs, 2, 3, inputs_ready=9, tag=k)
        assert p.group == 24 and p.depth == 72 and len(p) == 71
        got += p.drain()
    assert log[0] == ("create", -1, 24, 2)
    assert [t for t, _ in got] == list(range(80))
    assert all(r == 9 for _, r in sub) and [d for d, _ in sub] == list(range(80))
    assert log.index(("flush", 77)) < log.index(("wait", 9))  # drain flushes first
    assert log[-1] == ("destroy", 77)
    assert log.index(("wait", 0)) > log.index(("submit", 71))

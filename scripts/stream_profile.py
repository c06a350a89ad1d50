"""Where a ChunkStream's time goes (main thread, cProfile): one 1 GiB synthetic NAR
stream from an io.BytesIO at the reference's 8 MiB read size, SHA-256, default params.
Prints the top entries by total time, then the stream rate without the profiler."""
import os
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")  # placeholder GEAR: see tables/README.md
os.environ.pop("CHUNKER_READ_SLICE_CAP_BYTES", None)
os.environ["GPU_MAX_HW_QUEUES"] = "16"  # as bench.py
import cProfile  # noqa: E402
import io  # noqa: E402
import pstats  # noqa: E402
import sys  # noqa: E402
import time  # noqa: E402

sys.path.insert(0, ".")
import chunker_amd as ca  # noqa: E402
from chunker_amd.nar import synth_nars  # noqa: E402

N = 1 << 30
data, _ = synth_nars([N])
raw = data.tobytes()
list(ca.ChunkStream(io.BytesIO(raw[: 64 << 20])))  # warm
pr = cProfile.Profile()
pr.enable()
chunks = list(ca.ChunkStream(io.BytesIO(raw)))
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(14)
del chunks
class ViewReader:
    """A reader handing out zero-copy views of one buffer (no copy, no GIL-held memcpy)."""

    def __init__(self, b):
        self.mv, self.pos = memoryview(b), 0

    def read(self, n):
        v = self.mv[self.pos:self.pos + n]
        self.pos += len(v)
        return v


for _ in range(2):
    for name, mk in [("BytesIO", lambda: io.BytesIO(raw)), ("views", lambda: ViewReader(raw))]:
        t0 = time.perf_counter()
        chunks = list(ca.ChunkStream(mk()))
        dt = time.perf_counter() - t0
        print(f"ChunkStream/{name} {N / dt / 2**30:.3f} GiB/s ({len(chunks)} chunks)")
        del chunks

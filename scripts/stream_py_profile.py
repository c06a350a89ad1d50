"""cProfile of the Python ChunkStream over a 1 GiB synthetic NAR stream (BytesIO reader,
SHA-256, default params): where the mirror's time goes beyond the engine stream."""
import cProfile
import io
import os
import pstats
import sys
import time

os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
sys.path.insert(0, ".")
import chunker_amd as ca  # noqa: E402
from chunker_amd.nar import synth_nars  # noqa: E402

data, _ = synth_nars([1 << 30])
raw = data.tobytes()
n = sum(1 for _ in ca.chunking.ChunkStream(io.BytesIO(raw[: 64 << 20])))  # warm
t = time.perf_counter()
n = sum(1 for _ in ca.chunking.ChunkStream(io.BytesIO(raw)))
dt = time.perf_counter() - t
print(f"ChunkStream 1 GiB: {n} chunks, {dt:.3f} s, {(1 << 30) / dt / 2**30:.2f} GiB/s")
pr = cProfile.Profile()
pr.enable()
n = sum(1 for _ in ca.chunking.ChunkStream(io.BytesIO(raw)))
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)

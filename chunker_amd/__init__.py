"""chunker_amd -- MI355X (gfx950) FastCDC content-defined chunking + per-chunk
SHA-256/BLAKE3 engine, a drop-in for FlakeCache/chunker's hot path
(chunk_data / chunk_descriptors / ChunkStream / PushChunker, src/chunking.rs).

Importing this package loads the in-tree HIP library and raises if it is missing.
"""
from .chunking import (  # noqa: F401
    BoundsError, BufferLimitExceededError, ChunkDescriptor, ChunkingError, ChunkingOptions, ChunkMetadata,
    BlockingAsyncReadAdapter, ChunkStream, ChunkStreamAsync, DeviceUnavailableError, HashAlgorithm, InvalidOptionsError, IoError, PushChunker, TablesError,
    BatchInFlight, BatchPipeline, ZeroLengthChunkError, default_depth, chunk_batch, chunk_batch_device, chunk_batch_device_async, chunk_data, chunk_data_with_hash, chunk_descriptors,
    chunk_descriptors_array, chunk_descriptors_with_hash, chunk_data_async, chunk_stream, chunk_stream_async, chunk_stream_blocking_adapter,
    chunk_stream_with_hash, get_cdc_tables, metrics,
    selftest, set_cdc_tables, tables_verified,
)
from ._lib import DESC_DTYPE, lib  # noqa: F401

__all__ = [n for n in dir() if not n.startswith("_")]

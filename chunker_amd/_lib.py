"""ctypes binding of libchunker_amd.so (the C ABI in include/chunker_gpu.h).

The shared library is built in-tree (chunker_amd/libchunker_amd.so, see
chunker_amd/build.py).  If it is missing this module raises at import: the
package has no CPU fallback path.
"""
from __future__ import annotations

import ctypes
from pathlib import Path

import numpy as np

import os as _os

# CHUNKER_AMD_LIB: an alternative build of the same ABI (A/B measurements of compile-time
# variants, scripts/gpu_ab_*.sh); unset = the product library beside this file
LIB_PATH = Path(_os.environ.get("CHUNKER_AMD_LIB") or Path(__file__).resolve().parent / "libchunker_amd.so")
# diagnostics build (make -C chunker_amd/csrc diag): same ABI plus cg_diag_* kernels
DIAG_LIB_PATH = Path(__file__).resolve().parent / "libchunker_amd_diag.so"
ABI_VERSION = 3

# Opt-in that lifts the engine's fail-closed FastCDC table gate (include/chunker_gpu.h):
# with the placeholder GEAR installed every chunking call refuses to run unless it is "1".
ALLOW_PLACEHOLDER_ENV = "CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR"

CG_OK = 0
CG_E_BOUNDS = 1
CG_E_IO = 2
CG_E_ZERO_LENGTH_CHUNK = 3
CG_E_INVALID_OPTIONS = 4
CG_E_BUFFER_LIMIT = 5
CG_E_CAPACITY = 6
CG_E_NO_DEVICE = 7
CG_E_TABLES = 8

# cg_desc (48 bytes): ChunkDescriptor {offset, length, hash[32]}
DESC_DTYPE = np.dtype([("offset", "<u8"), ("length", "<u8"), ("hash", "u1", (32,))])
assert DESC_DTYPE.itemsize == 48

# every exported symbol declared in include/chunker_gpu.h
EXPORTS = (
    "cg_abi_version", "cg_last_error_message", "cg_last_error_detail", "cg_validate", "cg_capacity",
    "cg_chunk_descriptors", "cg_chunk_batch", "cg_chunk_batch_device", "cg_push_new", "cg_push_push",
    "cg_push_finish", "cg_push_bytes_consumed", "cg_push_out_capacity", "cg_push_free", "cg_hash_spans_device",
    "cg_set_cdc_tables", "cg_get_cdc_tables", "cg_set_gear_table", "cg_get_gear_table", "cg_gear_is_placeholder",
    "cg_selftest", "cg_tables_verified", "cg_set_profiling", "cg_last_stage_times", "cg_synth_nars", "cg_hash",
    "cg_cas_ids_device", "cg_cas_id", "cg_node_put_batch_device", "cg_node_put", "cg_stream_new", "cg_stream_push",
    "cg_stream_finish", "cg_stream_take", "cg_stream_pending", "cg_stream_bytes_consumed", "cg_stream_free",
    "cg_last_sha_tiers", "cg_chunk_batch_device_async", "cg_batch_wait", "cg_chunk_batch_device_async_after",
    "cg_pipeline_create", "cg_pipeline_submit", "cg_pipeline_flush", "cg_pipeline_stats", "cg_pipeline_destroy",
    "cg_batch_event", "cg_multi_create", "cg_multi_submit", "cg_multi_wait", "cg_multi_flush", "cg_multi_destroy",
)
# test hooks the product library exports beyond the header (tier caps, spin-guard limit)
TEST_HOOKS = ("cg_test_sha_quad_max", "cg_test_sha_split_max", "cg_test_sha_spin_limit", "cg_test_cas_pair_max",
              "cg_test_fail_alloc", "cg_test_sha_quad_fill", "cg_test_sha_pair_fill", "cg_test_scan_path", "cg_test_scan_kernel", "cg_test_coalesce", "cg_test_scan_grid",
              "cg_test_stream_group_cap", "cg_test_stream_max_lanes", "cg_test_stream_eager",
              "cg_test_b3_fused_plan", "cg_test_b3_packed", "cg_coalesce_stats",
              "cg_test_split_mode", "cg_test_sha_tiers", "cg_test_sha_tiers_fill", "cg_hw_queues",
              "cg_test_sha_occupancy")


def _load(path: Path = LIB_PATH) -> ctypes.CDLL:
    # PyTorch-ROCm ships its own libamdhip64 (SONAME libamdhip64.so.7) and links it as
    # "libamdhip64.so".  Loading torch first makes our DT_NEEDED libamdhip64.so.7
    # resolve to that same copy, so one process never holds two HIP runtimes.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not path.exists():
        raise ImportError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). chunker_amd has no CPU fallback.")
    L = ctypes.CDLL(str(path))
    u64, sz, p, i = ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int
    psz = ctypes.POINTER(sz)
    L.cg_abi_version.restype = ctypes.c_uint32
    L.cg_last_error_message.restype = ctypes.c_char_p
    L.cg_last_error_detail.argtypes = [p]
    L.cg_last_error_detail.restype = i
    L.cg_validate.argtypes = [u64, u64, u64, ctypes.c_char_p, sz]
    L.cg_validate.restype = i
    L.cg_capacity.argtypes = [u64, u64]
    L.cg_capacity.restype = sz
    L.cg_chunk_descriptors.argtypes = [p, u64, u64, u64, u64, i, p, sz, psz]
    L.cg_chunk_descriptors.restype = i
    L.cg_chunk_batch.argtypes = [p, p, sz, u64, u64, u64, i, p, sz, p]
    L.cg_chunk_batch.restype = i
    L.cg_chunk_batch_device.argtypes = [p, p, sz, u64, u64, u64, i, p, sz, p, p]
    L.cg_chunk_batch_device.restype = i
    L.cg_chunk_batch_device_async.argtypes = [p, p, sz, u64, u64, u64, i, p, sz, p, ctypes.POINTER(p)]
    L.cg_chunk_batch_device_async.restype = i
    L.cg_chunk_batch_device_async_after.argtypes = [p, p, sz, u64, u64, u64, i, p, sz, p, p, ctypes.POINTER(p)]
    L.cg_chunk_batch_device_async_after.restype = i
    L.cg_batch_wait.argtypes = [p, p]
    L.cg_batch_wait.restype = i
    u32_ = ctypes.c_uint32
    L.cg_pipeline_create.argtypes = [i, u32_, u32_, ctypes.POINTER(p)]
    L.cg_pipeline_create.restype = i
    L.cg_pipeline_submit.argtypes = [p, p, p, sz, u64, u64, u64, i, p, sz, p, ctypes.POINTER(p)]
    L.cg_pipeline_submit.restype = i
    L.cg_pipeline_flush.argtypes = [p]
    L.cg_pipeline_flush.restype = i
    L.cg_pipeline_stats.argtypes = [p, p]
    L.cg_pipeline_stats.restype = i
    L.cg_pipeline_destroy.argtypes = [p]
    L.cg_pipeline_destroy.restype = None
    L.cg_batch_event.argtypes = [p, ctypes.POINTER(p)]
    L.cg_batch_event.restype = i
    L.cg_multi_create.argtypes = [p, sz, u32_, u32_, ctypes.POINTER(p)]
    L.cg_multi_create.restype = i
    L.cg_multi_submit.argtypes = [p, p, p, p, u64, u64, u64, i, p, sz, p, ctypes.POINTER(p)]
    L.cg_multi_submit.restype = i
    L.cg_multi_wait.argtypes = [p, p]
    L.cg_multi_wait.restype = i
    L.cg_multi_flush.argtypes = [p]
    L.cg_multi_flush.restype = i
    L.cg_multi_destroy.argtypes = [p]
    L.cg_multi_destroy.restype = None
    L.cg_push_new.argtypes = [u64, u64, u64, i, ctypes.POINTER(i)]
    L.cg_push_new.restype = p
    L.cg_push_push.argtypes = [p, p, u64, p, sz, psz]
    L.cg_push_push.restype = i
    L.cg_push_finish.argtypes = [p, p, sz, psz]
    L.cg_push_finish.restype = i
    L.cg_push_bytes_consumed.argtypes = [p]
    L.cg_push_bytes_consumed.restype = u64
    L.cg_push_out_capacity.argtypes = [p, u64]
    L.cg_push_out_capacity.restype = sz
    L.cg_push_free.argtypes = [p]
    L.cg_push_free.restype = None
    L.cg_stream_new.argtypes = [u64, u64, u64, i, u64, u64, ctypes.POINTER(i)]
    L.cg_stream_new.restype = p
    L.cg_stream_push.argtypes = [p, p, u64]
    L.cg_stream_push.restype = i
    L.cg_stream_finish.argtypes = [p]
    L.cg_stream_finish.restype = i
    L.cg_stream_take.argtypes = [p, p, sz, psz, i]
    L.cg_stream_take.restype = i
    L.cg_stream_pending.argtypes = [p]
    L.cg_stream_pending.restype = u64
    L.cg_stream_bytes_consumed.argtypes = [p]
    L.cg_stream_bytes_consumed.restype = u64
    L.cg_stream_free.argtypes = [p]
    L.cg_stream_free.restype = None
    L.cg_hash_spans_device.argtypes = [p, p, p, sz, i, p, p]
    L.cg_hash_spans_device.restype = i
    L.cg_hash.argtypes = [p, u64, i, p]
    L.cg_hash.restype = i
    L.cg_cas_ids_device.argtypes = [p, p, p, sz, ctypes.c_uint32, p, p]
    L.cg_cas_ids_device.restype = i
    L.cg_cas_id.argtypes = [p, u64, ctypes.c_uint32, p]
    L.cg_cas_id.restype = i
    L.cg_node_put_batch_device.argtypes = [p, p, sz, u64, u64, u64, p, sz, p, p, p, p]
    L.cg_node_put_batch_device.restype = i
    L.cg_node_put.argtypes = [p, u64, u64, u64, u64, p, sz, psz, p, p]
    L.cg_node_put.restype = i
    L.cg_set_cdc_tables.argtypes = [p, p]
    L.cg_set_cdc_tables.restype = i
    L.cg_get_cdc_tables.argtypes = [p, p]
    L.cg_get_cdc_tables.restype = None
    L.cg_set_gear_table.argtypes = [p]
    L.cg_set_gear_table.restype = i
    L.cg_get_gear_table.argtypes = [p]
    L.cg_get_gear_table.restype = None
    L.cg_gear_is_placeholder.restype = i
    L.cg_selftest.restype = i
    L.cg_tables_verified.restype = i
    u32 = ctypes.c_uint32
    for name in ("cg_test_sha_quad_max", "cg_test_sha_split_max", "cg_test_sha_spin_limit", "cg_test_sha_quad_fill",
                 "cg_test_sha_pair_fill", "cg_test_scan_path", "cg_test_scan_kernel", "cg_test_coalesce"):
        getattr(L, name).argtypes = [u32]
        getattr(L, name).restype = u32
    for name in ("cg_test_sha_tiers", "cg_test_sha_tiers_fill"):
        getattr(L, name).argtypes = [u32, u32]
        getattr(L, name).restype = u32
    L.cg_test_scan_grid.argtypes = [u64]
    L.cg_test_scan_grid.restype = u64
    L.cg_test_cas_pair_max.argtypes = [ctypes.c_int64]
    L.cg_test_cas_pair_max.restype = ctypes.c_int64
    if hasattr(L, "cg_test_stream_group_cap"):  # (absent from builds before round 3: A/B runs)
        L.cg_test_stream_group_cap.argtypes = [u64]
        L.cg_test_stream_group_cap.restype = u64
        for name in ("cg_test_stream_eager", "cg_test_stream_max_lanes"):
            getattr(L, name).argtypes = [u32]
            getattr(L, name).restype = u32
    for name in ("cg_test_b3_fused_plan", "cg_test_b3_packed"):
        if hasattr(L, name):
            getattr(L, name).argtypes = [i]
            getattr(L, name).restype = i
    if hasattr(L, "cg_test_sha_occupancy"):
        L.cg_test_sha_occupancy.argtypes = [u32, u32]
        L.cg_test_sha_occupancy.restype = u32
    L.cg_hw_queues.argtypes = []
    L.cg_hw_queues.restype = i
    L.cg_test_split_mode.argtypes = [i]
    L.cg_test_split_mode.restype = i
    L.cg_coalesce_stats.argtypes = [p]
    L.cg_coalesce_stats.restype = None
    L.cg_test_fail_alloc.argtypes = [ctypes.c_uint32]
    L.cg_test_fail_alloc.restype = ctypes.c_uint32
    L.cg_set_profiling.argtypes = [i]
    L.cg_set_profiling.restype = None
    L.cg_last_stage_times.argtypes = [p, sz]
    L.cg_last_stage_times.restype = sz
    L.cg_last_sha_tiers.argtypes = [p]
    L.cg_last_sha_tiers.restype = i
    L.cg_synth_nars.argtypes = [p, p, sz, i, u64]
    L.cg_synth_nars.restype = None
    return L


# CHUNKER_AMD_DIAG=1 (scripts/diag_*.py only) loads the diagnostics build in its place;
# CHUNKER_AMD_LIB=<path> loads another build of the same ABI (kernel A/B experiments)
_env = __import__("os").environ
lib = _load(Path(_env["CHUNKER_AMD_LIB"]) if _env.get("CHUNKER_AMD_LIB")
            else DIAG_LIB_PATH if _env.get("CHUNKER_AMD_DIAG") == "1" else LIB_PATH)
assert lib.cg_abi_version() == ABI_VERSION

_diag = None


def diag_lib() -> ctypes.CDLL:
    """The diagnostics build (scripts/diag_*.py): built on demand, never used by the
    product path."""
    global _diag
    if _diag is None:
        if not DIAG_LIB_PATH.exists():
            import subprocess
            subprocess.run(["make", "-s", "-C", str(Path(__file__).resolve().parent / "csrc"), "diag"], check=True)
        _diag = _load(DIAG_LIB_PATH)
    return _diag


def last_error() -> str:
    msg = lib.cg_last_error_message()
    return msg.decode() if msg else ""


def last_error_detail() -> tuple[int, int, int, int]:
    """(status, a, b, c) of this thread's last failure: Bounds -> (data_len, offset,
    length), BufferLimitExceeded -> (attempted, limit, 0)."""
    out = (ctypes.c_uint64 * 3)()
    st = lib.cg_last_error_detail(out)
    return st, int(out[0]), int(out[1]), int(out[2])

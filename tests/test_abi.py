"""C-ABI and host-mirror checks that need no GPU: the library loads, exports every
symbol include/chunker_gpu.h declares, validates options with the reference's
messages, and the host-side types behave like the reference's."""
import ctypes
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.fixture(scope="module")
def ca():
    import chunker_amd

    return chunker_amd


def declared_symbols():
    text = (ROOT / "include" / "chunker_gpu.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(cg_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol(ca):
    from chunker_amd import _lib

    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(ca.lib, s), f"missing export {s}"
    assert set(syms) == set(_lib.EXPORTS)
    for s in _lib.TEST_HOOKS:
        assert hasattr(ca.lib, s), f"missing test hook {s}"
    assert ca.lib.cg_abi_version() == _lib.ABI_VERSION == 3


def test_product_library_has_no_diagnostic_kernels(ca):
    """Diagnostic kernels and modes live in libchunker_amd_diag.so only (make diag)."""
    import subprocess

    from chunker_amd import _lib

    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    assert "cg_diag_" not in out and "k_diag" not in out


def test_desc_layout(ca):
    assert ca.DESC_DTYPE.itemsize == 48
    assert ca.DESC_DTYPE.fields["hash"][1] == 16


def test_capacity(ca):
    assert ca.lib.cg_capacity(0, 1024) == 0
    assert ca.lib.cg_capacity(1, 1024) == 1
    assert ca.lib.cg_capacity(10 << 20, 256 << 10) == 41
    assert ca.lib.cg_capacity(1000, 65) == 1000 // 64 + 1


@pytest.mark.parametrize("mn,avg,mx,field", [((1 << 20) + 1, 1024, 4096, "min_size"),
                                             (64, (4 << 20) + 1, 16 << 20, "avg_size"),
                                             (64, 1024, (16 << 20) + 1, "max_size")])
def test_abi_validate_names_field(ca, mn, avg, mx, field):
    """src/chunking.rs:1378-1399."""
    msg = ctypes.create_string_buffer(256)
    assert ca.lib.cg_validate(mn, avg, mx, msg, 256) == 4
    assert field in msg.value.decode()
    with pytest.raises(ca.InvalidOptionsError) as ei:
        ca.ChunkingOptions.resolve(mn, avg, mx)
    assert field in str(ei.value) and str(ei.value).startswith("invalid_chunking_options: ")


def test_options_resolve(ca):
    o = ca.ChunkingOptions.resolve()
    assert (o.min_size, o.avg_size, o.max_size) == (256 * 1024, 1024 * 1024, 4 * 1024 * 1024)
    for t in [(64, 256, 1024), (64, 1024, 4096), (256 << 10, 1 << 20, 4 << 20), (1 << 20, 4 << 20, 16 << 20)]:
        o = ca.ChunkingOptions.resolve(*t)
        assert (o.min_size, o.avg_size, o.max_size) == t
    with pytest.raises(ca.InvalidOptionsError, match="min_size.*64"):
        ca.ChunkingOptions.resolve(32, 64, 128)
    with pytest.raises(ca.InvalidOptionsError):
        ca.ChunkingOptions.resolve(64, 64, 64)  # tests/streaming_chunking.rs:167-171
    with pytest.raises(ca.InvalidOptionsError):
        ca.ChunkingOptions.resolve(64, 1024, 64 * 1024 * 1024)
    with pytest.raises(ca.InvalidOptionsError, match="min_size must be <= avg_size"):
        ca.ChunkingOptions.resolve(4096, 1024, 8192)
    with pytest.raises(ca.InvalidOptionsError, match="avg_size must be <= max_size"):
        ca.ChunkingOptions.resolve(64, 8192, 4096)
    with pytest.raises(ca.InvalidOptionsError, match="got 0"):
        ca.ChunkingOptions.resolve(0, 1024, 4096)


def test_metadata_equality_ignores_payload(ca):
    """src/chunking.rs:1330-1358."""
    a = ca.ChunkMetadata(bytes([1]) * 32, 10, 5, b"payload-a")
    b = ca.ChunkMetadata(bytes([1]) * 32, 10, 5, b"payload-b")
    assert a == b and hash(a) == hash(b)
    assert ca.HashAlgorithm.Blake3 == 0 and ca.HashAlgorithm.Sha256 == 1


def test_error_display_strings(ca):
    assert str(ca.BoundsError(3, 1, 5)) == "bounds_check_failed: offset 1 + length 5 exceeds data length 3"
    assert str(ca.ZeroLengthChunkError()) == "zero_length_chunk: FastCDC returned a chunk with length 0"
    assert str(ca.BufferLimitExceededError(9, 8)) == "buffer_limit_exceeded: attempted 9 bytes, limit 8 bytes"
    assert str(ca.IoError("x")) == "io_error: x"


def test_no_cpu_fallback_without_gpu(ca):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(ca.DeviceUnavailableError):
        ca.chunk_descriptors(b"hello world")
    with pytest.raises(ca.DeviceUnavailableError):
        ca.PushChunker().push(bytes(300_000))
    import io
    with pytest.raises(ca.DeviceUnavailableError):
        ca.chunk_stream(io.BytesIO(bytes(300_000)))


def test_gear_table_plumbing(ca):
    from oracle import oracle as O

    g, m = ca.get_cdc_tables()
    assert np.array_equal(g, O.GEAR) and np.array_equal(m, O.MASKS)
    assert bool(ca.lib.cg_gear_is_placeholder()) == O.GEAR_IS_PLACEHOLDER
    alt = (O.GEAR ^ np.uint64(1)).astype(np.uint64)
    alt_m = O.MASKS.copy()
    alt_m[14] ^= np.uint64(1 << 3)
    try:
        ca.set_cdc_tables(alt, alt_m)
        g, m = ca.get_cdc_tables()
        assert np.array_equal(g, alt) and np.array_equal(m, alt_m) and ca.lib.cg_gear_is_placeholder() == 0
        assert not ca.tables_verified()  # a new set is unverified until the selftest passes
        ca.set_cdc_tables(O.GEAR)  # masks=None keeps the current MASKS
        g, m = ca.get_cdc_tables()
        assert np.array_equal(g, O.GEAR) and np.array_equal(m, alt_m)
        # the windowed GPU scan needs every tested bit within 48 bytes of history
        bad = O.MASKS.copy()
        bad[20] |= np.uint64(1 << 48)
        with pytest.raises(ca.InvalidOptionsError, match="bits above 47"):
            ca.set_cdc_tables(O.GEAR, bad)
    finally:
        ca.set_cdc_tables(O.GEAR, O.MASKS)
    assert bool(ca.lib.cg_gear_is_placeholder()) == O.GEAR_IS_PLACEHOLDER


def test_error_fields_cross_the_abi(ca):
    """ChunkingError::Bounds {data_len, offset, length} is rebuilt from
    cg_last_error_detail (src/chunking.rs:35-42) -- no device needed for this one:
    a device batch whose offsets do not start at 0 is rejected up front."""
    import ctypes as C

    offs = np.array([5, 10, 40], np.uint64)
    first = np.zeros(3, np.uint64)
    st = ca.lib.cg_chunk_batch_device(None, offs.ctypes.data, 2, 0, 0, 0, 1, None, 0, first.ctypes.data, None)
    assert st == 1
    assert ca._lib.last_error_detail() == (1, 40, 5, 0)
    with pytest.raises(ca.BoundsError) as ei:
        ca.chunk_batch_device(0, offs, 0, 0)
    e = ei.value
    assert (e.data_len, e.offset, e.length) == (40, 5, 0)
    assert str(e) == "bounds_check_failed: offset 5 + length 0 exceeds data length 40"
    # a successful call clears the detail
    assert ca.lib.cg_validate(0, 0, 0, None, 0) == 0
    assert ca._lib.last_error_detail() == (0, 0, 0, 0)
    msg = C.create_string_buffer(8)
    assert ca.lib.cg_validate(32, 64, 128, msg, 8) == 4 and ca._lib.last_error_detail()[0] == 4


def test_synthetic_nar_layout(ca):
    from chunker_amd.nar import SEED_BASE, synth_nars, xorshift_bytes_py

    data, offs = synth_nars([4096, 1024 + 112, 120], first_index=5)
    assert list(offs) == [0, 4096, 4096 + 1136, 4096 + 1136 + 120]
    for i in range(3):
        nar = data[offs[i]:offs[i + 1]].tobytes()
        assert nar[:8] == (13).to_bytes(8, "little") and nar[8:21] == b"nix-archive-1"
        L = len(nar) - 112
        assert nar[88:96] == L.to_bytes(8, "little")
        assert nar[96:96 + L] == xorshift_bytes_py(SEED_BASE ^ (5 + i), L)
        assert nar[-16:] == (1).to_bytes(8, "little") + b")" + bytes(7)
    z, _ = synth_nars([4096], zeros=True)
    assert not z[96:96 + 4096 - 112].any()


def test_cas_entry_validation_without_gpu(ca):
    """cg_cas_id / cg_cas_ids_device reject an unknown ObjectKind before touching a
    device (crates/core/cas/src/lib.rs:31-48 has kinds 1..7); no CPU fallback."""
    import torch

    from chunker_amd import cas

    buf = (ctypes.c_uint8 * 32)()
    for bad in (0, 8, 255):
        assert ca.lib.cg_cas_id(None, 0, bad, buf) == 4
        assert "object kind" in ca._lib.last_error()
        assert ca.lib.cg_cas_ids_device(None, None, None, 1, bad, None, None) == 4
    assert ca.lib.cg_cas_ids_device(None, None, None, 0, 1, None, None) == 0
    assert [int(k) for k in cas.ObjectKind] == list(range(1, 8))
    if not torch.cuda.is_available():
        with pytest.raises(ca.DeviceUnavailableError):
            cas.ContentId.compute(cas.ObjectKind.Chunk, b"hello")
        with pytest.raises(ca.DeviceUnavailableError):
            cas.node_put(bytes(100_000), 4096, 16_384, 65_536)


def test_stream_read_size(ca, monkeypatch):
    """ChunkStream refill size is the reference's formula (src/chunking.rs:713-716):
    max(min(max(max_size * 8, 4 MiB), cap), 4096), cap from CHUNKER_READ_SLICE_CAP_BYTES
    in 4 KiB..256 MiB, default 8 MiB (:417-433)."""
    from chunker_amd.chunking import stream_read_size

    monkeypatch.delenv("CHUNKER_READ_SLICE_CAP_BYTES", raising=False)
    assert stream_read_size(4 << 20) == 8 << 20
    assert stream_read_size(256 << 10) == 4 << 20
    assert stream_read_size(1024) == 4 << 20
    monkeypatch.setenv("CHUNKER_READ_SLICE_CAP_BYTES", str(64 << 20))
    assert stream_read_size(4 << 20) == 32 << 20
    monkeypatch.setenv("CHUNKER_READ_SLICE_CAP_BYTES", "4096")
    assert stream_read_size(1 << 20) == 4096
    monkeypatch.setenv("CHUNKER_READ_SLICE_CAP_BYTES", "12")  # out of range -> 8 MiB default
    assert stream_read_size(4 << 20) == 8 << 20


def test_nix_base32_reference_fixture(ca):
    """nix_base32_matches_nix (crates/proto/nix/src/narinfo.rs:383-385): the fixture's
    NarHash (SRI base64, :359) encodes to the reference's expected string (:361)."""
    import base64

    from chunker_amd.narinfo import nar_hash_field, nix_base32

    d = base64.b64decode("LHmbxrZuoUhZ7p0Q+oD4wBzxH/byKBAKbJsfAZXoBCU=")
    assert nix_base32(d) == "0984x2ah27wvdh510a7jyqgz2760z20gl44xxrcli8bfnv39ny9c"
    assert nar_hash_field(d) == "sha256:0984x2ah27wvdh510a7jyqgz2760z20gl44xxrcli8bfnv39ny9c"
    assert nix_base32(b"") == "" and len(nix_base32(bytes(32))) == 52

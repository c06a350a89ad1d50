"""Fail-closed FastCDC tables (include/chunker_gpu.h).

The crate's GEAR table (fastcdc 4.0.1, un-vendored: /root/reference/Cargo.lock:530-533)
is not in this build; tables/fastcdc_v2020_gear.txt is a labelled placeholder.  The
engine therefore refuses every chunking call while the placeholder is installed,
unless CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR=1, and runs any other table set only after
it reproduced the reference's golden fixture (src/chunking.rs:1266-1297) on the GPU.
conftest.py sets the opt-in for the rest of the suite; these tests remove it.
"""
import numpy as np
import pytest

from oracle import oracle as O

ENV = "CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR"
REFERENCE_FIXTURE = [(0, 6162), (6162, 7028), (13190, 7028), (20218, 7028), (27246, 7028), (34274, 7028),
                     (41302, 7028), (48330, 7028), (55358, 7028), (62386, 3273)]


@pytest.fixture
def ca():
    import chunker_amd

    return chunker_amd


def fixture_bytes():
    i = np.arange(64 * 1024 + 123, dtype=np.int64)
    return ((i * 31 + i // 7) % 251).astype(np.uint8)


@pytest.mark.skipif(not O.GEAR_IS_PLACEHOLDER, reason="the crate's GEAR table is installed")
def test_placeholder_refuses_every_chunking_entry(ca, monkeypatch):
    """No device needed: the placeholder check comes before any device work."""
    monkeypatch.delenv(ENV, raising=False)
    data = np.zeros(100_000, np.uint8)
    with pytest.raises(ca.TablesError, match="placeholder"):
        ca.chunk_data(data)
    with pytest.raises(ca.TablesError, match="CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR"):
        ca.chunk_batch([data, data])
    with pytest.raises(ca.TablesError):
        ca.PushChunker().push(b"x" * 1000)
    with pytest.raises(ca.TablesError):
        ca.PushChunker().finish()
    from chunker_amd import cas
    with pytest.raises(ca.TablesError):
        cas.node_put(data, 4096, 16_384, 65_536)
    offs = np.array([0, 10], np.uint64)
    with pytest.raises(ca.TablesError):
        ca.chunk_batch_device(0, offs, 0, 1)
    assert ca._lib.last_error_detail()[0] == 8
    # the opt-in is read per call ("1" only)
    monkeypatch.setenv(ENV, "yes")
    with pytest.raises(ca.TablesError):
        ca.chunk_data(data)


def test_opt_in_reaches_the_device_path(ca, monkeypatch):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the -m gpu tests")
    monkeypatch.setenv(ENV, "1")
    with pytest.raises(ca.DeviceUnavailableError):
        ca.chunk_data(b"hello world")


def test_oracle_fixture_status():
    """The oracle restatement against the reference fixture: exact once the crate's
    table is installed; with the placeholder it yields other boundaries (the number
    the GPU selftest must report)."""
    got = O.fastcdc(fixture_bytes(), 1024, 6000, 16 * 1024)
    if O.GEAR_IS_PLACEHOLDER:
        assert got != REFERENCE_FIXTURE
    else:
        assert got == REFERENCE_FIXTURE


@pytest.mark.gpu
def test_gpu_selftest(ca, gpu, monkeypatch):
    """cg_selftest runs the fixture through the GPU pipeline.  With the crate's table it
    passes; with the placeholder it fails and names what it found (the oracle's
    boundaries under the same table, i.e. the GPU path itself is exact)."""
    monkeypatch.delenv(ENV, raising=False)
    ref = O.fastcdc(fixture_bytes(), 1024, 6000, 16 * 1024)
    if not O.GEAR_IS_PLACEHOLDER:
        ca.selftest()
        assert ca.tables_verified()
        assert [(c.offset, c.length) for c in ca.chunk_descriptors(fixture_bytes(), 1024, 6000, 16384)] == \
            REFERENCE_FIXTURE
        return
    with pytest.raises(ca.TablesError) as ei:
        ca.selftest()
    msg = str(ei.value)
    assert f"gave {len(ref)} chunks" in msg and f"({ref[0][0]},{ref[0][1]})" in msg and "placeholder" in msg
    assert not ca.tables_verified()
    # the same fixture through the normal entry (opt-in) gives exactly the oracle's list
    monkeypatch.setenv(ENV, "1")
    got = ca.chunk_descriptors(fixture_bytes(), 1024, 6000, 16384)
    assert [(c.offset, c.length) for c in got] == ref


@pytest.mark.gpu
def test_gpu_unverified_table_runs_selftest_on_first_use(ca, gpu, monkeypatch):
    """A non-placeholder set is checked lazily on the first chunking call: one that
    does not reproduce the reference fixture is refused; masks with bits above 47 are
    rejected at install time."""
    alt = (O.GEAR * np.uint64(3) + np.uint64(7)).astype(np.uint64)
    monkeypatch.delenv(ENV, raising=False)
    try:
        ca.set_cdc_tables(alt, O.MASKS)
        assert ca.lib.cg_gear_is_placeholder() == 0 and not ca.tables_verified()
        with pytest.raises(ca.TablesError, match="selftest failed"):
            ca.chunk_data(np.zeros(5000, np.uint8), 1024, 4096, 8192)
        assert not ca.tables_verified()
        # with the opt-in the alternative table is used as installed (GPU == oracle under it)
        monkeypatch.setenv(ENV, "1")
        data = np.random.default_rng(3).integers(0, 256, 300_000, dtype=np.uint8)
        got = ca.chunk_descriptors_array(data, 1024, 4096, 16384)
        O.set_tables(alt, O.MASKS)
        try:
            ref = O.chunk_descriptors(data, 1024, 4096, 16384)
        finally:
            O.set_tables(O.GEAR, O.MASKS)
        assert np.array_equal(got["offset"], ref["offset"]) and np.array_equal(got["length"], ref["length"])
    finally:
        ca.set_cdc_tables(O.GEAR, O.MASKS)


def test_installer_parses_crate_source_and_refuses_a_wrong_table(tmp_path):
    """scripts/install_fastcdc_tables.py reads the crate's `GEAR` / `MASKS` array
    literals and writes nothing unless the oracle then reproduces the reference fixture;
    the placeholder written as such a source is refused with the boundaries it gives."""
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    src = "pub(super) const MASKS: [u64; 26] = [\n" + ",\n".join(f"    0x{int(v):016x}" for v in O.MASKS) + "\n];\n"
    src += "#[rustfmt::skip]\nconst GEAR: [u64; 256] = [\n"
    src += ",\n".join(f"    0x{int(v):016x}, // entry {i}"[:-len(f", // entry {i}")] + f" // {i}"
                      for i, v in enumerate(O.GEAR)) + "\n];\n"
    f = tmp_path / "mod.rs"
    f.write_text(src)
    before = (root / "tables" / "fastcdc_v2020_gear.txt").read_text()
    r = subprocess.run([sys.executable, str(root / "scripts" / "install_fastcdc_tables.py"), str(f)],
                       capture_output=True, text=True)
    if O.GEAR_IS_PLACEHOLDER:
        assert r.returncode != 0 and "REFUSED" in r.stderr + r.stdout
        ref = O.fastcdc(fixture_bytes(), 1024, 6000, 16 * 1024)
        assert f"give {len(ref)} chunks" in r.stderr + r.stdout
    assert (root / "tables" / "fastcdc_v2020_gear.txt").read_text() == before

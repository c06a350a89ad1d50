"""GPU parity: the gfx950 engine (through the C ABI) vs the CPU oracle.

Bit-exact on every (offset, length) and every digest.  Cases follow the
reference's own tests (src/chunking.rs:1168-1443, tests/streaming_chunking.rs,
tests/proptest_suite.rs, fuzz/fuzz_targets/chunking.rs) plus edge cases of the
GPU design (segment/halo seams, dense candidate segments, unaligned chunk
starts, empty and ragged NARs, digest padding boundaries).
"""
import ctypes
import hashlib
import io
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHA, B3 = 1, 0
D = (256 * 1024, 1024 * 1024, 4 * 1024 * 1024)
S = (64 * 1024, 256 * 1024, 1024 * 1024)
FIX = (1024, 6000, 16 * 1024)
TINY = (64, 256, 1024)
ODD = (65, 300, 1025)
ODD2 = (4097, 10000, 70001)


@pytest.fixture(scope="module")
def ca(gpu):
    import chunker_amd

    return chunker_amd


@pytest.fixture(scope="module")
def O():
    from oracle import oracle

    return oracle


def rand_bytes(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)


def fixture_bytes(n):
    i = np.arange(n, dtype=np.int64)
    return ((i * 31 + i // 7) % 251).astype(np.uint8)


def assert_same(got, ref, ctx=""):
    assert len(got) == len(ref), f"{ctx}: {len(got)} chunks vs oracle {len(ref)}"
    assert np.array_equal(got["offset"], ref["offset"]), ctx
    assert np.array_equal(got["length"], ref["length"]), ctx
    bad = np.nonzero(~np.all(got["hash"] == ref["hash"], axis=1))[0]
    assert len(bad) == 0, f"{ctx}: digest mismatch at chunks {bad[:8]}"


CASES = [
    ("empty", lambda: np.zeros(0, np.uint8), D),
    ("one", lambda: rand_bytes(1, 1), D),
    ("small_data", lambda: np.frombuffer(b"small data", np.uint8), D),
    ("63", lambda: rand_bytes(63, 2), TINY),
    ("min-1", lambda: rand_bytes(FIX[0] - 1, 3), FIX),
    ("min", lambda: rand_bytes(FIX[0], 4), FIX),
    ("min+1", lambda: rand_bytes(FIX[0] + 1, 5), FIX),
    ("fixture", lambda: fixture_bytes(64 * 1024 + 123), FIX),
    ("rand_fix_200k", lambda: rand_bytes(200_000, 6), FIX),
    ("rand_tiny_100k", lambda: rand_bytes(100_003, 7), TINY),
    ("rand_odd_300k", lambda: rand_bytes(300_001, 8), ODD),
    ("rand_odd2_3m", lambda: rand_bytes(3_000_017, 9), ODD2),
    ("zeros_10m", lambda: np.zeros(10 * 1024 * 1024, np.uint8), D),
    ("ff_1m", lambda: np.full(1 << 20, 0xFF, np.uint8), FIX),
    ("rand_D_10m", lambda: rand_bytes(10 * 1024 * 1024, 10), D),
    ("rand_S_5m", lambda: rand_bytes(5 * 1024 * 1024 + 77, 11), S),
    ("lowentropy_tiny", lambda: (rand_bytes(400_000, 12) & 3).astype(np.uint8), TINY),
    ("periodic_fix_S", lambda: fixture_bytes(3 * 1024 * 1024), S),
    ("repeat_phrase", lambda: np.frombuffer(b"descriptor parity test payload" * 8192, np.uint8), (1024, 4096, 8192)),
    ("max_sizes", lambda: rand_bytes(40 * 1024 * 1024 + 5, 13), (1 << 20, 4 << 20, 16 << 20)),
    ("all_min_sizes", lambda: rand_bytes(50_000, 14), (64, 256, 1024)),
]


@pytest.mark.parametrize("algo", [SHA, B3], ids=["sha256", "blake3"])
@pytest.mark.parametrize("name,make,params", CASES, ids=[c[0] for c in CASES])
def test_descriptors_match_oracle(ca, O, name, make, params, algo):
    data = make()
    got = ca.chunk_descriptors_array(data, *params, hash=algo)
    ref = O.chunk_descriptors(data, *params, algo=algo)
    assert_same(got, ref, name)
    # invariants of the reference tests: contiguity, full coverage, sizes
    if len(got):
        ends = got["offset"] + got["length"]
        assert got["offset"][0] == 0 and ends[-1] == len(data)
        assert np.array_equal(got["offset"][1:], ends[:-1])
        assert np.all(got["length"][:-1] >= 2 * (params[0] // 2)) and np.all(got["length"] <= params[2])
    else:
        assert len(data) == 0


@pytest.mark.parametrize("params,seed", [((1024, 6000, 16384), 22), ((4096, 16384, 65536), 22)])
def test_speculative_walk_rewalks(ca, O, params, seed):
    """Inputs whose cuts fall inside the 47-position warm-up window (where the
    windowed candidate list is not valid): the speculative walker must detect them in
    its verification pass and re-walk (and fall back to exact mode after 4)."""
    data = rand_bytes(30_000_000, seed)
    ref = O.chunk_descriptors(data, *params, algo=SHA)
    s_off = 2 * (params[0] // 2)
    warm = int(np.sum((ref["length"][:-1] >= s_off) & (ref["length"][:-1] < s_off + 47)))
    assert warm >= 2, "fixture no longer exercises warm-up cuts"
    assert_same(ca.chunk_descriptors_array(data, *params), ref, f"warm={warm}")
    # same bytes split into 3 NARs of one batch
    parts = [data[:9_999_991], data[9_999_991:20_000_003], data[20_000_003:]]
    got = ca.chunk_batch(parts, *params)
    for i, part in enumerate(parts):
        assert_same(got[i], O.chunk_descriptors(part, *params, algo=SHA), f"part{i}")


@pytest.mark.parametrize("params", [(4096, 16384, 65536), ODD2, (1024, 6000, 16384)], ids=["16k", "odd2", "fix"])
def test_piece_walks(ca, O, params):
    """NARs of two or more walk pieces (8 MiB here) are also walked piece by piece in
    parallel from each piece's first byte, and the NAR's walk takes whole runs of
    chunks from those lists once its sequence meets them: random NARs (sequences meet
    within a chunk or two), long zero runs (no candidates: max-size cuts that meet only
    when the piece length is a multiple of max, never for ODD2's 70001) and pieces
    that are zeros and random in turn, plus NARs just under / over two pieces."""
    rng = np.random.default_rng(31)
    mib = 1 << 20
    zr = np.zeros(20 * mib, np.uint8)
    zr[3 * mib:5 * mib] = rng.integers(0, 256, 2 * mib, dtype=np.uint8)
    zr[13 * mib + 77:15 * mib] = rng.integers(0, 256, 2 * mib - 77, dtype=np.uint8)
    nars = [rng.integers(0, 256, 40 * mib + 123, dtype=np.uint8), zr,
            rng.integers(0, 256, 16 * mib - 1, dtype=np.uint8), rng.integers(0, 256, 16 * mib + 1, dtype=np.uint8),
            np.zeros(17 * mib + 5, np.uint8)]
    got = ca.chunk_batch(nars, *params, hash=B3)
    for i, nar in enumerate(nars):
        assert_same(got[i], O.chunk_descriptors(nar, *params, algo=B3), f"nar{i} len={len(nar)}")


def tail_cut_case(O, params, tail_len, back, seed):
    """Bytes whose FastCDC cut lands `back` bytes before the end of a buffer whose length
    is 2 or 3 (mod 4): the last partial dword's bytes decide the cut.  (cut_gear tests
    positions up to 2 floor(len/2) - 1, so with len = 2 (mod 4) back is 1 or 2, with
    len = 3 (mod 4) it is 2 or 3.)  Built by choosing three bytes so that the Gear hash at
    position len - back matches mask_s, then keeping a case whose first cut the oracle
    puts there (no earlier position in the hashed region matches)."""
    mn, avg, mx = params
    bits = int(round(np.log2(avg)))
    mask_s = int(O.MASKS[bits + 1])
    G = O.GEAR.astype(np.uint64)
    rng = np.random.default_rng(seed)
    n = mn + 96 + tail_len
    assert n % 4 in (2, 3) and n < avg and n - back <= 2 * (n // 2) - 1
    for _ in range(64):
        data = rng.integers(0, 256, n, dtype=np.uint8)
        p = n - back  # the position whose hash must match
        w = 0  # windowed Gear hash up to p - 3 (bits <= 47 are exact after 48 bytes)
        for b in data[p - 3 - 60:p - 2]:
            w = ((w << 1) + int(G[b])) & (2 ** 64 - 1)
        x = np.arange(1 << 24, dtype=np.uint32)
        b0, b1, b2 = (x & 255), ((x >> 8) & 255), (x >> 16)
        h = np.uint64((w << 3) & (2 ** 64 - 1)) + (G[b0] << np.uint64(2)) + (G[b1] << np.uint64(1)) + G[b2]
        hit = np.flatnonzero((h & np.uint64(mask_s)) == 0)
        for v in hit[:32]:
            data[p - 2:p + 1] = [v & 255, (v >> 8) & 255, v >> 16]
            cuts = O.fastcdc(data, mn, avg, mx)
            if len(cuts) >= 2 and n - (cuts[0][0] + cuts[0][1]) <= 3:
                return data, cuts
    raise AssertionError("no tail-cut case found")


@pytest.mark.parametrize("tail,back", [(2, 1), (2, 2), (3, 2), (3, 3)], ids=["n2b1", "n2b2", "n3b2", "n3b3"])
def test_cut_in_last_partial_dword(ca, O, tail, back):
    """a batch whose length is not a multiple of 4 with a real FastCDC cut in
    its last 3 bytes.  K1 reads the batch's last rows through a buffer resource; the
    candidates there must come from the real bytes of the last (partial) dword, on the
    prefiltered flat kernel (avg 64 KiB) and the dense kernel (avg 4 KiB)."""
    for params in ((16384, 65536, 262144), (1024, 4096, 16384)):
        data, cuts = tail_cut_case(O, params, tail + 4 * 200, back, seed=back * 7 + tail + params[1])
        for algo in (SHA, B3):
            got = ca.chunking.chunk_descriptors_array(bytes(data), *params, hash=algo)
            ref = O.chunk_descriptors(data, *params, algo=algo)
            assert_same(got, ref, f"tail cut back={back} {params}")
            assert [(int(d["offset"]), int(d["length"])) for d in got] == cuts
        # the device entry over an exactly-sized device buffer (no slack after the batch)
        import torch

        d = torch.from_numpy(data.copy()).to("cuda")
        offs = np.array([0, len(data)], np.uint64)
        cap = ca.chunking.batch_capacity(offs, params[0])
        out = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
        first = ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params, hash=SHA)
        got = out[: int(first[-1]) * 48].cpu().numpy().view(ca.DESC_DTYPE)
        assert_same(got, O.chunk_descriptors(data, *params, algo=SHA), "device entry")


@pytest.mark.parametrize("algo", [SHA, B3], ids=["sha256", "blake3"])
def test_batch_ragged_unaligned(ca, O, algo):
    rng = np.random.default_rng(99)
    lens = [0, 1, 7, 1023, 1024, 1025, 65_535, 100_001, 0, 333_333, 1_048_577, 2_000_003, 5, 4_194_305]
    nars = [rng.integers(0, 256, n, dtype=np.uint8) for n in lens]
    params = (4096, 16384, 65536)
    got = ca.chunk_batch(nars, *params, hash=algo)
    for i, nar in enumerate(nars):
        assert_same(got[i], O.chunk_descriptors(nar, *params, algo=algo), f"nar{i} len={lens[i]}")


@pytest.mark.parametrize("params", [D, S], ids=["D", "S"])
def test_batch_synthetic_nars(ca, O, params):
    from chunker_amd.nar import synth_nars

    sizes = [4 * 1024 * 1024] * 24 + [1024 * 1024 + 8 * k for k in range(8)]
    data, offs = synth_nars(sizes)
    nars = [data[offs[i]:offs[i + 1]] for i in range(len(sizes))]
    got = ca.chunk_batch(nars, *params)
    for i, nar in enumerate(nars):
        assert_same(got[i], O.chunk_descriptors(nar, *params, algo=SHA), f"nar{i}")


def test_device_batch_matches_host(ca, O):
    import torch

    from chunker_amd.nar import synth_nars

    sizes = [2 * 1024 * 1024 + 8 * k for k in range(16)]
    data, offs = synth_nars(sizes, first_index=7)
    d = torch.from_numpy(data).cuda()
    cap = ca.chunking.batch_capacity(offs, D[0])
    out = torch.zeros(cap * 48, dtype=torch.uint8, device="cuda")
    first = ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *D,
                                  stream=torch.cuda.current_stream().cuda_stream)
    descs = out.cpu().numpy().view(ca.DESC_DTYPE)
    for i in range(len(sizes)):
        ref = O.chunk_descriptors(data[offs[i]:offs[i + 1]], *D, algo=SHA)
        assert_same(descs[int(first[i]):int(first[i + 1])], ref, f"nar{i}")


# --- streaming: tests/streaming_chunking.rs -----------------------------------
@pytest.mark.parametrize("slice_size", [512, 8_192, 65_536, 400_000, 1_500_000])
def test_push_matches_in_memory_across_slice_sizes(ca, slice_size):
    data = rand_bytes(1_500_000, 1234).tobytes()
    params = (8_192, 32_768, 131_072)
    expected = ca.chunk_data_with_hash(data, *params, hash=ca.HashAlgorithm.Blake3)
    pc = ca.PushChunker(*params, hash=ca.HashAlgorithm.Blake3)
    got, re = [], bytearray()
    for k in range(0, len(data), slice_size):
        for c in pc.push(data[k:k + slice_size]):
            re += c.payload
            got.append(c)
    for c in pc.finish():
        re += c.payload
        got.append(c)
    assert got == expected
    assert bytes(re) == data
    for c in got:
        assert len(c.payload) == c.length <= 131_072
        assert c.payload == data[c.offset:c.offset + c.length]


def test_push_nonuniform_with_empties(ca, O):
    data = rand_bytes(800_000, 99).tobytes()
    params = (8_192, 32_768, 131_072)
    expected = ca.chunk_data_with_hash(data, *params)
    pc = ca.PushChunker(*params)
    steps = [1, 7, 33, 1, 60_000, 3, 131_073, 500, 250_000, 9]
    got, pos, i = [], 0, 0
    while pos < len(data):
        assert pc.push(b"") == []
        step = min(steps[i % len(steps)], len(data) - pos)
        i += 1
        got += pc.push(data[pos:pos + step])
        pos += step
    got += pc.finish()
    assert got == expected
    # and the oracle's PushChunker restatement agrees chunk for chunk
    op = O.Push(*params, algo=SHA)
    ref = []
    pos, i = 0, 0
    while pos < len(data):
        step = min(steps[i % len(steps)], len(data) - pos)
        i += 1
        ref += list(op.push(data[pos:pos + step]))
        pos += step
    ref += list(op.finish())
    assert [(int(r["offset"]), int(r["length"]), bytes(r["hash"])) for r in ref] == \
        [(c.offset, c.length, c.hash) for c in got]


def test_push_empty_and_after_finish(ca):
    pc = ca.PushChunker()
    assert pc.push(b"") == [] and pc.finish() == []
    pc = ca.PushChunker()
    pc.push(b"hello streaming world")
    pc.finish()
    with pytest.raises(ca.ChunkingError):
        pc.push(b"more")


@pytest.mark.parametrize("params,seed,n", [((None, None, None), 42, 2_500_000),
                                           ((8_192, 32_768, 131_072), 84, 3_000_000)])
def test_stream_matches_in_memory(ca, params, seed, n):
    data = rand_bytes(n, seed).tobytes()
    stream = ca.chunk_stream_with_hash(io.BufferedReader(io.BytesIO(data)), *params, hash=ca.HashAlgorithm.Blake3)
    eager = ca.chunk_data_with_hash(data, *params, hash=ca.HashAlgorithm.Blake3)
    assert stream == eager
    total = 0
    for c in stream:  # fuzz_targets/chunking.rs invariants
        assert c.offset == total and c.payload == data[c.offset:c.offset + c.length]
        total += c.length
    assert total == len(data)


@pytest.mark.parametrize("algo", [SHA, B3], ids=["sha256", "blake3"])
@pytest.mark.parametrize("cap,inflight", [(65_536, 1), (300_000, 2 << 20), (4 << 20, 64 << 20)],
                         ids=["4slots", "wrap", "wide"])
def test_pipelined_stream_many_slices(ca, O, monkeypatch, algo, cap, inflight):
    """The pipelined ChunkStream (cg_stream_*) over many read slices: slots wrap around
    the arena (inflight=1 -> the 4-slot minimum, so pushes wait for digests), groups
    span slices, and every chunk equals the oracle's eager result, in order."""
    monkeypatch.setenv("CHUNKER_READ_SLICE_CAP_BYTES", str(cap))
    monkeypatch.setenv("CHUNKER_AMD_STREAM_INFLIGHT_BYTES", str(inflight))
    data = rand_bytes(9_000_017, 77).tobytes()
    params = (16_384, 65_536, 262_144)
    got = list(ca.ChunkStream(io.BytesIO(data), *params, hash=algo))
    ref = O.chunk_descriptors(data, *params, algo=algo, nthreads=8)
    assert [(c.offset, c.length, c.hash) for c in got] == \
        [(int(r["offset"]), int(r["length"]), bytes(r["hash"])) for r in ref]
    assert b"".join(c.payload for c in got) == data


def test_stream_abi_push_take_interleaved(ca, O):
    """cg_stream_* directly: uneven pushes (empty, tiny, larger than a slot), takes with
    wait = 0 between them, then finish + blocking takes; same chunks as the oracle."""
    import ctypes

    data = rand_bytes(5_000_000, 91).tobytes()
    params = (8_192, 32_768, 131_072)
    st = ctypes.c_int(0)
    h = ca.lib.cg_stream_new(*params, SHA, 100_000, 1 << 20, ctypes.byref(st))
    assert h and st.value == 0
    out = np.zeros(64, ca.DESC_DTYPE)
    n = ctypes.c_size_t(0)
    got = []
    steps = [0, 1, 7, 100_000, 999_999, 3, 250_000, 1_500_000]
    pos, i = 0, 0
    try:
        while pos < len(data):
            k = min(steps[i % len(steps)], len(data) - pos)
            i += 1
            buf = np.frombuffer(data[pos:pos + k], np.uint8) if k else np.zeros(1, np.uint8)
            assert ca.lib.cg_stream_push(h, buf.ctypes.data, k) == 0
            pos += k
            assert ca.lib.cg_stream_take(h, out.ctypes.data, len(out), ctypes.byref(n), 0) == 0
            got += [(int(d["offset"]), int(d["length"]), bytes(d["hash"])) for d in out[: n.value]]
        assert ca.lib.cg_stream_bytes_consumed(h) == len(data)
        assert ca.lib.cg_stream_finish(h) == 0
        assert ca.lib.cg_stream_push(h, out.ctypes.data, 1) == 4  # push after finish
        while True:
            assert ca.lib.cg_stream_take(h, out.ctypes.data, len(out), ctypes.byref(n), 1) == 0
            if n.value == 0:
                break
            got += [(int(d["offset"]), int(d["length"]), bytes(d["hash"])) for d in out[: n.value]]
        assert ca.lib.cg_stream_pending(h) == 0
    finally:
        ca.lib.cg_stream_free(h)
    ref = O.chunk_descriptors(data, *params, algo=SHA, nthreads=8)
    assert got == [(int(r["offset"]), int(r["length"]), bytes(r["hash"])) for r in ref]


def test_stream_small_read_cap(ca, monkeypatch):
    monkeypatch.setenv("CHUNKER_READ_SLICE_CAP_BYTES", "4096")
    data = (b"streaming chunker parity test" * 2048)
    assert ca.chunk_stream(io.BytesIO(data)) == ca.chunk_data(data)
    data = bytes([42]) * (3 * 1024 * 1024 + 321)
    chunks = ca.chunk_stream(io.BytesIO(data), 16 * 1024, 32 * 1024, 64 * 1024)
    assert sum(c.length for c in chunks) == len(data) and len(chunks) > 1


# --- reference unit tests, src/chunking.rs:1168-1443 --------------------------
def test_reference_unit_cases(ca):
    chunks = ca.chunk_data(bytes(1024 * 1024))
    assert chunks and [c.offset for c in chunks] == list(np.cumsum([0] + [c.length for c in chunks[:-1]]))
    assert sum(c.length for c in chunks) == 1024 * 1024
    small = ca.chunk_data(b"small data")
    assert len(small) == 1 and small[0].offset == 0 and small[0].length == 10
    sha = ca.chunk_data_with_hash(bytes([7]) * 4096, hash=ca.HashAlgorithm.Sha256)
    b3 = ca.chunk_data_with_hash(bytes([7]) * 4096, hash=ca.HashAlgorithm.Blake3)
    assert len(sha) == len(b3) and sha[0].hash != b3[0].hash
    data = b"descriptor parity test payload" * 8192
    d = ca.chunk_descriptors(data, 1024, 4096, 8192)
    m = ca.chunk_data(data, 1024, 4096, 8192)
    assert [(x.hash, x.offset, x.length) for x in d] == [(x.hash, x.offset, x.length) for x in m]
    assert ca.chunk_data(bytes(100), 1024, 4096, 4 * 1024 * 1024)
    data = b"stream hash parity test payload" * 1024
    assert ca.chunk_data_with_hash(data, 1024, 4096, 8192, hash=ca.HashAlgorithm.Blake3) == \
        ca.chunk_stream_with_hash(io.BytesIO(data), 1024, 4096, 8192, hash=ca.HashAlgorithm.Blake3)
    # zeros: every chunk is max-size (the reference's published-bench regime)
    z = ca.chunk_descriptors(bytes(10 * 1024 * 1024))
    assert [c.length for c in z] == [4 << 20, 4 << 20, 2 << 20]


# --- digests ------------------------------------------------------------------
def test_digest_kats(ca):
    from chunker_amd.hashing import blake3_hash, sha256_hash

    assert sha256_hash(b"hello world") == "b94d27b9934d3e08a52e52d7da7dabfac484efe37a5380ee9088f7ace2efcde9"
    assert blake3_hash(b"hello world") == "d74981efa70a0c880b8d8c1985d075dbcbf679b99a5f9914e5aaf96b831a9e24"
    assert blake3_hash(b"") == "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262"


def test_digest_spans_all_lengths(ca, O):
    import torch

    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
    lens = list(range(0, 300)) + [511, 512, 513, 1023, 1024, 1025, 2047, 2048, 2049, 4095, 4096, 4097, 65535,
                                  65536, 65537, 65536 * 3 + 1, 1 << 20, (1 << 20) + 3, 3 << 20,
                                  # BLAKE3 lane subtrees (4 leaves) and wave groups (256 leaves)
                                  3071, 3072, 3073, 5119, 5120, 5121, 7169, 8192, 261120, 262143, 262144, 262145,
                                  263168, 266241, 524289, 786432 + 2049]
    offs = [int(rng.integers(0, len(data) - n + 1)) for n in lens]
    d = torch.from_numpy(data).cuda()
    o = torch.tensor(offs, dtype=torch.int64).cuda()
    ln = torch.tensor(lens, dtype=torch.int64).cuda()
    for algo in (SHA, B3):
        dig = torch.zeros(len(lens) * 32, dtype=torch.uint8, device="cuda")
        st = ca.lib.cg_hash_spans_device(d.data_ptr(), o.data_ptr(), ln.data_ptr(), len(lens), algo, dig.data_ptr(),
                                         None)
        assert st == 0
        dig = dig.cpu().numpy().reshape(-1, 32)
        for k, (a, n) in enumerate(zip(offs, lens)):
            span = data[a:a + n].tobytes()
            want = hashlib.sha256(span).digest() if algo == SHA else O.blake3(span)
            assert bytes(dig[k]) == want, (algo, n, a)


@pytest.mark.parametrize("occ", [1, 2, 4])
def test_sha_fill_launch_occupancy(ca, occ):
    """A GPU-filling SHA-256 launch (40,000 spans: sha256_grid's fill tiers) at 1-4
    workgroups per CU (cg_test_sha_occupancy; the LDS pad that enforces it): every digest
    equals hashlib's, for span lengths 0..5,000 at random unaligned offsets plus the
    padding boundaries; the launch's one-lane workgroups cover the chunks the quad and pair
    tiers leave, 64 each."""
    import torch

    rng = np.random.default_rng(77)
    data = rng.integers(0, 256, 8 << 20, dtype=np.uint8)
    n = 40_000
    lens = rng.integers(0, 5001, n)
    lens[:130] = np.arange(130)
    lens[130:140] = [55, 56, 57, 63, 64, 65, 119, 120, 121, 128]
    offs = np.array([int(rng.integers(0, len(data) - int(m) + 1)) for m in lens], np.int64)
    d = torch.from_numpy(data).cuda()
    o = torch.from_numpy(offs).cuda()
    ln = torch.from_numpy(lens.astype(np.int64)).cuda()
    old_o = ca.lib.cg_test_sha_occupancy(1, occ)
    try:
        dig = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
        assert ca.lib.cg_hash_spans_device(d.data_ptr(), o.data_ptr(), ln.data_ptr(), n, SHA, dig.data_ptr(), None) == 0
        tiers = (ctypes.c_uint32 * 4)()
        ca.lib.cg_last_sha_tiers(tiers)
    finally:
        ca.lib.cg_test_sha_occupancy(1, old_o)
    nq, npair, nlane = int(tiers[0]), int(tiers[1]), int(tiers[2])
    assert nlane * 64 >= n - 8 * nq - 32 * npair > nlane * 64 - 64
    dig = dig.cpu().numpy().reshape(-1, 32)
    bad = [k for k in range(n) if bytes(dig[k]) != hashlib.sha256(data[offs[k]:offs[k] + lens[k]].tobytes()).digest()]
    assert not bad, (len(bad), bad[:8], [int(lens[k]) for k in bad[:8]])


def _sha_kinds(ca, quad_max, pair_max):
    """Cap the quad and pair workgroups of the SHA-256 launch; returns the old caps."""
    return ca.lib.cg_test_sha_quad_max(quad_max), ca.lib.cg_test_sha_split_max(pair_max)


def test_dpp_bank_mask_lane_probe(ca):
    """The split-lane SHA-256 rounds pair lanes 4 apart in a DPP row: a row_shl:4 add
    with bank_mask 0x5 writes lanes 0-3 and 8-11 of each row from lanes 4-7 / 12-15
    and leaves the others untouched (probe kernel in the diagnostics build)."""
    from chunker_amd._lib import DIAG_LIB_PATH, diag_lib

    if not DIAG_LIB_PATH.exists():
        pytest.skip("diagnostics build not present (make -C chunker_amd/csrc diag)")
    D = diag_lib()
    D.cg_diag_dpp_probe.argtypes = [ctypes.c_void_p]
    out = np.zeros(64, np.uint32)
    assert D.cg_diag_dpp_probe(out.ctypes.data) == 0
    want = [(1000 + 2 * L + 4) if ((L >> 2) & 1) == 0 else L for L in range(64)]
    assert out.tolist() == want


@pytest.mark.parametrize("params", [FIX, (16 * 1024, 64 * 1024, 256 * 1024), S, D], ids=["fix", "16k", "S", "D"])
def test_diag_scan_variants_agree(ca, params):
    """The alternative candidate-scan kernels kept in the diagnostics build for DESIGN.md
    §4's A/B (quad transpose, LDS-staged, page per wave, own segment per lane, the flat
    row kernel's ring-depth / load-policy variants) give the product's descriptors on a
    ragged multi-NAR batch, so the timings compared there are of correct kernels."""
    from chunker_amd._lib import DIAG_LIB_PATH, diag_lib
    from chunker_amd.chunking import DESC_DTYPE

    if not DIAG_LIB_PATH.exists():
        pytest.skip("diagnostics build not present (make -C chunker_amd/csrc diag)")
    Dl = diag_lib()
    Dl.cg_diag_scan_variant.argtypes = [ctypes.c_uint32]
    Dl.cg_diag_scan_mode.argtypes = [ctypes.c_uint32]
    sizes = [3 * 2**20 + 17, 2**20, 5 * 2**20 + 1000, 12345, 2 * 2**20 + 4095, 700 * 1024, 33]
    nars = [rand_bytes(s, 900 + i) for i, s in enumerate(sizes)]
    want, want_first = ca.chunking.chunk_batch_flat(np.concatenate(nars), np.cumsum([0] + sizes), *params, hash=B3)
    flat = np.concatenate(nars)
    offs = np.cumsum([0] + sizes).astype(np.uint64)
    cap = ca.chunking.batch_capacity(offs, params[0])
    try:
        for v, mode in [(0, 0), (1, 0), (2, 0), (3, 0), (4, 0), (5, 0), (5, 1), (5, 2), (5, 3), (5, 4), (5, 6), (5, 7), (5, 9), (5, 11), (5, 12), (5, 13), (5, 14), (5, 15), (5, 20), (5, 21), (5, 22)]:
            Dl.cg_diag_scan_variant(v)
            Dl.cg_diag_scan_mode(mode)
            out = np.zeros(cap, DESC_DTYPE)
            first = np.zeros(len(sizes) + 1, np.uint64)
            rc = Dl.cg_chunk_batch(flat.ctypes.data_as(ctypes.c_void_p), offs.ctypes.data_as(ctypes.c_void_p),
                                   ctypes.c_size_t(len(sizes)), ctypes.c_uint64(params[0]),
                                   ctypes.c_uint64(params[1]), ctypes.c_uint64(params[2]), ctypes.c_int(B3),
                                   out.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(cap),
                                   first.ctypes.data_as(ctypes.c_void_p))
            assert rc == 0, f"variant {v}/{mode}: status {rc}"
            assert np.array_equal(first, want_first), f"variant {v}/{mode}"
            assert_same(out[: int(first[-1])], want, f"variant {v}/{mode}")
    finally:
        Dl.cg_diag_scan_variant(0)
        Dl.cg_diag_scan_mode(0)


@pytest.mark.parametrize("quad_max,pair_max", [(0, 0), (0, 3), (2, 3), (1 << 20, 0), (0, 1 << 20)],
                         ids=["one_lane", "pair_mixed", "quad_pair_one", "quad", "pair"])
def test_sha_workgroup_kinds_agree(ca, O, quad_max, pair_max):
    """k_sha256 runs the longest chunks on quad workgroups (a round spread over 8
    lanes), the next on pair workgroups (2 lanes) and the rest one chunk per lane;
    every mix gives hashlib's digests, over every padding boundary, unaligned starts
    and multi-block chunks."""
    import torch

    prev = _sha_kinds(ca, quad_max, pair_max)
    split_max = (quad_max, pair_max)
    try:
        rng = np.random.default_rng(17)
        data = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
        lens = list(range(0, 200)) + [511, 512, 513, 4095, 4096, 4097, 65537, 1 << 20, (1 << 20) + 3, 2_000_001]
        offs = [int(rng.integers(0, len(data) - n + 1)) for n in lens]
        d = torch.from_numpy(data).cuda()
        o = torch.tensor(offs, dtype=torch.int64).cuda()
        ln = torch.tensor(lens, dtype=torch.int64).cuda()
        dig = torch.zeros(len(lens) * 32, dtype=torch.uint8, device="cuda")
        assert ca.lib.cg_hash_spans_device(d.data_ptr(), o.data_ptr(), ln.data_ptr(), len(lens), SHA,
                                           dig.data_ptr(), None) == 0
        dig = dig.cpu().numpy().reshape(-1, 32)
        for k, (a, n) in enumerate(zip(offs, lens)):
            assert bytes(dig[k]) == hashlib.sha256(data[a:a + n].tobytes()).digest(), (split_max, n, a)
        # and through the whole pipeline
        from chunker_amd.nar import synth_nars

        sizes = [1024 * 1024 + 8 * k for k in range(6)]
        nd, no = synth_nars(sizes, first_index=3)
        nars = [nd[no[i]:no[i + 1]] for i in range(len(sizes))]
        got = ca.chunk_batch(nars, 4096, 16384, 65536)
        for i, nar in enumerate(nars):
            assert_same(got[i], O.chunk_descriptors(nar, 4096, 16384, 65536, algo=SHA), f"nar{i}")
    finally:
        _sha_kinds(ca, *prev)


@pytest.mark.parametrize("quad_pm,pair_pm", [(850, 600), (1000, 1000), (1, 1), (900, 0), (500, 499)],
                         ids=["product", "longest_only", "all_quad", "no_one_lane", "close"])
def test_sha_latency_tiers_agree(ca, O, quad_pm, pair_pm):
    """Latency tiers (k_len_base -> k_sha256): the chunks needing a quad / a pair are
    counted on the device from the length histogram and the workgroup kinds follow them,
    so a chunk's lane count depends on its length; every threshold pair gives hashlib's
    digests over the span sweep and the oracle's descriptors through the pipeline."""
    import torch

    prev = ca.lib.cg_test_sha_tiers(quad_pm, pair_pm)
    prev_fill = ca.lib.cg_test_sha_tiers_fill(quad_pm, pair_pm)
    try:
        rng = np.random.default_rng(23)
        data = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
        lens = list(range(0, 130)) + [511, 4097, 65537, 300_000, 600_000, 900_000, 1 << 20, 1_500_000, 2_000_001]
        offs = [int(rng.integers(0, len(data) - n + 1)) for n in lens]
        d = torch.from_numpy(data).cuda()
        o = torch.tensor(offs, dtype=torch.int64).cuda()
        ln = torch.tensor(lens, dtype=torch.int64).cuda()
        dig = torch.zeros(len(lens) * 32, dtype=torch.uint8, device="cuda")
        assert ca.lib.cg_hash_spans_device(d.data_ptr(), o.data_ptr(), ln.data_ptr(), len(lens), SHA,
                                           dig.data_ptr(), None) == 0
        dig = dig.cpu().numpy().reshape(-1, 32)
        for k, (a, n) in enumerate(zip(offs, lens)):
            assert bytes(dig[k]) == hashlib.sha256(data[a:a + n].tobytes()).digest(), (quad_pm, pair_pm, n, a)
        from chunker_amd.nar import synth_nars

        sizes = [2 * 1024 * 1024 + 8 * k for k in range(6)]
        nd, no = synth_nars(sizes, first_index=5)
        nars = [nd[no[i]:no[i + 1]] for i in range(len(sizes))]
        got = ca.chunk_batch(nars, 4096, 16384, 65536)
        for i, nar in enumerate(nars):
            assert_same(got[i], O.chunk_descriptors(nar, 4096, 16384, 65536, algo=SHA), f"nar{i}")
    finally:
        ca.lib.cg_test_sha_tiers(prev >> 16, prev & 0xFFFF)
        ca.lib.cg_test_sha_tiers_fill(prev_fill >> 16, prev_fill & 0xFFFF)


@pytest.mark.slow
def test_full_size_config2_batch(ca, O):
    """BASELINE config 2 at full size (256 x 4 MiB NARs, defaults, SHA-256): every
    boundary and digest equal to the oracle."""
    from chunker_amd.nar import synth_nars

    sizes = [4 * 1024 * 1024] * 256
    data, offs = synth_nars(sizes)
    nars = [data[offs[i]:offs[i + 1]] for i in range(len(sizes))]
    got = ca.chunk_batch(nars, *D)
    nt = min(16, os.cpu_count() or 1)
    for i, nar in enumerate(nars):
        assert_same(got[i], O.chunk_descriptors(nar, *D, algo=SHA, nthreads=nt), f"nar{i}")


def _random_options(rng, large):
    """Valid (min, avg, max) spread over the option space (src/chunking.rs:190-231),
    log-uniform, so every scan / walk path is drawn: dense masks (k_scan<false>, exact
    walk), 14 prefilter bits (k_scan + speculative walk), >= 15 (k_scan_flat, drawn
    with `large`: averages of 256 KiB .. 4 MiB)."""
    avg = int(2 ** (rng.uniform(18, 22) if large else rng.uniform(8, 18)))
    mn = int(min(avg, 2 ** rng.uniform(6, min(20, np.log2(avg) + 0.01))))
    mx = int(max(avg, 1024, 2 ** rng.uniform(np.log2(max(avg, 1024)), 24)))
    return max(mn, 64), avg, min(mx, 16 * 1024 * 1024)


def _random_nar(rng, n):
    kind = rng.integers(0, 4)
    if kind == 0:
        return rng.integers(0, 256, n, dtype=np.uint8)
    if kind == 1:  # low entropy: few symbols
        return rng.integers(0, 3, n, dtype=np.uint8) * 85
    if kind == 2:  # zero runs with random islands
        a = np.zeros(n, np.uint8)
        for _ in range(int(rng.integers(0, 6))):
            s = int(rng.integers(0, max(n, 1)))
            e = min(n, s + int(rng.integers(1, 200_000)))
            a[s:e] = rng.integers(0, 256, e - s, dtype=np.uint8)
        return a
    return fixture_bytes(n)


@pytest.mark.parametrize("seed", range(12))
def test_randomized_options_batches(ca, O, seed):
    """Property sweep (in the spirit of tests/proptest_suite.rs): random valid options,
    random ragged batches of random / low-entropy / zero-run / fixture-pattern NARs, both
    digests; every NAR bit-exact vs the oracle."""
    rng = np.random.default_rng(1000 + seed)
    params = _random_options(rng, large=seed % 2 == 0)
    sizes = [int(x) for x in rng.integers(0, 3 * 1024 * 1024, int(rng.integers(1, 9)))]
    if seed % 3 == 0:
        sizes.append(int(rng.integers(16, 40)) * 1024 * 1024 + int(rng.integers(0, 4096)))  # multi-piece walk
    nars = [_random_nar(rng, n) for n in sizes]
    algo = SHA if seed % 4 < 2 else B3
    got = ca.chunk_batch(nars, *params, hash=algo)
    for i, nar in enumerate(nars):
        assert_same(got[i], O.chunk_descriptors(nar, *params, algo=algo), f"{params} nar{i} len={len(nar)}")


def _dense_region(O, rng, prefix, nbytes, mask):
    """Bytes that, appended to `prefix`, make about every 2nd-32nd position a candidate
    for `mask` (each byte pair chosen among 65536 so the windowed hash after it has the
    mask's bits clear): dense segments -- more candidates than the per-segment slots --
    that the scan must mark and the walker rescan exactly."""
    G = O.GEAR.astype(np.uint64)
    pair = (np.uint64(2) * G[:, None] + G[None, :]).reshape(-1)
    m64 = (1 << 64) - 1
    h = 0
    for x in prefix[-64:]:
        h = (h * 2 + int(G[x])) & m64
    out = np.empty(nbytes, np.uint8)
    with np.errstate(over="ignore"):
        for i in range(0, nbytes, 2):
            cand = np.uint64((4 * h) & m64) + pair
            ok = np.flatnonzero((cand & np.uint64(mask)) == 0)
            k = int(ok[0]) if len(ok) else int(rng.integers(0, 65536))
            out[i], out[i + 1] = k >> 8, k & 255
            h = int(cand[k])
    return out


@pytest.mark.parametrize("params", [D, S], ids=["D_flat", "S_kscan"])
def test_dense_candidate_segments(ca, O, params):
    """Adversarial bytes with candidates at a large fraction of positions, for the
    L mask past the chunk's center and for the S mask before it: every such 4 KiB
    segment overflows its candidate slots, the scan (k_scan_flat at D, k_scan at S)
    marks it dense and the walker re-scans it exactly."""
    import math

    rng = np.random.default_rng(77)
    bits = round(math.log2(params[1]))
    ms, ml = int(O.MASKS[bits + 1]), int(O.MASKS[bits - 1])
    a = rng.integers(0, 256, params[1] + params[1] // 3, dtype=np.uint8)  # past center: L region
    b = _dense_region(O, rng, a, 48 * 1024, ml)
    c = rng.integers(0, 256, params[0] + 5000, dtype=np.uint8)
    d = _dense_region(O, rng, np.concatenate([a, b, c]), 24 * 1024, ms)  # S candidates
    e = rng.integers(0, 256, 2 * params[2], dtype=np.uint8)
    nar = np.concatenate([a, b, c, d, e])
    # premise: the crafted regions hold far more candidates per 4 KiB than any slot list
    m64, g = (1 << 64) - 1, [int(v) for v in O.GEAR]
    for lo, hi, mask in ((len(a), len(a) + len(b), ml), (len(a) + len(b) + len(c), len(nar) - len(e), ms)):
        h, hits = 0, 0
        for p in range(lo - 64, lo + 4096):
            h = (h * 2 + g[nar[p]]) & m64
            hits += p >= lo and (h & mask) == 0
        assert hits > 32, f"only {hits} candidates in the first crafted segment"  # slots: 16 here
    for algo in (SHA, B3):
        got = ca.chunk_descriptors_array(nar, *params, hash=algo)
        assert_same(got, O.chunk_descriptors(nar, *params, algo=algo), f"algo={algo}")


@pytest.mark.parametrize("mx", [1024, 2048, 3072, 65536, 66560, 132096, 196608, 4 << 20])
def test_blake3_tree_shapes(ca, O, mx):
    """All-zero data cuts every chunk at max (the reference's published-bench regime), so
    max picks the BLAKE3 tree each chunk gets: 1-3 leaves (root at k_b3_fold's first or
    second level), one full 64-leaf group, a group plus a one-leaf group (65 leaves), and
    several groups folded by k_b3_top; the ragged tail chunk adds one more shape."""
    data = np.zeros(5 * mx + 777, np.uint8)
    params = (max(64, mx // 4), max(256, mx // 2), mx)
    got = ca.chunk_batch([data], *params, hash=B3)[0]
    want = O.chunk_descriptors(data, *params, algo=B3)
    assert_same(got, want, f"max={mx}")


@pytest.mark.parametrize("path", [1, 2, 3], ids=["one_block", "reduce", "top_scan"])
def test_scan_paths_agree(ca, O, path):
    """Every exclusive-scan path (scan.hip launch_scan_impl: one block, tile sums + a
    reducing apply, tile sums + top scan + apply), forced by the cg_test_scan_path hook at
    sizes where the default would pick another, gives the oracle's descriptors: the segment
    scan with its fused compaction (dense segments included), the per-NAR chunk counts and
    the BLAKE3 group counts."""
    rng = np.random.default_rng(31)
    lens = [0, 1, 1025, 65_535, 333_333, 2_000_003, 7, 4_194_305, 3_000_001]
    nars = [rng.integers(0, 256, n, dtype=np.uint8) for n in lens]
    params = (4096, 16384, 65536)
    bits = 14
    a = rng.integers(0, 256, params[1] + params[1] // 3, dtype=np.uint8)
    dense = np.concatenate([a, _dense_region(O, rng, a, 16 * 1024, int(O.MASKS[bits - 1])),
                            rng.integers(0, 256, 3 * params[2], dtype=np.uint8)])
    old = ca.lib.cg_test_scan_path(path)
    try:
        for algo in (SHA, B3):
            got = ca.chunk_batch(nars, *params, hash=algo)
            for i, nar in enumerate(nars):
                assert_same(got[i], O.chunk_descriptors(nar, *params, algo=algo), f"path={path} nar{i} algo={algo}")
            got = ca.chunk_descriptors_array(dense, *params, hash=algo)
            assert_same(got, O.chunk_descriptors(dense, *params, algo=algo), f"path={path} dense algo={algo}")
    finally:
        ca.lib.cg_test_scan_path(old)


@pytest.mark.parametrize("kernel", [2, 1, 0], ids=["persistent", "oneshot", "product"])
def test_scan_kernels_agree(ca, O, kernel):
    """K1's persistent form (k_scan_flat32p: resident grid, per-XCD unit queue, halo row
    per unit; the product from 4 GiB on) and the one-shot k_scan_flat32 (the product below),
    each forced at any size by cg_test_scan_kernel, both give the oracle's descriptors on
    batches whose NAR and unit seams fall everywhere: units of 16 segments (64 KiB) against
    NARs of odd lengths, a batch of many tiny NARs, a batch ending inside a unit's first
    row, one with fewer units than waves, and back-to-back launches (the queue must come
    back zeroed after each)."""
    rng = np.random.default_rng(77 + kernel)
    params = (16384, 65536, 262144)  # 16 prefilter bits: the flat kernels
    unit = 65536
    batches = [
        [rng.integers(0, 256, n, dtype=np.uint8) for n in (unit * 3 + 5, 2048, 1, unit - 1, unit + 2049, 500_001)],
        [rng.integers(0, 256, int(n), dtype=np.uint8) for n in rng.integers(1, 9000, 300)],
        [rng.integers(0, 256, unit * 5 + 100, dtype=np.uint8)],
        [rng.integers(0, 256, 6_000_011, dtype=np.uint8), rng.integers(0, 256, 2_000_000, dtype=np.uint8)],
    ]
    old = ca.lib.cg_test_scan_kernel(kernel)
    try:
        for rep in range(2):
            for b, nars in enumerate(batches):
                got = ca.chunk_batch(nars, *params, hash=SHA)
                for i, nar in enumerate(nars):
                    assert_same(got[i], O.chunk_descriptors(nar, *params, algo=SHA), f"kernel={kernel} b{b} nar{i}")
    finally:
        ca.lib.cg_test_scan_kernel(old)


@pytest.mark.parametrize("fused,packed", [(1, 1), (1, 0), (0, 0)], ids=["packed_leaves", "assembly_map", "plan_kernel"])
def test_blake3_group_map_paths(ca, O, fused, packed):
    """The BLAKE3 group map (group_base / gmap) comes from the walk + descriptor assembly
    (each NAR's group count, k_assemble_counts) or from k_b3_plan (cg_test_b3_fused_plan),
    and with the assembly's map the leaves run packed across chunks (k_b3_leaves,
    cg_test_b3_packed) or one group per wave: every form gives the oracle's digests on
    ragged NARs (empty ones, sub-leaf chunks, chunks of 1 .. 256 groups: max 16 MiB on
    zeros; tiny chunks that put many chunks in one wave) and many-NAR batches."""
    rng = np.random.default_rng(57)
    lens = [0, 1, 1023, 1024, 1025, 65_536, 65_537, 0, 3_000_001, 131_072 * 3 + 5, 7]
    nars = [rng.integers(0, 256, n, dtype=np.uint8) for n in lens] + [np.zeros(40 << 20, np.uint8)]
    old = ca.lib.cg_test_b3_fused_plan(fused)
    old_p = ca.lib.cg_test_b3_packed(packed)
    try:
        tiny = [rng.integers(0, 256, int(n), dtype=np.uint8) for n in rng.integers(0, 5000, 300)]
        got = ca.chunk_batch(tiny, 64, 256, 1024, hash=B3)
        for i in (0, 1, 150, 299):
            assert_same(got[i], O.chunk_descriptors(tiny[i], 64, 256, 1024, algo=B3), f"tiny nar{i}")
        for params in ((4096, 16384, 65536), (1 << 20, 4 << 20, 16 << 20)):
            got = ca.chunk_batch(nars, *params, hash=B3)
            for i, nar in enumerate(nars):
                assert_same(got[i], O.chunk_descriptors(nar, *params, algo=B3), f"fused={fused} {params} nar{i}")
        many = [rng.integers(0, 256, int(n), dtype=np.uint8) for n in rng.integers(0, 300_000, 600)]
        got = ca.chunk_batch(many, 4096, 16384, 65536, hash=B3)
        for i in (0, 1, 299, 598, 599):
            assert_same(got[i], O.chunk_descriptors(many[i], 4096, 16384, 65536, algo=B3), f"many nar{i}")
    finally:
        ca.lib.cg_test_b3_fused_plan(old)
        ca.lib.cg_test_b3_packed(old_p)


def test_blake3_group_map_capacity_error(ca):
    """A descriptor array too small for the batch: the fused group map writes only inside
    its bounds and the call fails as the SHA-256 path does."""
    import torch

    from chunker_amd.nar import synth_nars

    data, offs = synth_nars([1 << 20] * 8, first_index=5)
    d = torch.from_numpy(data).cuda()
    out = torch.zeros(8 * 48, dtype=torch.uint8, device="cuda")
    for algo in (B3, SHA):
        with pytest.raises(ca.ChunkingError, match="too small"):
            ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), 8, 4096, 16384, 65536, hash=algo,
                                  stream=torch.cuda.current_stream().cuda_stream)
    # the engine is still usable afterwards
    cap = ca.chunking.batch_capacity(offs, 4096)
    out = torch.zeros(cap * 48, dtype=torch.uint8, device="cuda")
    first = ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, 4096, 16384, 65536, hash=B3,
                                  stream=torch.cuda.current_stream().cuda_stream)
    assert int(first[-1]) > 8


def test_async_batches_match_sync(ca, O):
    """cg_chunk_batch_device_async + cg_batch_wait: several batches queued on one stream
    (each with its own workspace) give the synchronous entry's descriptors and index; waits
    may come in any order; an unwaited handle is reclaimed; a capacity error surfaces at
    the wait and the engine stays usable."""
    import torch

    from chunker_amd.nar import synth_nars

    stream = torch.cuda.current_stream().cuda_stream
    batches = []
    for seed, algo in ((1, SHA), (2, B3), (3, SHA), (4, B3)):
        sizes = [1 << 20] * 5 + [8 * seed + 4096, 200_008]
        data, offs = synth_nars(sizes, first_index=100 * seed)
        d = torch.from_numpy(data).cuda()
        cap = ca.chunking.batch_capacity(offs, 4096)
        ref_out = torch.zeros(cap * 48, dtype=torch.uint8, device="cuda")
        ref_first = ca.chunk_batch_device(d.data_ptr(), offs, ref_out.data_ptr(), cap, 4096, 16384, 65536, hash=algo,
                                          stream=stream)
        batches.append((d, offs, cap, algo, ref_out.cpu().numpy(), ref_first, data))
    outs = [torch.zeros(b[2] * 48, dtype=torch.uint8, device="cuda") for b in batches]
    inflight = [ca.chunk_batch_device_async(b[0].data_ptr(), b[1], o.data_ptr(), b[2], 4096, 16384, 65536, hash=b[3],
                                            stream=stream) for b, o in zip(batches, outs)]
    for k in (2, 0, 3, 1):  # out of order
        first = inflight[k].wait()
        d, offs, cap, algo, ref_out, ref_first, data = batches[k]
        assert np.array_equal(first, ref_first), k
        got = outs[k].cpu().numpy()
        n = int(first[-1])
        assert np.array_equal(got[: n * 48], ref_out[: n * 48]), k
        descs = got.view(ca.DESC_DTYPE)
        ref = O.chunk_descriptors(data[offs[5]:offs[6]], 4096, 16384, 65536, algo=algo)
        assert_same(descs[int(first[5]):int(first[6])], ref, f"batch{k} nar5")
    with pytest.raises(ca.IoError):
        inflight[0].wait()
    # an unwaited handle goes back to the pool when collected
    b = batches[0]
    h = ca.chunk_batch_device_async(b[0].data_ptr(), b[1], outs[0].data_ptr(), b[2], 4096, 16384, 65536, hash=SHA,
                                    stream=stream)
    del h
    # capacity error at the wait
    h = ca.chunk_batch_device_async(b[0].data_ptr(), b[1], outs[0].data_ptr(), 3, 4096, 16384, 65536, hash=B3,
                                    stream=stream)
    with pytest.raises(ca.ChunkingError, match="too small"):
        h.wait()
    first = ca.chunk_batch_device_async(b[0].data_ptr(), b[1], outs[0].data_ptr(), b[2], 4096, 16384, 65536,
                                        hash=SHA, stream=stream).wait()
    assert np.array_equal(first, b[5])


@pytest.mark.parametrize("mode", [1, 2], ids=["boundary_split", "whole_batch_split"])
def test_async_after_inputs_ready_matches_sync(ca, O, mode):
    """cg_chunk_batch_device_async_after: each batch's input is written on ANOTHER stream
    (a pinned H2D copy) and its boundary stages wait only for that copy's event, not for the
    batch queued before on the digest stream -- so they run under that batch's digest.
    Every batch (SHA-256 and BLAKE3, all five queued before the first wait) equals the
    synchronous entry's descriptors and index, and the oracle on a sampled NAR."""
    import torch

    from chunker_amd.nar import synth_nars

    stream = torch.cuda.Stream()
    copy = torch.cuda.Stream()
    batches = []
    old_mode = ca.lib.cg_test_split_mode(mode)  # 2: the digests of queued batches overlap too
    try:
        for seed, algo in ((11, SHA), (12, B3), (13, SHA), (14, SHA), (15, B3)):
            sizes = [4 << 20] * 12 + [8 * seed + 4096, 300_008]
            data, offs = synth_nars(sizes, first_index=1000 * seed)
            cap = ca.chunking.batch_capacity(offs, 16384)
            ref = torch.from_numpy(data).cuda()
            ref_out = torch.zeros(cap * 48, dtype=torch.uint8, device="cuda")
            ref_first = ca.chunk_batch_device(ref.data_ptr(), offs, ref_out.data_ptr(), cap, 16384, 65536, 262144,
                                              hash=algo, stream=torch.cuda.current_stream().cuda_stream)
            del ref
            batches.append((torch.from_numpy(data).pin_memory(), offs, cap, algo, ref_out.cpu().numpy(), ref_first, data))
        torch.cuda.synchronize()
        devs = [torch.empty(len(b[6]) + 256, dtype=torch.uint8, device="cuda") for b in batches]
        outs = [torch.full((b[2] * 48,), 0xAB, dtype=torch.uint8, device="cuda") for b in batches]
        inflight = []
        for k, b in enumerate(batches):
            with torch.cuda.stream(copy):  # the input arrives on the copy stream
                devs[k][: len(b[6])].copy_(b[0], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
            inflight.append(ca.chunk_batch_device_async(devs[k].data_ptr(), b[1], outs[k].data_ptr(), b[2], 16384, 65536,
                                                        262144, hash=b[3], stream=stream.cuda_stream,
                                                        inputs_ready=ev.cuda_event))
        # work queued on `stream` after the calls follows every batch (mode 2 joins each batch's
        # end into it): copies queued now, before any wait, must see the finished descriptors
        tails = [torch.empty_like(o) for o in outs]
        with torch.cuda.stream(stream):
            for t, o in zip(tails, outs):
                t.copy_(o)
        stream.synchronize()  # waits for the copies, which wait for every batch
        for k, h in enumerate(inflight):
            first = h.wait()
            _, offs, cap, algo, ref_out, ref_first, data = batches[k]
            assert torch.equal(tails[k], outs[k]), f"batch{k}: work queued after it on the stream ran early"
            assert np.array_equal(first, ref_first), k
            n = int(first[-1])
            got = outs[k].cpu().numpy()
            assert np.array_equal(got[: n * 48], ref_out[: n * 48]), k
            descs = got.view(ca.DESC_DTYPE)
            want = O.chunk_descriptors(data[offs[12]:offs[13]], 16384, 65536, 262144, algo=algo)
            assert_same(descs[int(first[12]):int(first[13])], want, f"batch{k} nar12")
    finally:
        ca.lib.cg_test_split_mode(old_mode)


@pytest.mark.parametrize("depth,group", [(None, None), (1, None), (3, 2), (20, 4), (None, 0), (3, 0), (20, 0)],
                         ids=["default", "one", "three_g2", "twenty_g4", "perbatch_default", "perbatch_three",
                              "perbatch_twenty"])
def test_batch_pipeline_matches_sync(ca, O, depth, group):
    """chunker_amd.BatchPipeline (one thread, up to `depth` batches in flight, each after
    its own inputs-ready event, DESIGN.md §7 "Batches in flight"), as the digest pipeline
    (group None = default_group, or merged groups of 2 / 4) and as the round-5 per-batch
    stream path (group 0; default depth 2 at this process's 4 hardware queues): twelve or
    more SHA-256 batches (with fewer output arrays than the depth the test drains early)
    come back in submission order, each equal to the synchronous entry, with the oracle on a
    sampled NAR; the output arrays rotate, each reused only after its batch was returned."""
    import torch

    from chunker_amd.nar import synth_nars

    sizes = [2 << 20] * 6 + [12345 * 8, 300_008]
    data, offs = synth_nars(sizes, first_index=77)
    cap = ca.chunking.batch_capacity(offs, 16384)
    d = torch.from_numpy(np.concatenate([data, np.zeros(256, np.uint8)])).cuda()
    ref_out = torch.zeros(cap * 48, dtype=torch.uint8, device="cuda")
    ref_first = ca.chunk_batch_device(d.data_ptr(), offs, ref_out.data_ptr(), cap, 16384, 65536, 262144)
    ref = ref_out.cpu().numpy()
    n_out = 4 if depth is None else depth + 1
    nb = 12 if depth is None or depth < 12 else depth + 4
    outs = [torch.full((cap * 48,), 0xAB, dtype=torch.uint8, device="cuda") for _ in range(n_out)]
    ready = torch.cuda.Event()
    ready.record()
    stream = torch.cuda.Stream()
    results = []
    free = list(range(n_out))
    busy = {}
    with ca.BatchPipeline(depth, 16384, 65536, 262144, stream=stream.cuda_stream, group=group) as pipe:
        for k in range(nb):
            j = free.pop(0)
            busy[k] = j
            for tag, first in pipe.submit(d.data_ptr(), offs, outs[j].data_ptr(), cap, inputs_ready=ready.cuda_event,
                                          tag=k):
                results.append((tag, first, outs[busy[tag]].cpu().numpy()))
                free.append(busy.pop(tag))
            if not free:  # more batches in flight than output arrays: take the oldest back
                for tag, first in pipe.drain():
                    results.append((tag, first, outs[busy[tag]].cpu().numpy()))
                    free.append(busy.pop(tag))
        for tag, first in pipe.drain():
            results.append((tag, first, outs[busy[tag]].cpu().numpy()))
    assert [t for t, _, _ in results] == list(range(nb))
    n = int(ref_first[-1])
    want = O.chunk_descriptors(data[offs[6]:offs[7]], 16384, 65536, 262144, algo=SHA)
    for k, first, got in results:
        assert np.array_equal(first, ref_first), k
        assert np.array_equal(got[: n * 48], ref[: n * 48]), k
        assert_same(got.view(ca.DESC_DTYPE)[int(first[6]):int(first[7])], want, f"batch{k} nar6")


def test_batch_pipeline_depth_rule(ca):
    """default_depth (the pipeline's and bench.py's rule) and the pipeline's option checks."""
    assert ca.default_depth(ca.HashAlgorithm.Blake3, 1 << 30) == 2
    with pytest.raises(ca.InvalidOptionsError):
        ca.BatchPipeline(0)

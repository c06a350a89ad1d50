"""CPU oracle checks (no GPU): the restatement against every pin the reference
holds for this path, plus internal consistency and the golden fixtures.

Pins: SHA-256 KAT (src/lib.rs:54-69) and hashlib (independent, complete);
BLAKE3 KAT (src/hashing.rs:173-182) and the published BLAKE3 test vectors
(tests/golden/blake3_vectors.json); FastCDC golden fixture
(src/chunking.rs:1266-1297) -- pinned only once the crate's GEAR table is
installed (tables/README.md), xfail while the placeholder table is in place.
"""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = Path(__file__).resolve().parent / "golden"
SHA, B3 = O.SHA256, O.BLAKE3


def test_sha256_kat_and_hashlib():
    assert O.sha256(b"hello world").hex() == "b94d27b9934d3e08a52e52d7da7dabfac484efe37a5380ee9088f7ace2efcde9"
    rng = np.random.default_rng(0)
    for force_scalar in (0, 1):
        O.lib().or_sha256_force_scalar(force_scalar)
        for n in list(range(0, 130)) + [1000, 4096, 65536 + 7, 1 << 20]:
            d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            assert O.sha256(d) == hashlib.sha256(d).digest(), (n, force_scalar)
    O.lib().or_sha256_force_scalar(0)


def test_blake3_kat_and_vectors():
    assert O.blake3(b"hello world").hex() == "d74981efa70a0c880b8d8c1985d075dbcbf679b99a5f9914e5aaf96b831a9e24"
    vec = json.loads((GOLDEN / "blake3_vectors.json").read_text())
    for case in vec["cases"]:
        n = case["input_len"]
        d = bytes(i % 251 for i in range(n))
        assert O.blake3(d).hex() == case["hash"], n


def test_blake3_tree_forms_agree():
    rng = np.random.default_rng(1)
    for n in [0, 1, 1023, 1024, 1025, 2047, 2048, 2049, 3072, 5 * 1024 + 1, 31 * 1024, 64 * 1024,
              64 * 1024 + 1, 65 * 1024, 200_000, 1 << 20]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert O.blake3(d) == O.blake3_stack(d), n


def _fixture_data():
    return bytes(((i * 31 + i // 7) % 251) for i in range(64 * 1024 + 123))


REFERENCE_FIXTURE = [(0, 6162), (6162, 7028), (13190, 7028), (20218, 7028), (27246, 7028), (34274, 7028),
                     (41302, 7028), (48330, 7028), (55358, 7028), (62386, 3273)]


def test_reference_golden_fixture():
    """src/chunking.rs:1266-1297 ("generated with fastcdc 3.2.1")."""
    got = O.fastcdc(_fixture_data(), 1024, 6000, 16 * 1024)
    if O.GEAR_IS_PLACEHOLDER:
        pytest.xfail("GEAR table is the placeholder (tables/README.md): FastCDC boundary parity unpinned")
    assert got == REFERENCE_FIXTURE


def py_cut_gear(src: bytes, mn, avg, mx, gear, masks):
    """Second, pure-Python transliteration of fastcdc v2020 cut_gear [ext]
    (SURVEY.md Appendix A.2), used only to cross-check the C restatement."""
    M = (1 << 64) - 1
    bits = int(round(np.log2(avg)))
    ms, ml = int(masks[bits + 1]), int(masks[bits - 1])
    remaining = len(src)
    if remaining <= mn:
        return remaining
    center = avg
    if remaining > mx:
        remaining = mx
    elif remaining < center:
        center = remaining
    index, h = mn // 2, 0
    while index < center // 2:
        a = index * 2
        h = ((h << 2) + (int(gear[src[a]]) << 1)) & M
        if h & (ms << 1) == 0:
            return a
        h = (h + int(gear[src[a + 1]])) & M
        if h & ms == 0:
            return a + 1
        index += 1
    while index < remaining // 2:
        a = index * 2
        h = ((h << 2) + (int(gear[src[a]]) << 1)) & M
        if h & (ml << 1) == 0:
            return a
        h = (h + int(gear[src[a + 1]])) & M
        if h & ml == 0:
            return a + 1
        index += 1
    return remaining


@pytest.mark.parametrize("params", [(64, 256, 1024), (65, 300, 1025), (1024, 6000, 16384), (1024, 4096, 16384)])
def test_cut_gear_two_restatements_agree(params):
    rng = np.random.default_rng(sum(params))
    for trial in range(6):
        n = int(rng.integers(1, 40_000))
        data = rng.integers(0, 256 if trial % 2 else 4, n, dtype=np.uint8).tobytes()
        want, pos = [], 0
        while pos < n:
            ln = py_cut_gear(data[pos:], *params, O.GEAR, O.MASKS)
            want.append((pos, ln))
            pos += ln
        assert O.fastcdc(data, *params) == want


def test_windowed_hash_premise():
    """The GPU design's premise: for positions >= 47 bytes
    past the hash start, the tested bits of the restarted hash equal those of the
    48-byte windowed hash."""
    M = (1 << 64) - 1
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, 4000, dtype=np.uint8)
    low48 = (1 << 48) - 1
    for s in (0, 100, 1234):
        h = 0
        for p in range(s, s + 300):
            h = ((h << 1) + int(O.GEAR[data[p]])) & M
            if p >= s + 47:
                w = 0
                for q in range(p - 47, p + 1):
                    w = ((w << 1) + int(O.GEAR[data[q]])) & M
                assert (h & low48) == (w & low48)


@pytest.mark.parametrize("params", [(1024, 4096, 16384)])
def test_proptest_reconstruct(params):
    """tests/proptest_suite.rs:23-31: chunks reconstruct the input (1..10 KiB)."""
    rng = np.random.default_rng(4)
    for _ in range(50):
        n = int(rng.integers(1024, 10 * 1024))
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        chunks = O.fastcdc(data, *params)
        assert b"".join(data[o:o + ln] for o, ln in chunks) == data


def test_zeros_and_small():
    z = O.fastcdc(np.zeros(10 * 1024 * 1024, np.uint8), 256 * 1024, 1024 * 1024, 4 * 1024 * 1024)
    assert z == [(0, 4 << 20), (4 << 20, 4 << 20), (8 << 20, 2 << 20)]  # benches/throughput.rs regime
    assert O.fastcdc(b"small data", 256 * 1024, 1024 * 1024, 4 * 1024 * 1024) == [(0, 10)]
    assert O.fastcdc(b"", 1024, 4096, 16384) == []


def test_validate_messages():
    """src/chunking.rs:1360-1442, tests/streaming_chunking.rs:165-183."""
    assert O.validate(1 << 20, 4 << 20, 16 << 20)[0] == 0
    for mn, avg, mx in [(64, 256, 1024), (64, 1024, 4096), (256 << 10, 1 << 20, 4 << 20)]:
        assert O.validate(mn, avg, mx)[0] == 0
    for mn, avg, mx, field in [((1 << 20) + 1, 1024, 4096, "min_size"), (64, (4 << 20) + 1, 16 << 20, "avg_size"),
                               (64, 1024, (16 << 20) + 1, "max_size")]:
        st, msg = O.validate(mn, avg, mx)
        assert st == 4 and field in msg
    st, msg = O.validate(32, 64, 128)
    assert st == 4 and "min_size" in msg and "64" in msg
    assert O.validate(64, 64, 64)[0] == 4
    assert O.validate(64, 1024, 64 << 20)[0] == 4


@pytest.mark.parametrize("slice_size", [512, 8_192, 65_536, 400_000, 1_500_000])
def test_push_restatement_matches_eager(slice_size):
    rng = np.random.default_rng(1234)
    data = rng.integers(0, 256, 1_500_000, dtype=np.uint8).tobytes()
    params = (8_192, 32_768, 131_072)
    ref = O.chunk_descriptors(data, *params, algo=B3, nthreads=4)
    p = O.Push(*params, algo=B3, nthreads=1 if slice_size < 100_000 else 4)
    got = []
    for k in range(0, len(data), slice_size):
        got += list(p.push(data[k:k + slice_size]))
    got += list(p.finish())
    assert [(int(g["offset"]), int(g["length"]), bytes(g["hash"])) for g in got] == \
        [(int(r["offset"]), int(r["length"]), bytes(r["hash"])) for r in ref]
    assert p.bytes_consumed() == len(data)


def test_golden_fixtures_reproduce():
    """tests/golden/cdc_golden.json (made by tests/golden/make_golden.py with the
    table recorded in it): the oracle still reproduces every boundary and digest."""
    g = json.loads((GOLDEN / "cdc_golden.json").read_text())
    assert g["gear_sha256"] == hashlib.sha256(O.GEAR.tobytes()).hexdigest(), "table changed: regenerate goldens"
    import sys
    sys.path.insert(0, str(GOLDEN))
    from make_golden import make_input

    for case in g["cases"]:
        data = make_input(case["input"])
        descs = O.chunk_descriptors(data, *case["params"], algo=case["algo"], nthreads=4)
        assert [[int(d["offset"]), int(d["length"]), bytes(d["hash"]).hex()] for d in descs] == case["chunks"]


# --- CAS content ids -------------------------------------
def _keccak_f(a):
    """FIPS 202 Keccak-f[1600], pure Python (a second restatement to pin hashlib)."""
    M = (1 << 64) - 1
    R = [0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14]
    rot = lambda v, n: ((v << n) | (v >> (64 - n))) & M if n else v  # noqa: E731
    rc = 1
    for _ in range(24):
        c = [a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20] for x in range(5)]
        a = [a[i] ^ c[(i % 5 + 4) % 5] ^ rot(c[(i % 5 + 1) % 5], 1) for i in range(25)]
        b = [0] * 25
        for x in range(5):
            for y in range(5):
                b[y + 5 * ((2 * x + 3 * y) % 5)] = rot(a[x + 5 * y], R[x + 5 * y])
        a = [b[i] ^ (~b[(i % 5 + 1) % 5 + 5 * (i // 5)] & b[(i % 5 + 2) % 5 + 5 * (i // 5)]) for i in range(25)]
        # iota: round constant from the LFSR x^8 + x^6 + x^5 + x^4 + 1
        v = 0
        for j in range(7):
            if rc & 1:
                v |= 1 << ((1 << j) - 1)
            rc = ((rc << 1) ^ (0x71 if rc & 0x80 else 0)) & 0xFF
        a[0] ^= v
    return a


def _shake256_py(msg: bytes, n: int = 32) -> bytes:
    rate = 136
    m = bytearray(msg) + b"\x1f"
    m += bytes(-len(m) % rate)
    m[-1] |= 0x80
    a = [0] * 25
    for k in range(0, len(m), rate):
        for i in range(rate // 8):
            a[i] ^= int.from_bytes(m[k + 8 * i:k + 8 * i + 8], "little")
        a = _keccak_f(a)
    return b"".join(x.to_bytes(8, "little") for x in a)[:n]


def test_shake256_kat_and_independent_keccak():
    # crates/core/crypto/src/hash.rs:46-57 (NIST empty-input vector)
    kat = "46b9dd2b0ba88d13233b3feb743eeb243fcd52ea62b81b82b50c27646ed5762f"
    assert O.shake256_256(b"").hex() == kat and _shake256_py(b"").hex() == kat
    # short_digest_is_long_digest_prefix (:59-65)
    assert hashlib.shake_256(b"flakecache").digest(16) == O.shake256_256(b"flakecache")[:16]
    rng = np.random.default_rng(1)
    for n in (1, 109, 110, 111, 135, 136, 137, 271, 272, 273, 1000):
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert O.shake256_256(d) == _shake256_py(d), n


def test_content_id_framing_and_golden():
    """ContentId::compute framing (crates/core/cas/src/lib.rs:59-69) and the committed
    vectors (tests/golden/cas_vectors.json, made by tests/golden/make_cas_vectors.py)."""
    p = b"hello"
    framed = b"flakecache-cas" + b"\x00" + b"\x01" + b"\x01\x00" + (5).to_bytes(8, "little") + p
    assert len(framed) - len(p) == 26
    assert O.content_id(O.KIND_CHUNK, p) == _shake256_py(framed)
    # id_is_deterministic_and_kind_separated (crates/core/cas/src/lib.rs:254-261)
    assert O.content_id(1, p) == O.content_id(1, p) != O.content_id(4, p)
    g = json.loads((GOLDEN / "cas_vectors.json").read_text())
    import sys
    sys.path.insert(0, str(GOLDEN))
    from make_cas_vectors import payload
    for case in g["cases"]:
        assert O.content_id(case["kind"], payload(case["len"], case["seed"])).hex() == case["id"], case


def test_node_put_oracle_structure():
    """Node::put (crates/node/src/lib.rs:114-132): the manifest is the Level1Manifest id of
    the concatenated chunk ids; identical input -> identical manifest (:226-239)."""
    rng = np.random.default_rng(2)
    data = rng.integers(0, 256, 300_000, dtype=np.uint8)
    descs, ids, man = O.node_put(data, 4096, 16_384, 65_536, nthreads=4)
    assert len(ids) == len(descs) > 3
    assert ids == [O.content_id(O.KIND_CHUNK, data[int(d["offset"]):int(d["offset"] + d["length"])])
                   for d in descs]
    assert man == O.content_id(O.KIND_LEVEL1_MANIFEST, b"".join(ids))
    assert O.node_put(data, 4096, 16_384, 65_536)[2] == man
    assert O.node_put(b"", 4096, 16_384, 65_536)[2] == O.content_id(O.KIND_LEVEL1_MANIFEST, b"")

"""GPU parity of the CAS content-id kernel (K5, chunker_amd/csrc/cas.hip) and the
fused Node::put entries against the oracle (hashlib SHAKE-256 over the framing of
crates/core/cas/src/lib.rs:53-69; oracle.node_put restating crates/node/src/lib.rs:114-132).

Bit-exact on every id.  Cases: every message length around the 136-byte SHAKE rate
(framed length = 26 + payload, so payload 109/110/111 straddle the first block and
109 puts the 0x1F and 0x80 pad bits in one byte), all payload alignments mod 4,
every ObjectKind, the reference's own CAS and Node tests
(crates/core/cas/src/lib.rs:254-310, crates/node/src/lib.rs:214-280), empty and
ragged NAR batches, and enough spans to engage the longest-first order.
"""
import contextlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NODE = (4096, 16_384, 65_536)  # Node::with_chunk_sizes in the reference's node tests (lib.rs:210)
D = (256 * 1024, 1024 * 1024, 4 * 1024 * 1024)


@pytest.fixture(scope="module")
def cas(gpu):
    from chunker_amd import cas

    return cas


@pytest.fixture(scope="module")
def O():
    from oracle import oracle

    return oracle


def pseudo_random(seed, n):
    """crates/node/src/lib.rs:192-203 (xorshift64, u64 little-endian words)."""
    out = np.empty((n + 7) // 8, np.uint64)
    s = np.uint64(seed | 1)
    with np.errstate(over="ignore"):
        for i in range(len(out)):
            s ^= s << np.uint64(13)
            s ^= s >> np.uint64(7)
            s ^= s << np.uint64(17)
            out[i] = s
    return out.view(np.uint8)[:n].copy()


def test_shake_kat_and_reference_cas_cases(cas, O):
    # crates/core/crypto/src/hash.rs:46-57 frames nothing; the CAS id of the same
    # empty payload is the framed digest, which the oracle restates
    for kind in cas.ObjectKind:
        for payload in (b"", b"hello", b"some chunk bytes", b"trusted payload", b"payload"):
            assert cas.ContentId.compute(kind, payload).as_bytes() == O.content_id(int(kind), payload)
    # id_is_deterministic_and_kind_separated (crates/core/cas/src/lib.rs:254-261)
    a = cas.ContentId.compute(cas.ObjectKind.Chunk, b"hello")
    b = cas.ContentId.compute(cas.ObjectKind.Chunk, b"hello")
    c = cas.ContentId.compute(cas.ObjectKind.Refcount, b"hello")
    assert a == b and a != c and len(a.to_hex()) == 64


@contextlib.contextmanager
def _pair_max(v):
    """Cap the CAS pair tier (test hook cg_test_cas_pair_max) for the block: -1 = wave
    budget only, 0 = one lane per span everywhere, k = the k longest spans on lane pairs.
    The old cap comes back even when the block fails, so no tier leaks into later tests."""
    from chunker_amd import lib

    old = lib.cg_test_cas_pair_max(v)
    try:
        yield
    finally:
        lib.cg_test_cas_pair_max(old)


TIERS = pytest.mark.parametrize("pair_max", [-1, 0, 37], ids=["pairs", "single", "mixed"])


@TIERS
def test_cas_ids_all_lengths_and_alignments(cas, O, pair_max):
    import torch

    rng = np.random.default_rng(17)
    data = rng.integers(0, 256, 4 << 20, dtype=np.uint8)
    lens = list(range(0, 420)) + [135 * k + d for k in (4, 5, 7, 100) for d in (-1, 0, 1)] + \
        [136 * k - 26 + d for k in (2, 3, 50, 1000) for d in (-1, 0, 1)] + [65_536, 1 << 20, (1 << 20) + 3, 3 << 20]
    offs = [int(rng.integers(0, len(data) - n + 1)) for n in lens]
    d = torch.from_numpy(data).cuda()
    o = torch.tensor(offs, dtype=torch.int64).cuda()
    ln = torch.tensor(lens, dtype=torch.int64).cuda()
    for kind in (cas.ObjectKind.Chunk, cas.ObjectKind.Commit):
        ids = torch.zeros(len(lens) * 32, dtype=torch.uint8, device="cuda")
        with _pair_max(pair_max):
            cas.content_ids_device(d.data_ptr(), o.data_ptr(), ln.data_ptr(), len(lens), kind, ids.data_ptr())
        ids = ids.cpu().numpy().reshape(-1, 32)
        for k, (a, n) in enumerate(zip(offs, lens)):
            assert bytes(ids[k]) == O.content_id(int(kind), data[a:a + n]), (int(kind), n, a)


def test_node_put_matches_oracle(cas, O):
    for seed, n, params in ((42, 500_000, NODE), (7, 400_000, NODE), (11, 120_000, NODE), (3, 0, NODE),
                            (5, 100, NODE), (9, 3_000_017, D)):
        data = pseudo_random(seed, n)
        got = cas.node_put(data, *params)
        descs, ids, man = O.node_put(data, *params)
        assert [(c.offset, c.length, c.hash) for c in got.chunks] == \
            [(int(x["offset"]), int(x["length"]), bytes(x["hash"])) for x in descs], (seed, n)
        assert [i.as_bytes() for i in got.chunk_ids] == ids, (seed, n)
        assert got.manifest.as_bytes() == man, (seed, n)
        assert b"".join(c.payload for c in got.chunks) == data.tobytes()


def test_reference_node_dedup_cases(cas):
    # identical_input_is_fully_deduplicated (crates/node/src/lib.rs:226-239)
    data = pseudo_random(7, 400_000)
    assert cas.node_put(data, *NODE).manifest == cas.node_put(data, *NODE).manifest
    # shared_content_shares_chunks (:241-264)
    base = pseudo_random(1, 400_000)
    extended = np.concatenate([base, pseudo_random(2, 150_000)])
    r1, r2 = cas.node_put(base, *NODE), cas.node_put(extended, *NODE)
    refs = len(r1.chunk_ids) + len(r2.chunk_ids)
    assert len(set(r1.chunk_ids) | set(r2.chunk_ids)) < refs
    # put_get_round_trip: the manifest is the id of the concatenated chunk ids
    r = cas.node_put(pseudo_random(42, 500_000), *NODE)
    assert r.manifest == cas.ContentId.compute(cas.ObjectKind.Level1Manifest,
                                               b"".join(i.as_bytes() for i in r.chunk_ids))


@pytest.mark.parametrize("params", [NODE, D], ids=["node", "D"])
def test_node_put_batch_device(cas, O, params):
    import torch

    import chunker_amd as ca
    from chunker_amd.nar import synth_nars

    sizes = [120, 2 * 1024 * 1024 + 8, 0 + 128, 5 * 1024 * 1024 + 16, 1024 * 1024, 3 * 1024 * 1024 + 40]
    data, offs = synth_nars(sizes, first_index=3)
    # an empty NAR in the middle of the batch
    offs = np.insert(offs, 2, offs[2])
    d = torch.from_numpy(data).cuda()
    cap = ca.chunking.batch_capacity(offs, params[0])
    out = torch.zeros(cap * 48, dtype=torch.uint8, device="cuda")
    ids = torch.zeros(cap * 32, dtype=torch.uint8, device="cuda")
    first, man = cas.node_put_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, ids.data_ptr(), *params)
    descs = out.cpu().numpy().view(ca.DESC_DTYPE)
    ids = ids.cpu().numpy().reshape(-1, 32)
    for i in range(len(offs) - 1):
        ref, rids, rman = O.node_put(data[offs[i]:offs[i + 1]], *params)
        lo, hi = int(first[i]), int(first[i + 1])
        assert np.array_equal(descs[lo:hi]["offset"], ref["offset"]), i
        assert np.array_equal(descs[lo:hi]["length"], ref["length"]), i
        assert np.array_equal(descs[lo:hi]["hash"], ref["hash"]), i
        assert [bytes(x) for x in ids[lo:hi]] == rids, i
        assert bytes(man[i]) == rman, i


@TIERS
def test_cas_many_spans_ordered(cas, O, pair_max):
    """> 64 spans of mixed lengths: the longest-first order path."""
    import torch

    rng = np.random.default_rng(23)
    data = rng.integers(0, 256, 8 << 20, dtype=np.uint8)
    lens = rng.integers(0, 200_000, 700).tolist() + [2 << 20, 1 << 20]
    offs = [int(rng.integers(0, len(data) - n + 1)) for n in lens]
    d = torch.from_numpy(data).cuda()
    o = torch.tensor(offs, dtype=torch.int64).cuda()
    ln = torch.tensor(lens, dtype=torch.int64).cuda()
    ids = torch.zeros(len(lens) * 32, dtype=torch.uint8, device="cuda")
    with _pair_max(pair_max):
        cas.content_ids_device(d.data_ptr(), o.data_ptr(), ln.data_ptr(), len(lens), cas.ObjectKind.Chunk,
                               ids.data_ptr())
    ids = ids.cpu().numpy().reshape(-1, 32)
    want = O.content_ids(data, np.array(list(zip(offs, lens)), dtype=[("offset", "<u8"), ("length", "<u8")]),
                         O.KIND_CHUNK, nthreads=8)
    assert [bytes(x) for x in ids] == want


def test_nar_hashes_device(gpu):
    """Whole-NAR SHA-256 (narinfo NarHash, crates/proto/nix/src/narinfo.rs:127-157) of a
    device batch: one span per NAR, vs hashlib."""
    import hashlib

    import torch

    from chunker_amd.nar import synth_nars
    from chunker_amd.narinfo import nar_hash, nar_hash_field, nar_hashes_device

    data, offs = synth_nars([120, 4096, 3 * 1024 * 1024 + 8, 17 * 1024 * 1024 + 16, 1 << 20], first_index=9)
    d = torch.from_numpy(data).cuda()
    dig = torch.zeros(32 * (len(offs) - 1), dtype=torch.uint8, device="cuda")
    nar_hashes_device(d.data_ptr(), offs, dig.data_ptr())
    dig = dig.cpu().numpy().reshape(-1, 32)
    for i in range(len(offs) - 1):
        want = hashlib.sha256(data[offs[i]:offs[i + 1]].tobytes()).digest()
        assert bytes(dig[i]) == want, i
    one = data[offs[1]:offs[2]].tobytes()
    assert nar_hash(one) == hashlib.sha256(one).digest()
    assert nar_hash_field(nar_hash(one)).startswith("sha256:") and len(nar_hash_field(nar_hash(one))) == 59

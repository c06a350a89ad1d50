"""Batch parts (runtime.hip run_parts, DESIGN.md §4 "Batch parts"): a batch cut at NAR
boundaries into parts whose boundary stages overlap the previous part's digest on a
second stream.  The result must be bit-identical to the whole-batch run and to the
oracle: descriptors, digests and the NAR -> first-chunk index, whichever NAR starts
qualify as cut points (only 16-B aligned ones do), for both digests, through the host
and the device entries.
"""
import numpy as np
import pytest

from test_gpu_parity import B3, D, SHA, assert_same, rand_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ca(gpu):
    import chunker_amd

    return chunker_amd


@pytest.fixture(scope="module")
def O():
    from oracle import oracle

    return oracle


class parts_policy:
    """cg_set_batch_parts for the duration of a block (restored on failure too)."""

    def __init__(self, ca, k):
        self.ca, self.k = ca, k

    def __enter__(self):
        self.prev = self.ca.lib.cg_set_batch_parts(self.k)

    def __exit__(self, *exc):
        self.ca.lib.cg_set_batch_parts(self.prev)


# ragged NARs: most lengths multiples of 16 (aligned cut points), some not (skipped
# cut points), empties, NARs below min and one spanning several max-size chunks
# (odd lengths come in pairs that restore the alignment)
LENS = [0, 160, 1_048_576, 7, 9, 1_000_000, 2_000_016, 0, 333_333, 333_339, 65_536, 4_194_320, 5, 11, 1_500_000, 96,
        3_000_000, 1_048_577, 15, 2_097_152]


@pytest.mark.parametrize("algo", [SHA, B3], ids=["sha256", "blake3"])
@pytest.mark.parametrize("k", [2, 3, 4, 8])
def test_parts_ragged_match_oracle(ca, O, algo, k):
    rng = np.random.default_rng(1234 + k)
    nars = [rng.integers(0, 256, n, dtype=np.uint8) for n in LENS]
    params = (4096, 16384, 65536)
    with parts_policy(ca, k):
        got = ca.chunk_batch(nars, *params, hash=algo)
        used = ca.lib.cg_last_batch_parts()
    assert 2 <= used <= k
    for i, nar in enumerate(nars):
        assert_same(got[i], O.chunk_descriptors(nar, *params, algo=algo), f"k={k} nar{i} len={LENS[i]}")


@pytest.mark.parametrize("algo", [SHA, B3], ids=["sha256", "blake3"])
def test_parts_flat_index_equals_whole_batch(ca, algo):
    """The merged NAR index and descriptor array equal the unsplit run's exactly."""
    rng = np.random.default_rng(7)
    lens = [int(x) * 16 for x in rng.integers(0, 200_000, 40)] + [13, 0, 0, 4096]
    flat = rng.integers(0, 256, sum(lens), dtype=np.uint8)
    offs = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    with parts_policy(ca, 1):
        ref, ref_first = ca.chunking.chunk_batch_flat(flat, offs, 1024, 6000, 16384, hash=algo)
        ref = ref.copy()
        assert ca.lib.cg_last_batch_parts() == 1
    for k in (2, 5, 8):
        with parts_policy(ca, k):
            got, first = ca.chunking.chunk_batch_flat(flat, offs, 1024, 6000, 16384, hash=algo)
            assert ca.lib.cg_last_batch_parts() == k
        assert np.array_equal(first, ref_first), k
        assert np.array_equal(got.view(np.uint8), ref.view(np.uint8)), k


def test_parts_no_aligned_cut_runs_whole(ca, O):
    """No NAR start after the first is 16-B aligned: the batch runs unsplit."""
    lens = [100_001, 100_001, 100_001]
    rng = np.random.default_rng(5)
    nars = [rng.integers(0, 256, n, dtype=np.uint8) for n in lens]
    # offsets 100001 and 200002 are odd: no qualifying cut point
    with parts_policy(ca, 4):
        got = ca.chunk_batch(nars, 1024, 6000, 16384, hash=B3)
        assert ca.lib.cg_last_batch_parts() == 1
    for i, nar in enumerate(nars):
        assert_same(got[i], O.chunk_descriptors(nar, 1024, 6000, 16384, algo=B3), f"nar{i}")


def test_parts_capacity_error(ca):
    """An output array too small for the merged batch fails as it does unsplit."""
    import torch

    from chunker_amd.nar import synth_nars

    sizes = [1 << 20] * 8
    data, offs = synth_nars(sizes, first_index=3)
    d = torch.from_numpy(data).cuda()
    out = torch.zeros(8 * 48, dtype=torch.uint8, device="cuda")  # 8 descriptors: far too few
    for k in (1, 4):
        with parts_policy(ca, k):
            with pytest.raises(ca.ChunkingError, match="too small"):
                ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), 8, 4096, 16384, 65536, hash=B3,
                                      stream=torch.cuda.current_stream().cuda_stream)


def test_parts_by_size_device_blake3(ca, O):
    """Default policy: a >= 256 MiB BLAKE3 batch of several NARs runs as 4 parts on the
    device entry, bit-identical to the unsplit run; SHA-256 batches stay whole."""
    import torch

    from chunker_amd.nar import synth_nars_device

    sizes = np.full(80, 4 << 20, np.uint64)
    sizes[5] += 16
    sizes[39] -= 8  # NAR 40 starts unaligned: the middle cut point moves to NAR 41
    sizes[40] += 8
    d, offs = synth_nars_device(sizes, first_index=11)
    cap = ca.chunking.batch_capacity(offs, D[0])
    stream = torch.cuda.current_stream().cuda_stream
    outs, firsts = [], []
    for k in (0, 1):
        out = torch.zeros(cap * 48, dtype=torch.uint8, device="cuda")
        with parts_policy(ca, k):
            firsts.append(ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *D, hash=B3, stream=stream))
            assert ca.lib.cg_last_batch_parts() == (4 if k == 0 else 1)
        outs.append(out.cpu().numpy())
    assert np.array_equal(firsts[0], firsts[1])
    assert np.array_equal(outs[0], outs[1])
    descs = outs[0].view(ca.DESC_DTYPE)
    host = d.cpu().numpy()
    for i in (0, 5, 39, 40, 79):
        ref = O.chunk_descriptors(host[offs[i]:offs[i + 1]], *D, algo=B3)
        assert_same(descs[int(firsts[0][i]):int(firsts[0][i + 1])], ref, f"nar{i}")
    out = torch.zeros(cap * 48, dtype=torch.uint8, device="cuda")
    ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *D, hash=SHA, stream=stream)
    assert ca.lib.cg_last_batch_parts() == 1


def test_parts_small_batches_and_single_nar(ca, O):
    """Forced parts never split a one-NAR batch; a two-NAR batch splits into two."""
    rng = np.random.default_rng(9)
    one = [rng.integers(0, 256, 3_000_000, dtype=np.uint8)]
    two = [rng.integers(0, 256, 1_000_000, dtype=np.uint8), rng.integers(0, 256, 500_000, dtype=np.uint8)]
    with parts_policy(ca, 8):
        g1 = ca.chunk_batch(one, 4096, 16384, 65536, hash=B3)
        assert ca.lib.cg_last_batch_parts() == 1
        g2 = ca.chunk_batch(two, 4096, 16384, 65536, hash=B3)
        assert ca.lib.cg_last_batch_parts() == 2
    assert_same(g1[0], O.chunk_descriptors(one[0], 4096, 16384, 65536, algo=B3), "one")
    for i in range(2):
        assert_same(g2[i], O.chunk_descriptors(two[i], 4096, 16384, 65536, algo=B3), f"two{i}")

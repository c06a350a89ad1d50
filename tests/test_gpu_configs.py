"""BASELINE.json configs at full size on the GPU, checked against the oracle.

* config 3: 256 x 4 MiB synthetic NARs, default params, BLAKE3 -- every NAR oracle-checked;
* configs 4 / 5 put > 4 GiB into one flat batch buffer: a 5-NAR batch of 1 GiB + 1 MiB
  NARs (NAR 3 straddles the 4 GiB flat offset) at S and at D, SHA-256, the NARs on both
  sides of 4 GiB oracle-checked, every NAR checked for coverage and contiguity;
* config 5's per-GPU shard: 16 x 1 GiB at D (16 GiB in HBM), coverage + contiguity for
  every NAR and oracle checks on a sample including the last NAR (flat offsets ~16 GiB).

Inputs are written straight into HBM NAR group by NAR group (nar.synth_nars_device),
so no test holds the whole batch in host memory.
"""
import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

D = (256 * 1024, 1024 * 1024, 4 * 1024 * 1024)
S = (64 * 1024, 256 * 1024, 1024 * 1024)
GIB = 1 << 30


@pytest.fixture(scope="module")
def ca(gpu):
    import chunker_amd

    return chunker_amd


@pytest.fixture(scope="module")
def O():
    from oracle import oracle

    return oracle


def run_device_batch(ca, sizes, params, algo, first_index):
    import torch

    from chunker_amd.nar import synth_nars_device

    d, offs = synth_nars_device(sizes, first_index=first_index)
    cap = ca.chunking.batch_capacity(offs, params[0])
    out = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
    first = ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params, hash=algo,
                                  stream=torch.cuda.current_stream().cuda_stream)
    descs = out[: int(first[-1]) * 48].cpu().numpy().view(ca.DESC_DTYPE)
    del out
    return d, offs, first, descs


def check_cover(descs, first, offs, params):
    for i in range(len(offs) - 1):
        a, b = int(first[i]), int(first[i + 1])
        nar_len = int(offs[i + 1] - offs[i])
        x = descs[a:b]
        assert b > a and x["offset"][0] == 0, i
        ends = x["offset"] + x["length"]
        assert ends[-1] == nar_len and np.array_equal(x["offset"][1:], ends[:-1]), i
        assert np.all(x["length"][:-1] >= 2 * (params[0] // 2)) and np.all(x["length"] <= params[2]), i


def oracle_check(O, d, offs, first, descs, i, params, algo):
    nar = d[int(offs[i]):int(offs[i + 1])].cpu().numpy()
    ref = O.chunk_descriptors(nar, *params, algo=algo, nthreads=16)
    got = descs[int(first[i]):int(first[i + 1])]
    assert len(got) == len(ref), (i, len(got), len(ref))
    assert np.array_equal(got["offset"], ref["offset"]) and np.array_equal(got["length"], ref["length"]), i
    bad = np.nonzero(~np.all(got["hash"] == ref["hash"], axis=1))[0]
    assert len(bad) == 0, (i, bad[:8])


def test_config3_blake3_full_batch(ca, O):
    sizes = [4 << 20] * 256
    d, offs, first, descs = run_device_batch(ca, sizes, D, 0, 0)
    check_cover(descs, first, offs, D)
    host = d[: int(offs[-1])].cpu().numpy()
    for i in range(len(sizes)):
        ref = O.chunk_descriptors(host[int(offs[i]):int(offs[i + 1])], *D, algo=0, nthreads=16)
        got = descs[int(first[i]):int(first[i + 1])]
        assert len(got) == len(ref) and np.array_equal(got["length"], ref["length"]), i
        assert np.array_equal(got["hash"], ref["hash"]), i


@pytest.mark.parametrize("params", [S, D], ids=["S", "D"])
def test_batch_past_4gib_flat_offsets(ca, O, params):
    sizes = [GIB + (1 << 20) + 8 * k for k in range(5)]  # NAR 3 = [3.003, 4.004) GiB
    d, offs, first, descs = run_device_batch(ca, sizes, params, 1, 40)
    assert offs[3] < 4 * GIB < offs[4] and offs[-1] > 5 * GIB
    check_cover(descs, first, offs, params)
    for i in (3, 4):
        oracle_check(O, d, offs, first, descs, i, params, 1)


def test_config5_shard_16x1gib(ca, O):
    sizes = [GIB] * 16
    d, offs, first, descs = run_device_batch(ca, sizes, D, 1, 48)  # rank 3's shard of 128 NARs
    check_cover(descs, first, offs, D)
    n = int(first[-1])
    assert 16 * 600 < n < 16 * 1100  # ~820 chunks per GiB at D on random data
    for i in (0, 7, 15):
        oracle_check(O, d, offs, first, descs, i, D, 1)


def test_config4_full_16x1gib(ca, O):
    """BASELINE config 4 at full size (16 x 1 GiB at S, SHA-256, the bench's NARs): the
    only shape whose expected chunk count (~54 K) fills the GPU, so the digest runs the
    GPU-filling tier mix (a few quad workgroups for the longest chunks, then pairs, then
    one-lane workgroups, cg_last_sha_tiers).  Every NAR covered contiguously; NARs 0, 7
    and 15 oracle-checked chunk by chunk."""
    import ctypes

    sizes = [GIB] * 16
    d, offs, first, descs = run_device_batch(ca, sizes, S, 1, 0)
    tiers = (ctypes.c_uint32 * 4)()
    assert ca.lib.cg_last_sha_tiers(tiers) == 1
    nquad, npair, nlane, _ = (int(t) for t in tiers)
    assert 0 < nquad < 256 and npair > 0 and nlane > 0, list(tiers)
    check_cover(descs, first, offs, S)
    n = int(first[-1])
    assert 16 * 2600 < n < 16 * 4000  # ~3.3 K chunks per GiB at S on random data
    for i in (0, 7, 15):
        oracle_check(O, d, offs, first, descs, i, S, 1)

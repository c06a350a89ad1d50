"""Randomized parity sweep over the device entries (slow): random valid options, ragged
batches of 1..64 NARs of random / low-entropy / zero-run / fixture-pattern bytes, both
digests, through the queued-batch pair (cg_chunk_batch_device_async[_after] + cg_batch_wait: NAR
index written into mapped host memory, host tables through the stage-in kernel, the
BLAKE3 group map from the assembly) and the host entry; every NAR bit-exact vs the oracle.
In the spirit of the reference's tests/proptest_suite.rs and fuzz/fuzz_targets/chunking.rs.
"""
import os

import numpy as np
import pytest

from test_gpu_parity import B3, SHA, _random_nar, _random_options, assert_same

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


@pytest.fixture(scope="module")
def ca(gpu):
    import chunker_amd

    return chunker_amd


@pytest.fixture(scope="module")
def O():
    from oracle import oracle

    return oracle


# CHUNKER_AMD_FUZZ_SEEDS widens the sweep for a dedicated run (profiles/r03_v36_fuzz_*)
@pytest.mark.parametrize("seed", range(int(os.environ.get("CHUNKER_AMD_FUZZ_SEEDS", "96"))))
def test_fuzz_device_batches(ca, O, seed):
    import torch

    rng = np.random.default_rng(7000 + seed)
    params = _random_options(rng, large=seed % 3 != 0)
    n = int(rng.choice([1, 2, 3, 7, 16, 33, 64]))
    sizes = [int(x) for x in rng.integers(0, 2 * 1024 * 1024, n)]
    if seed % 8 == 0:
        sizes[int(rng.integers(0, n))] = int(rng.integers(17, 40)) * 1024 * 1024 + int(rng.integers(0, 999))
    nars = [_random_nar(rng, s) for s in sizes]
    offs = np.zeros(n + 1, np.uint64)
    np.cumsum(sizes, out=offs[1:])
    flat = np.concatenate(nars) if sum(sizes) else np.zeros(0, np.uint8)
    d = torch.from_numpy(np.concatenate([flat, np.zeros(256, np.uint8)])).cuda()
    cap = max(ca.chunking.batch_capacity(offs, params[0]), 1)
    stream = torch.cuda.current_stream().cuda_stream
    for algo in (SHA, B3):
        outs = [torch.zeros(cap * 48, dtype=torch.uint8, device="cuda") for _ in range(2)]
        # two queued batches on one stream, the second waited for first; on odd seeds the
        # second is ordered after an inputs-ready event only (cg_chunk_batch_device_async_after,
        # the bench's path), so it runs beside the first
        ready = torch.cuda.Event()  # (recorded before `a` is queued: it does not wait for `a`)
        ready.record()
        a = ca.chunk_batch_device_async(d.data_ptr(), offs, outs[0].data_ptr(), cap, *params, hash=algo,
                                        stream=stream)
        b = ca.chunk_batch_device_async(d.data_ptr(), offs, outs[1].data_ptr(), cap, *params, hash=algo,
                                        stream=stream, inputs_ready=ready.cuda_event if seed % 2 else 0)
        fb, fa = b.wait(), a.wait()
        assert np.array_equal(fa, fb)
        ga, gb = outs[0].cpu().numpy(), outs[1].cpu().numpy()
        m = int(fa[-1]) * 48
        assert np.array_equal(ga[:m], gb[:m])
        descs = ga.view(ca.DESC_DTYPE)
        host = ca.chunk_batch(nars, *params, hash=algo)
        for i, nar in enumerate(nars):
            ref = O.chunk_descriptors(nar, *params, algo=algo)
            ctx = f"seed={seed} {params} algo={algo} nar{i} len={len(nar)}"
            assert_same(descs[int(fa[i]):int(fa[i + 1])], ref, ctx)
            assert_same(host[i], ref, ctx + " (host entry)")

"""GPU robustness of the engine behind the C ABI: concurrent callers, failure
reporting, and the reference's error variants with their fields.

* Re-entrancy (include/chunker_gpu.h "Threading"): the reference's callers are
  concurrent -- thread-per-connection HTTP (crates/proto/nix/src/lib.rs:153-162),
  BEAM dirty schedulers, rayon -- so 8 host threads chunk distinct inputs at once,
  through the host entry and through the device entry on 8 distinct streams; every
  result equals the oracle's.
* The SHA-256 producer/consumer spin guard (sha256.hip) reports an expired wait as
  CG_E_IO instead of returning digests computed from a stale ring slot.
* BufferLimitExceeded{attempted, limit} (src/chunking.rs:49-50) carries its fields.
"""
import ctypes
import os
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = (16_384, 65_536, 262_144)


@pytest.fixture(scope="module")
def ca(gpu):
    import chunker_amd

    return chunker_amd


@pytest.fixture(scope="module")
def O():
    from oracle import oracle

    return oracle


def _same(got, ref):
    return (len(got) == len(ref) and np.array_equal(got["offset"], ref["offset"])
            and np.array_equal(got["length"], ref["length"]) and np.array_equal(got["hash"], ref["hash"]))


@pytest.mark.parametrize("algo", [1, 0], ids=["sha256", "blake3"])
def test_concurrent_host_callers(ca, O, algo):
    from chunker_amd.nar import synth_nars

    n_threads, per = 8, 6
    batches = []
    for t in range(n_threads):
        sizes = [(3 << 20) + 8 * ((t * 7 + k) % 13) for k in range(per)]
        data, offs = synth_nars(sizes, first_index=100 + t * per)
        batches.append((data, offs))
    results, errors = [None] * n_threads, []
    start = threading.Barrier(n_threads)

    def work(t):
        try:
            data, offs = batches[t]
            start.wait()
            for _ in range(2):  # twice: workspaces are recycled between callers
                results[t] = ca.chunk_batch([data[offs[i]:offs[i + 1]] for i in range(per)], *P, hash=algo)
        except Exception as e:  # noqa: BLE001
            errors.append((t, repr(e)))

    th = [threading.Thread(target=work, args=(t,)) for t in range(n_threads)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=100)
    assert not errors, errors
    for t, (data, offs) in enumerate(batches):
        for i in range(per):
            ref = O.chunk_descriptors(data[offs[i]:offs[i + 1]], *P, algo=algo, nthreads=8)
            assert _same(results[t][i], ref), (t, i)


def test_concurrent_device_callers_on_distinct_streams(ca, O):
    import torch

    from chunker_amd.nar import synth_nars

    n_threads, per = 8, 4
    jobs = []
    for t in range(n_threads):
        sizes = [(4 << 20) + 8 * k for k in range(per)]
        data, offs = synth_nars(sizes, first_index=300 + t * per)
        d = torch.from_numpy(data).cuda()
        cap = ca.chunking.batch_capacity(offs, P[0])
        out = torch.zeros(cap * 48, dtype=torch.uint8, device="cuda")
        jobs.append((data, offs, d, out, cap, torch.cuda.Stream()))
    torch.cuda.synchronize()
    firsts, errors = [None] * n_threads, []
    start = threading.Barrier(n_threads)

    def work(t):
        try:
            data, offs, d, out, cap, s = jobs[t]
            start.wait()
            firsts[t] = ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *P, stream=s.cuda_stream)
        except Exception as e:  # noqa: BLE001
            errors.append((t, repr(e)))

    th = [threading.Thread(target=work, args=(t,)) for t in range(n_threads)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=100)
    assert not errors, errors
    torch.cuda.synchronize()
    for t, (data, offs, d, out, cap, s) in enumerate(jobs):
        descs = out.cpu().numpy().view(ca.DESC_DTYPE)
        first = firsts[t]
        for i in range(per):
            ref = O.chunk_descriptors(data[offs[i]:offs[i + 1]], *P, algo=1, nthreads=8)
            assert _same(descs[int(first[i]):int(first[i + 1])], ref), (t, i)


def _coalesced_jobs(ca, n_threads, seed):
    """Per thread: a batch of a few NARs of different shapes (ragged, tiny, one empty,
    one holding several max-size chunks) on its own stream."""
    import torch

    rng = np.random.default_rng(seed)
    jobs = []
    for t in range(n_threads):
        lens = [int(x) for x in rng.integers(1, 3 << 20, 3)] + [0, 77, 2 * P[2] + 5]
        nars = [rng.integers(0, 256, n, dtype=np.uint8) for n in lens]
        offs = np.zeros(len(nars) + 1, np.uint64)
        np.cumsum(lens, out=offs[1:])
        data = np.concatenate(nars)
        d = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).cuda()
        cap = ca.chunking.batch_capacity(offs, P[0])
        out = torch.zeros(cap * 48, dtype=torch.uint8, device="cuda")
        jobs.append((nars, offs, d, out, cap, torch.cuda.Stream()))
    torch.cuda.synchronize()
    return jobs


def _run_threads(ca, jobs, reps=1):
    firsts, errors = [None] * len(jobs), []
    start = threading.Barrier(len(jobs))

    def work(t):
        try:
            nars, offs, d, out, cap, s = jobs[t]
            start.wait()
            for _ in range(reps):
                firsts[t] = ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *P, stream=s.cuda_stream)
        except Exception as e:  # noqa: BLE001
            errors.append((t, e))

    th = [threading.Thread(target=work, args=(t,)) for t in range(len(jobs))]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=200)
    return firsts, errors


@pytest.mark.parametrize("coalesce", [1, 0], ids=["coalesced", "per_batch"])
def test_concurrent_sha_callers_share_one_digest(ca, O, coalesce):
    """Round 4 coalescer: concurrent callers of the synchronous device entry have their
    SHA-256 digests merged into one launch (runtime.hip coalesced_sha256); every caller
    still gets exactly its own batch's oracle descriptors (digests scattered back to the
    right arrays, empty NARs and max-size chunks included), over several rounds of
    groups; and the same with coalescing off (cg_test_coalesce)."""
    import torch

    old = ca.lib.cg_test_coalesce(coalesce)
    try:
        jobs = _coalesced_jobs(ca, 12, seed=5 + coalesce)
        firsts, errors = _run_threads(ca, jobs, reps=3)
    finally:
        ca.lib.cg_test_coalesce(old)
    assert not errors, errors
    torch.cuda.synchronize()
    for t, (nars, offs, d, out, cap, s) in enumerate(jobs):
        descs = out.cpu().numpy().view(ca.DESC_DTYPE)
        first = firsts[t]
        for i, nar in enumerate(nars):
            ref = O.chunk_descriptors(nar, *P, algo=1, nthreads=8)
            assert _same(descs[int(first[i]):int(first[i + 1])], ref), (t, i)


def _merging_callers():
    """More concurrent callers than the coalescer lets launch alone (runtime.hip coal_min:
    the process's hardware queues less 4, at least 4): 12 at HIP's default 4 queues."""
    try:
        q = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
    except ValueError:
        q = 4
    return max(12, max(q - 4, 4) + 8)


def _coal_stats(ca):
    out = (ctypes.c_uint64 * 4)()
    ca.lib.cg_coalesce_stats(out)
    return [int(x) for x in out]  # groups, members, leader wait us, windows run out


def test_lone_and_few_callers_never_wait_for_the_window(ca, O):
    """The coalescer's latency cost: a lone SHA-256 caller, calling
    back to back, and no more concurrent callers than per-batch launches run side by side
    (runtime.hip coal_min: 4 at HIP's default 4 hardware queues) never enter a merged group, so no leader window
    delays them (cg_coalesce_stats: no group formed, no window run out); 12 callers do form
    groups, and every result is oracle-exact."""
    import torch

    old = ca.lib.cg_test_coalesce(1)
    try:
        jobs = _coalesced_jobs(ca, _merging_callers(), seed=21)
        time.sleep(0.1)  # (callers that returned within the last 50 ms count as expected back)
        s0 = _coal_stats(ca)
        _, errors = _run_threads(ca, jobs[:1], reps=4)  # a lone caller
        assert not errors, errors
        s1 = _coal_stats(ca)
        assert s1 == s0, (s0, s1)
        time.sleep(0.1)
        _, errors = _run_threads(ca, jobs[:4], reps=2)  # a few callers
        assert not errors, errors
        s2 = _coal_stats(ca)
        assert s2 == s1, (s1, s2)
        firsts, errors = _run_threads(ca, jobs, reps=2)  # 12+ callers: merged groups
        assert not errors, errors
        s3 = _coal_stats(ca)
        assert s3[0] > s2[0] and 2 <= s3[1] - s2[1] <= 2 * len(jobs), (s2, s3)
    finally:
        ca.lib.cg_test_coalesce(old)
    torch.cuda.synchronize()
    for t, (nars, offs, d, out, cap, s) in enumerate(jobs):
        descs = out.cpu().numpy().view(ca.DESC_DTYPE)
        first = firsts[t]
        for i, nar in enumerate(nars):
            ref = O.chunk_descriptors(nar, *P, algo=1, nthreads=8)
            assert _same(descs[int(first[i]):int(first[i + 1])], ref), (t, i)


def test_sixteen_hardware_queues():
    """The deployment setting DESIGN.md §7 / INTEGRATION.md recommend for concurrent
    callers, GPU_MAX_HW_QUEUES=16, in a fresh process (HIP reads it once, at start): 20
    concurrent device callers with merged digests, 12 with per-batch launches, 12 with
    coalescing off, and a ChunkStream using
    all 8 of its digest lanes (one HIP stream each, queues - 2), all oracle-exact
    (tests/hw16_child.py)."""
    import subprocess
    import sys

    env = dict(os.environ, GPU_MAX_HW_QUEUES="16", CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR="1")
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hw16_child.py")
    r = subprocess.run([sys.executable, child], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "hw16 ok" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])


def test_coalesced_spin_guard_reaches_every_member(ca):
    """A spin-guard expiry inside a merged digest fails every member's call with CG_E_IO
    (the merged launch's error word is copied into each member's), and the next round is
    exact again."""
    jobs = _coalesced_jobs(ca, _merging_callers(), seed=9)  # past coal_min: the merged path
    old = ca.lib.cg_test_sha_spin_limit(0)
    try:
        _, errors = _run_threads(ca, jobs)
    finally:
        ca.lib.cg_test_sha_spin_limit(old)
    assert len(errors) == len(jobs) and all(isinstance(e, ca.IoError) for _, e in errors), errors
    firsts, errors = _run_threads(ca, jobs)
    assert not errors, errors


def test_sha_spin_guard_timeout_is_an_error(ca, O):
    """With the spin limit forced to 0 every hand-off wait expires at once: the kernel
    finishes (no hang) but flags the launch, and the call fails with CG_E_IO instead of
    returning digests read from stale LDS ring slots.  Restored, the same call is exact."""
    data = np.random.default_rng(11).integers(0, 256, 6 << 20, dtype=np.uint8)
    old = ca.lib.cg_test_sha_spin_limit(0)
    try:
        with pytest.raises(ca.IoError, match="spin guard"):
            ca.chunk_descriptors_array(data, *P)
        assert ca._lib.last_error_detail()[0] == 2
    finally:
        ca.lib.cg_test_sha_spin_limit(old)
    assert _same(ca.chunk_descriptors_array(data, *P), O.chunk_descriptors(data, *P, algo=1, nthreads=8))


def test_buffer_limit_fields(ca):
    """A device batch too large for HBM: BufferLimitExceeded{attempted, limit} with the
    failed allocation's size and the device's free bytes (no kernel is launched)."""
    import torch

    free, _ = torch.cuda.mem_get_info()
    d = torch.zeros(1024, dtype=torch.uint8, device="cuda")
    offs = np.array([0, 1 << 50], np.uint64)  # claims a 1 PiB batch
    with pytest.raises(ca.BufferLimitExceededError) as ei:
        ca.chunk_batch_device(d.data_ptr(), offs, d.data_ptr(), 1)
    e = ei.value
    assert e.attempted > free and 0 < e.limit <= free + (64 << 20)
    assert str(e) == f"buffer_limit_exceeded: attempted {e.attempted} bytes, limit {e.limit} bytes"
    # the engine is still usable afterwards
    assert len(ca.chunk_descriptors(b"hello world")) == 1


def test_push_handle_survives_a_failed_push(ca):
    """A push that fails inside the engine leaves the handle as it was: the
    same slice pushed again continues the stream exactly."""
    data = np.random.default_rng(5).integers(0, 256, 2_000_000, dtype=np.uint8).tobytes()
    params = (8_192, 32_768, 131_072)
    want = ca.chunk_data(data, *params)
    pc = ca.PushChunker(*params)
    got = list(pc.push(data[:700_000]))
    old = ca.lib.cg_test_sha_spin_limit(0)
    try:
        with pytest.raises(ca.IoError):
            pc.push(data[700_000:1_400_000])
    finally:
        ca.lib.cg_test_sha_spin_limit(old)
    got += pc.push(data[700_000:1_400_000])
    got += pc.push(data[1_400_000:])
    got += pc.finish()
    assert got == want
    assert b"".join(c.payload for c in got) == data


@pytest.mark.parametrize("nth", [1, 2])
def test_push_handle_survives_failed_buffer_growth(ca, nth):
    """a push that has to grow the device buffers and runs out of memory on
    the first (nth=1) or the second (nth=2) of the two allocations reports
    BufferLimitExceeded and leaves the handle holding its retained tail: the same slice
    pushed again continues the stream exactly."""
    data = np.random.default_rng(11).integers(0, 256, 3_000_000, dtype=np.uint8).tobytes()
    params = (8_192, 32_768, 131_072)
    want = ca.chunk_data(data, *params)
    pc = ca.PushChunker(*params)
    got = list(pc.push(data[:50_000]))
    big = data[50_000:2_600_000]  # far past the buffers sized for the first push
    ca.lib.cg_test_fail_alloc(nth)
    try:
        with pytest.raises(ca.BufferLimitExceededError):
            pc.push(big)
    finally:
        ca.lib.cg_test_fail_alloc(0)
    got += pc.push(big)
    got += pc.push(data[2_600_000:])
    got += pc.finish()
    assert got == want
    assert b"".join(c.payload for c in got) == data


def test_async_batches_from_threads(ca, O):
    """Four host threads, each keeping two asynchronous batches queued on its own stream
    (cg_chunk_batch_device_async / cg_batch_wait): every batch equals the synchronous
    result, whatever the interleaving of launches and waits across threads."""
    import threading

    import torch

    from chunker_amd.nar import synth_nars

    params = (4096, 16384, 65536)
    data, offs = synth_nars([1 << 20] * 6 + [300_016], first_index=77)
    d = torch.from_numpy(data).cuda()
    cap = ca.chunking.batch_capacity(offs, params[0])
    refs = {}
    for algo in (0, 1):
        out = torch.zeros(cap * 48, dtype=torch.uint8, device="cuda")
        first = ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params, hash=algo)
        refs[algo] = (first, out.cpu().numpy()[: int(first[-1]) * 48].copy())
    errs = []

    def work(t):
        try:
            s = torch.cuda.Stream()
            outs = [torch.zeros(cap * 48, dtype=torch.uint8, device="cuda") for _ in range(2)]
            # the zero fills run on torch's current stream, the batches on `s` (non-blocking):
            # without this the fill could land after a batch's descriptors
            torch.cuda.current_stream().synchronize()
            algo = t % 2
            pending = ca.chunk_batch_device_async(d.data_ptr(), offs, outs[0].data_ptr(), cap, *params, hash=algo,
                                                  stream=s.cuda_stream)
            for k in range(6):
                nxt = ca.chunk_batch_device_async(d.data_ptr(), offs, outs[(k + 1) % 2].data_ptr(), cap, *params,
                                                  hash=algo, stream=s.cuda_stream)
                first = pending.wait()
                got = outs[k % 2].cpu().numpy()[: int(first[-1]) * 48]
                if not (np.array_equal(first, refs[algo][0]) and np.array_equal(got, refs[algo][1])):
                    errs.append(f"thread {t} step {k}")
                pending = nxt
            pending.wait()
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs[:4]

"""GPU: the digest pipeline (cg_pipeline_*, chunker_amd.BatchPipeline; pipeline.hip).

One caller's SHA-256 batches are digested G at a time by ONE merged k_sha256 launch
(k_pipe_merge + per-member completion words), BLAKE3 batches in submission order on the
pipeline's boundary stream.  Every batch must equal the synchronous per-batch entry
(cg_chunk_batch_device) and the CPU oracle, bit for bit, whatever group it landed in, its
position in the group, the order of the waits, and how the group was launched (full, a
wait on an open group, an explicit flush, the pipeline's destruction).
"""
import ctypes
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHA, B3 = 1, 0
P16 = (16384, 65536, 262144)


@pytest.fixture(scope="module")
def ca(gpu):
    import chunker_amd

    return chunker_amd


@pytest.fixture(scope="module")
def O():
    from oracle import oracle

    return oracle


def assert_same(got, ref, ctx=""):
    assert len(got) == len(ref), f"{ctx}: {len(got)} chunks vs oracle {len(ref)}"
    assert np.array_equal(got["offset"], ref["offset"]), ctx
    assert np.array_equal(got["length"], ref["length"]), ctx
    bad = np.nonzero(~np.all(got["hash"] == ref["hash"], axis=1))[0]
    assert len(bad) == 0, f"{ctx}: digest mismatch at chunks {bad[:8]}"


def make_batch(ca, sizes, seed, params, algo=SHA, zeros=False):
    """A device batch of synthetic NARs (distinct per seed) with its reference results from
    the synchronous entry."""
    import torch

    from chunker_amd.nar import synth_nars

    if len(sizes):
        data, offs = synth_nars(sizes, first_index=1000 * seed, zeros=zeros)
    else:
        data, offs = np.zeros(0, np.uint8), np.zeros(1, np.uint64)
    cap = max(ca.chunking.batch_capacity(offs, params[0]), 1)
    d = torch.from_numpy(np.concatenate([data, np.zeros(256, np.uint8)])).cuda()
    ref_out = torch.zeros(cap * 48, dtype=torch.uint8, device="cuda")
    ref_first = ca.chunk_batch_device(d.data_ptr(), offs, ref_out.data_ptr(), cap, *params, hash=algo)
    return {"d": d, "offs": offs, "cap": cap, "algo": algo, "params": params, "data": data,
            "ref_first": ref_first, "ref": ref_out.cpu().numpy(),
            "out": torch.full((cap * 48,), 0xAB, dtype=torch.uint8, device="cuda")}


def check_batch(ca, O, b, first, ctx, oracle_nars=None):
    assert np.array_equal(first, b["ref_first"]), ctx
    n = int(first[-1])
    got = b["out"].cpu().numpy()
    assert np.array_equal(got[: n * 48], b["ref"][: n * 48]), ctx
    descs = got.view(ca.DESC_DTYPE)
    offs = b["offs"]
    nars = range(len(offs) - 1) if oracle_nars is None else oracle_nars
    for i in nars:
        want = O.chunk_descriptors(b["data"][offs[i]:offs[i + 1]], *b["params"], algo=b["algo"])
        assert_same(descs[int(first[i]):int(first[i + 1])], want, f"{ctx} nar{i}")


SHAPES = [
    [1 << 20, 1 << 20, 300_008],          # ordinary
    [],                                    # no NARs at all
    [120, 128, 4096 + 8],                  # tiny NARs: one chunk each
    [2 << 20, 8 * 12345 + 120, 200],       # ragged, unaligned NAR starts
    [3 << 20],                              # one NAR
    [1 << 20] * 9,
    [512 * 1024 + 8, 4096 + 16],
]


@pytest.mark.parametrize("group,lanes", [(3, 2), (1, 1), (7, 3), (64, 2)], ids=["g3l2", "g1l1", "g7l3", "g64l2"])
def test_pipeline_groups_match_oracle(ca, O, group, lanes):
    """Batches of every shape (none, tiny, ragged, one NAR) in merged groups of `group`:
    each equals the synchronous entry and the oracle on every NAR, in submission order."""
    batches = [make_batch(ca, s, k + 1, P16) for k, s in enumerate(SHAPES * 2)]
    results = []
    with ca.BatchPipeline(len(batches) + 1, *P16, group=group, lanes=lanes) as pipe:
        for k, b in enumerate(batches):
            results += pipe.submit(b["d"].data_ptr(), b["offs"], b["out"].data_ptr(), b["cap"], tag=k)
        results += pipe.drain()
        st = pipe.stats()
    assert [t for t, _ in results] == list(range(len(batches)))
    assert st["batches"] == len(batches) and st["groups"] == -(-len(batches) // group)
    for k, first in results:
        check_batch(ca, O, batches[k], first, f"batch{k}")


def _raw_pipeline(ca, group, lanes, device=-1):
    h = ctypes.c_void_p()
    rc = ca.lib.cg_pipeline_create(device, group, lanes, ctypes.byref(h))
    return rc, h.value


def _raw_submit(ca, p, b, ready=0):
    h = ctypes.c_void_p()
    o = b["params"]
    rc = ca.lib.cg_pipeline_submit(ctypes.c_void_p(p), ctypes.c_void_p(b["d"].data_ptr()), b["offs"].ctypes.data,
                                   len(b["offs"]) - 1, o[0], o[1], o[2], b["algo"],
                                   ctypes.c_void_p(b["out"].data_ptr()), b["cap"], ctypes.c_void_p(ready or None),
                                   ctypes.byref(h))
    assert rc == 0, ca.chunking._lib.last_error()
    return ca.chunking.BatchInFlight(h.value, len(b["offs"]) - 1)


def test_pipeline_waits_in_any_order_and_destroy(ca, O):
    """Raw C ABI: waits in reverse order (the first wait launches the open group), batches
    of a full group waited before the next group is flushed, batches still queued when
    the pipeline is destroyed (destroy launches their group; they are waited for after),
    cg_batch_event on an open group, mixed SHA-256 / BLAKE3 submissions."""
    import torch

    batches = [make_batch(ca, [1 << 20, 600_008], 40 + k, P16, algo=(B3 if k in (2, 5) else SHA)) for k in range(8)]
    rc, p = _raw_pipeline(ca, 3, 2)
    assert rc == 0
    hs = [_raw_submit(ca, p, b) for b in batches[:5]]
    for k in (4, 3, 0, 2, 1):  # batch 4 (SHA) and 3 sit in the open group: the wait launches it
        check_batch(ca, O, batches[k], hs[k].wait(), f"batch{k}")
    hs = [_raw_submit(ca, p, b) for b in batches[5:]]
    ev = ctypes.c_void_p()
    assert ca.lib.cg_batch_event(ctypes.c_void_p(hs[2]._h), ctypes.byref(ev)) == 0 and ev.value
    torch.cuda.synchronize()
    ca.lib.cg_pipeline_destroy(ctypes.c_void_p(p))
    for k, h in zip(range(5, 8), hs):
        check_batch(ca, O, batches[k], h.wait(), f"batch{k} after destroy")


def test_pipeline_inputs_ready_on_copy_stream(ca, O):
    """Each batch's input arrives by a pinned H2D copy on ANOTHER stream; the pipeline's
    boundary stream waits only for that copy's event.  One pipeline takes SHA-256 and
    BLAKE3 batches (the algorithm is per submit in the C ABI; BatchPipeline has one)."""
    import torch

    copy = torch.cuda.Stream()
    batches = [make_batch(ca, [4 << 20] * 3 + [8 * k + 4096], 60 + k, P16, algo=(B3 if k % 3 == 1 else SHA))
               for k in range(6)]
    for b in batches:  # fresh device buffers, written only by the copy stream
        b["host"] = torch.from_numpy(b["data"]).pin_memory()
        b["d"] = torch.empty(len(b["data"]) + 256, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    rc, p = _raw_pipeline(ca, 2, 2)
    assert rc == 0
    hs, evs = [], []
    try:
        for b in batches:
            with torch.cuda.stream(copy):
                b["d"][: len(b["data"])].copy_(b["host"], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
            evs.append(ev)
            hs.append(_raw_submit(ca, p, b, ready=ev.cuda_event))
        firsts = [h.wait() for h in hs]
    finally:
        ca.lib.cg_pipeline_destroy(ctypes.c_void_p(p))
    for k, first in enumerate(firsts):
        check_batch(ca, O, batches[k], first, f"batch{k}", oracle_nars=[0, 3])


def test_async_after_blake3_waits_for_inputs_ready(ca, O):
    """cg_chunk_batch_device_async_after with a BLAKE3 batch queued FIRST on an idle stream,
    its input copied on a separate non-blocking stream: the batch must wait for the copy's
    event as well as stream order (the event was ignored for BLAKE3)."""
    import torch

    b = make_batch(ca, [8 << 20] * 4, 77, P16, algo=B3)
    host = torch.from_numpy(b["data"]).pin_memory()
    d = torch.empty(len(b["data"]) + 256, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    copy = torch.cuda.Stream()
    idle = torch.cuda.Stream()
    with torch.cuda.stream(copy):
        torch.cuda._sleep(50_000_000)  # hold the copy back (~20-50 ms)
        d[: len(b["data"])].copy_(host, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
    h = ca.chunk_batch_device_async(d.data_ptr(), b["offs"], b["out"].data_ptr(), b["cap"], *P16, hash=B3,
                                    stream=idle.cuda_stream, inputs_ready=ev.cuda_event)
    check_batch(ca, O, b, h.wait(), "blake3 after copy", oracle_nars=[0])


def test_pipeline_member_completes_before_its_group(ca):
    """Per-member completion: in one merged group, a batch of small chunks is handed back
    long before a batch holding 16 MiB chunks (all-zero payloads: no cut before max_size;
    ~0.27 s SHA-256 chains) completes.  A member completes when the last workgroup holding
    one of its chunks ends; the length order fills the one quad workgroup with the big
    batch's eight 16 MiB chunks, so the small chunks share no workgroup with them."""
    P = (1 << 20, 4 << 20, 16 << 20)
    big = make_batch(ca, [(16 << 20) + 4096] * 8, 90, P, zeros=True)
    small = make_batch(ca, [256 * 1024] * 4, 91, P)
    lens = big["ref"].view(ca.DESC_DTYPE)["length"][: int(big["ref_first"][-1])]
    assert int((lens == 16 << 20).sum()) == 8 and int(lens.max()) == 16 << 20
    longest = int(lens.max())
    rc, p = _raw_pipeline(ca, 2, 1)
    assert rc == 0
    try:
        t0 = time.perf_counter()
        hb = _raw_submit(ca, p, big)
        hs = _raw_submit(ca, p, small)  # the group is full: one merged launch
        fs = hs.wait()
        t_small = time.perf_counter() - t0
        fb = hb.wait()
        t_big = time.perf_counter() - t0
    finally:
        ca.lib.cg_pipeline_destroy(ctypes.c_void_p(p))
    assert np.array_equal(fs, small["ref_first"]) and np.array_equal(fb, big["ref_first"])
    n = int(fb[-1])
    assert np.array_equal(big["out"].cpu().numpy()[: n * 48], big["ref"][: n * 48])
    assert t_small < 0.5 * t_big, (t_small, t_big, longest)


def test_pipeline_spin_guard_and_capacity_errors(ca):
    """A spin-guard expiry in the merged digest fails each member's wait with CG_E_IO; a
    member whose output array is too small fails with CG_E_CAPACITY at its wait while the
    other members of its group succeed; the pipeline stays usable."""
    bs = [make_batch(ca, [1 << 20, 300_008], 95 + k, P16) for k in range(3)]
    with ca.BatchPipeline(8, *P16, group=3, lanes=1) as pipe:
        pipe._open(int(bs[0]["offs"][-1]))
        old = ca.lib.cg_test_sha_spin_limit(0)
        try:
            hs = [ca.chunking.pipeline_submit(pipe._p, b["d"].data_ptr(), b["offs"], b["out"].data_ptr(), b["cap"],
                                              pipe.options, pipe.hash) for b in bs]
            for h in hs:
                with pytest.raises(ca.IoError, match="spin guard"):
                    h.wait()
        finally:
            ca.lib.cg_test_sha_spin_limit(old)
        small = ca.chunking.pipeline_submit(pipe._p, bs[0]["d"].data_ptr(), bs[0]["offs"], bs[0]["out"].data_ptr(), 2,
                                            pipe.options, pipe.hash)
        ok = [ca.chunking.pipeline_submit(pipe._p, b["d"].data_ptr(), b["offs"], b["out"].data_ptr(), b["cap"],
                                          pipe.options, pipe.hash) for b in bs[1:]]
        with pytest.raises(ca.ChunkingError, match="too small"):
            small.wait()
        for b, h in zip(bs[1:], ok):
            assert np.array_equal(h.wait(), b["ref_first"])


def test_pipeline_device_argument(ca):
    """A pipeline on an explicit device index runs there and leaves the caller's current
    device alone; an index past the visible devices is CG_E_NO_DEVICE; bad group / lanes
    are InvalidOptions."""
    import torch

    b = make_batch(ca, [1 << 20], 99, P16)
    rc, p = _raw_pipeline(ca, 4, 2, device=0)
    assert rc == 0
    try:
        h = _raw_submit(ca, p, b)
        assert np.array_equal(h.wait(), b["ref_first"])
        assert torch.cuda.current_device() == 0
    finally:
        ca.lib.cg_pipeline_destroy(ctypes.c_void_p(p))
    rc, _ = _raw_pipeline(ca, 4, 2, device=torch.cuda.device_count())
    assert rc == ca._lib.CG_E_NO_DEVICE
    assert _raw_pipeline(ca, 65, 2)[0] == ca._lib.CG_E_INVALID_OPTIONS
    assert _raw_pipeline(ca, 4, 9)[0] == ca._lib.CG_E_INVALID_OPTIONS


@pytest.mark.slow
def test_pipeline_bench_shape_distinct_c2(ca, O):
    """The shape bench.py times: BASELINE config 2 batches (256 x 4 MiB NARs, 256K/1M/4M)
    through the default BatchPipeline (group 24, 3 lanes, depth 96) over depth + 4 DISTINCT
    batches, each in its own input and output array, at this process's hardware queues
    (HIP's default 4: the pipeline needs no more).  Every batch equals the per-batch entry
    on the same input, and one sampled NAR of every batch equals the oracle."""
    import torch

    from chunker_amd.nar import synth_nars_device

    params = (256 << 10, 1 << 20, 4 << 20)
    sizes = np.full(256, 4 << 20, np.uint64)
    pipe = ca.BatchPipeline(None, *params)
    depth = ((ca.chunking.default_lanes(SHA, int(sizes.sum())) + 1)
             * ca.chunking.default_group(SHA, int(sizes.sum())))
    nb = depth + 4
    ins, outs, firsts = [], [], {}
    offs = None
    for k in range(nb):
        d, offs = synth_nars_device(sizes, first_index=5000 + 256 * k)
        ins.append(d)
    cap = ca.chunking.batch_capacity(offs, params[0])
    outs = [torch.full((cap * 48,), 0xAB, dtype=torch.uint8, device="cuda") for _ in range(nb)]
    with pipe:
        for k in range(nb):
            for tag, first in pipe.submit(ins[k].data_ptr(), offs, outs[k].data_ptr(), cap, tag=k):
                firsts[tag] = first
        for tag, first in pipe.drain():
            firsts[tag] = first
    assert pipe.depth == depth and sorted(firsts) == list(range(nb))
    ref_out = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
    for k in range(nb):
        ref_first = ca.chunk_batch_device(ins[k].data_ptr(), offs, ref_out.data_ptr(), cap, *params)
        n = int(ref_first[-1])
        assert np.array_equal(firsts[k], ref_first), k
        got = outs[k][: n * 48].cpu().numpy()
        assert np.array_equal(got, ref_out[: n * 48].cpu().numpy()), k
        i = (37 * k) % 256  # one sampled NAR per batch against the oracle
        nar = ins[k][int(offs[i]):int(offs[i + 1])].cpu().numpy()
        want = O.chunk_descriptors(nar, *params, algo=SHA)
        assert_same(got.view(ca.DESC_DTYPE)[int(ref_first[i]):int(ref_first[i + 1])], want, f"batch{k} nar{i}")


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]], ids=["one", "same_twice", "same_thrice"])
def test_multi_device_gather_matches_single_batch(ca, O, devices):
    """cg_multi_* (MultiDevicePipeline): a batch of NARs sharded over `devices` (the one GPU
    of this box listed 1-3 times: the same sharding, per-device pipelines and descriptor
    gather as on 8 GPUs, with device-to-device copies in place of xGMI peer copies) equals
    one synchronous call over all the NARs in order, and the oracle on every NAR; steps
    stay in order with several in flight; a too-small output array fails at the wait."""
    import torch

    from chunker_amd.dist import shard_nars
    from chunker_amd.nar import synth_nars

    sizes = [1 << 20] * 5 + [300_008, 120, 8 * 777 + 4096]
    steps = []
    for s in range(4):
        data, offs = synth_nars(sizes, first_index=7000 + 100 * s)
        cap = ca.chunking.batch_capacity(offs, P16[0])
        whole = torch.from_numpy(np.concatenate([data, np.zeros(256, np.uint8)])).cuda()
        ref = torch.zeros(cap * 48, dtype=torch.uint8, device="cuda")
        ref_first = ca.chunk_batch_device(whole.data_ptr(), offs, ref.data_ptr(), cap, *P16)
        shards = []
        for k in range(len(devices)):
            r = shard_nars(len(sizes), len(devices), k)
            lo, hi = int(offs[r.start]), int(offs[r.stop])
            d = torch.from_numpy(np.concatenate([data[lo:hi], np.zeros(256, np.uint8)])).cuda()
            shards.append((d, offs[r.start:r.stop + 1] - offs[r.start]))
        steps.append({"data": data, "offs": offs, "cap": cap, "ref": ref.cpu().numpy(), "ref_first": ref_first,
                      "shards": shards, "out": torch.full((cap * 48,), 0xAB, dtype=torch.uint8, device="cuda")})
    got = []
    with ca.chunking.MultiDevicePipeline(devices, *P16, group=2, depth=3) as mp:
        for k, st in enumerate(steps):
            got += mp.submit([(d.data_ptr(), o) for d, o in st["shards"]], st["out"].data_ptr(), st["cap"], tag=k)
        got += mp.drain()
        assert [t for t, _ in got] == list(range(len(steps)))
        for k, first in got:
            st = steps[k]
            assert np.array_equal(first, st["ref_first"]), k
            n = int(first[-1])
            out = st["out"].cpu().numpy()
            assert np.array_equal(out[: n * 48], st["ref"][: n * 48]), k
            descs = out.view(ca.DESC_DTYPE)
            for i in range(len(sizes)):
                want = O.chunk_descriptors(st["data"][st["offs"][i]:st["offs"][i + 1]], *P16, algo=SHA)
                assert_same(descs[int(first[i]):int(first[i + 1])], want, f"step{k} nar{i}")
        st = steps[0]
        mp.submit([(d.data_ptr(), o) for d, o in st["shards"]], st["out"].data_ptr(), 3, tag="small")
        with pytest.raises(ca.ChunkingError, match="too small"):
            mp.drain()

"""Child process of tests/test_gpu_robust.py::test_sixteen_hardware_queues.

Runs with GPU_MAX_HW_QUEUES=16 set by the parent before anything in this process touches
HIP (HIP reads the variable once, at initialisation; the library sizes its stream lanes
from the value it saw at load, stream.hip g_hw_queues_at_load): concurrent callers of
the synchronous device entry (20 merged -- past the 12 callers 16 queues run side by
side, runtime.hip coal_min --, 12 per-batch, 12 with coalescing off), and a
ChunkStream whose 8 digest
lanes (queues - 2) each hold a HIP stream of their own -- every result checked against
the oracle.  Prints one line "hw16 ok ..." on success; any mismatch raises."""
import io
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")

import torch  # noqa: E402

import chunker_amd as ca  # noqa: E402
from oracle import oracle as O  # noqa: E402

P = (65536, 262144, 1 << 20)


def same(got, ref):
    return (len(got) == len(ref) and np.array_equal(got["offset"], ref["offset"])
            and np.array_equal(got["length"], ref["length"]) and np.array_equal(got["hash"], ref["hash"]))


def concurrent_callers(n_threads, coalesce, seed):
    rng = np.random.default_rng(seed)
    jobs = []
    for _ in range(n_threads):
        lens = [int(x) for x in rng.integers(1, 3 << 20, 3)] + [0, 2 * P[2] + 5]
        nars = [rng.integers(0, 256, n, dtype=np.uint8) for n in lens]
        offs = np.zeros(len(nars) + 1, np.uint64)
        np.cumsum(lens, out=offs[1:])
        d = torch.from_numpy(np.concatenate(nars + [np.zeros(16, np.uint8)])).cuda()
        cap = ca.chunking.batch_capacity(offs, P[0])
        jobs.append((nars, offs, d, torch.zeros(cap * 48, dtype=torch.uint8, device="cuda"), cap, torch.cuda.Stream()))
    torch.cuda.synchronize()
    firsts, errors = [None] * n_threads, []
    bar = threading.Barrier(n_threads)

    def work(t):
        nars, offs, d, out, cap, s = jobs[t]
        try:
            bar.wait()
            for _ in range(2):
                firsts[t] = ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *P, stream=s.cuda_stream)
        except Exception as e:  # noqa: BLE001
            errors.append((t, repr(e)))

    old = ca.lib.cg_test_coalesce(coalesce)
    try:
        th = [threading.Thread(target=work, args=(t,)) for t in range(n_threads)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=100)
    finally:
        ca.lib.cg_test_coalesce(old)
    assert not errors, errors
    torch.cuda.synchronize()
    for t, (nars, offs, d, out, cap, s) in enumerate(jobs):
        descs = out.cpu().numpy().view(ca.DESC_DTYPE)
        for i, nar in enumerate(nars):
            got = descs[int(firsts[t][i]):int(firsts[t][i + 1])]
            assert same(got, O.chunk_descriptors(nar, *P, algo=1, nthreads=8)), (coalesce, t, i)


def stream_with_all_lanes():
    data = np.random.default_rng(3).integers(0, 256, 40 << 20, dtype=np.uint8).tobytes()
    got = [(c.offset, c.length, c.hash) for c in ca.chunking.ChunkStream(io.BytesIO(data), *P)]
    ref = [(int(r["offset"]), int(r["length"]), bytes(r["hash"])) for r in O.chunk_descriptors(data, *P, algo=1, nthreads=8)]
    assert got == ref, "ChunkStream at 16 queues differs from the oracle"
    return len(got)


if __name__ == "__main__":
    assert os.environ.get("GPU_MAX_HW_QUEUES") == "16", "the parent sets GPU_MAX_HW_QUEUES=16"
    torch.cuda.set_device(0)
    import ctypes

    def groups():
        out = (ctypes.c_uint64 * 4)()
        ca.lib.cg_coalesce_stats(out)
        return int(out[0])

    g0 = groups()
    concurrent_callers(12, 1, seed=23)  # per-batch launches (coalescing on, no more callers than coal_min)
    g1 = groups()
    assert g1 == g0, ("12 callers at 16 queues merged", g0, g1)
    concurrent_callers(20, 1, seed=21)  # more callers than coal_min: merged digests
    assert groups() > g1, "20 callers at 16 queues formed no merged group"
    concurrent_callers(12, 0, seed=22)
    n = stream_with_all_lanes()
    print(f"hw16 ok: 20 / 12 callers coalesced + per-batch, ChunkStream {n} chunks")

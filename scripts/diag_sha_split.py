"""Diagnostic: split-lane vs one-lane SHA-256 digest workgroups.

Prints one JSON line: the DPP bank-mask lane probe the split rounds rely on, cycles
per round of a lone wave for the split rounds (cg_diag_sha_rounds_split) and the
one-lane rounds (cg_diag_sha_rounds), and for configs 2 and a quarter of config 4
the digest-stage time at several caps on split workgroups
(cg_test_sha_split_max; 0 = one lane per chunk everywhere), with the digests
compared against the one-lane run."""
import os
os.environ["CHUNKER_AMD_DIAG"] = "1"  # load libchunker_amd_diag.so (make -C chunker_amd/csrc diag)
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")
import ctypes
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import chunker_amd as ca  # noqa: E402
from chunker_amd._lib import lib  # noqa: E402
from chunker_amd.nar import synth_nars  # noqa: E402

lib.cg_test_sha_split_max.argtypes = [ctypes.c_uint32]
lib.cg_test_sha_split_max.restype = ctypes.c_uint32
lib.cg_diag_dpp_probe.argtypes = [ctypes.c_void_p]
lib.cg_test_sha_quad_max.argtypes = [ctypes.c_uint32]
lib.cg_test_sha_quad_max.restype = ctypes.c_uint32
lib.cg_diag_sha_rounds_split.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                         ctypes.c_void_p]
lib.cg_diag_sha_rounds.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]

res = {}
probe = np.zeros(64, np.uint32)
assert lib.cg_diag_dpp_probe(probe.ctypes.data) == 0
want = np.array([(1000 + 2 * L + 4) if ((L >> 2) & 1) == 0 else L for L in range(64)], np.uint32)
res["dpp_probe_ok"] = bool(np.array_equal(probe, want))
if not res["dpp_probe_ok"]:
    res["dpp_probe"] = probe.tolist()

it = 2000
cyc = np.zeros(1, np.uint64)
lib.cg_diag_sha_rounds_split(it, 1, 64, 0, cyc.ctypes.data)
res["pair_cycles_per_round_1wave"] = float(cyc[0]) / (it * 64)
lib.cg_diag_sha_rounds_split(it, 1, 64, 1, cyc.ctypes.data)
res["quad_cycles_per_round_1wave"] = float(cyc[0]) / (it * 64)
cyc2 = np.zeros(2, np.uint64)
lib.cg_diag_sha_rounds(it, 1, 64, cyc2.ctypes.data)
res["onelane_cycles_per_round_1wave"] = float(cyc2[0]) / (it * 64)

CFG = {"c2": (256, 4 << 20, (256 << 10, 1 << 20, 4 << 20)),
       "c4q": (4, 1 << 30, (64 << 10, 256 << 10, 1 << 20))}
buf = (ctypes.c_double * 5)()
for name, (n, size, params) in CFG.items():
    host, offs = synth_nars(np.full(n, size, np.uint64))
    d = torch.empty(len(host) + 256, dtype=torch.uint8, device="cuda")
    d[: len(host)].copy_(torch.from_numpy(host))
    del host
    cap = ca.chunking.batch_capacity(offs, params[0])
    out = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    ref = None
    row = {}
    for qmax, smax in ((0, 0), (0, 256), (256, 0), (256, 256), (64, 256)):
        prevq = lib.cg_test_sha_quad_max(qmax)
        prev = lib.cg_test_sha_split_max(smax)
        lib.cg_set_profiling(1)
        times = []
        for _ in range(3):
            first = ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params, stream=st)
            lib.cg_last_stage_times(buf, 5)
            times.append(buf[4])
        lib.cg_set_profiling(0)
        lib.cg_test_sha_split_max(prev)
        lib.cg_test_sha_quad_max(prevq)
        nch = int(first[-1])
        dig = out[: nch * 48].view(-1, 48)[:, 16:].cpu().numpy()
        if ref is None:
            ref = dig
        row[f"quad{qmax}_pair{smax}"] = {"digest_ms": round(float(np.median(times)), 3), "chunks": nch,
                          "same_as_onelane": bool(np.array_equal(dig, ref))}
    res[name] = row
    del d, out
    torch.cuda.empty_cache()
print(json.dumps(res))

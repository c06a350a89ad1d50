"""Diagnostic: where and when the SHA-256 digest's workgroups ran on a GPU-filling
batch (BASELINE config-4 shape by default: 16 x 1 GiB at 64K/256K/1M).

Uses the diagnostics build's per-workgroup record (k_sha256 diag: consumer start/end on
the 100 MHz global clock, shader-clock totals, and each wave's HW_ID/XCC_ID) to answer:
which tier's workgroup ends the stage, how many cycles per round each quad consumer ran
at against its lone-wave 41.8, and whether the quad consumers shared their CU / SIMD
with other workgroups' waves while they ran.  Prints one JSON object."""
import os
os.environ["CHUNKER_AMD_DIAG"] = "1"
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")
import argparse  # noqa: E402
import ctypes  # noqa: E402
import json  # noqa: E402
import sys  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, ".")
import chunker_amd as ca  # noqa: E402
from chunker_amd.nar import synth_nars_device  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nars", type=int, default=16)
ap.add_argument("--nar-mib", type=int, default=1024)
ap.add_argument("--params", default="65536,262144,1048576")
ap.add_argument("--quad-fill", type=int, default=-1, help="cg_test_sha_quad_fill override (-1: product)")
args = ap.parse_args()
params = tuple(int(x) for x in args.params.split(","))
lib = ca.lib
lib.cg_diag_sha_stats.argtypes = [ctypes.c_uint32, ctypes.c_void_p]
if args.quad_fill >= 0:
    lib.cg_test_sha_quad_fill(args.quad_fill)

d, offs = synth_nars_device(np.full(args.nars, args.nar_mib << 20, np.uint64))
cap = ca.chunking.batch_capacity(offs, params[0])
out = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
sp = torch.cuda.current_stream().cuda_stream
first = ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params, hash=1, stream=sp)
nwg = (cap + 7) // 8 + 8
lib.cg_diag_sha_stats(nwg, None)
lib.cg_set_profiling(1)
first = ca.chunk_batch_device(d.data_ptr(), offs, out.data_ptr(), cap, *params, hash=1, stream=sp)
st = (ctypes.c_double * 5)()
lib.cg_last_stage_times(st, 5)
tiers = (ctypes.c_uint32 * 4)()
lib.cg_last_sha_tiers(tiers)
nq, npair, n1, pad = (int(t) for t in tiers)
buf = np.zeros(8 * nwg, np.uint64)
lib.cg_diag_sha_stats(nwg, buf.ctypes.data)
lib.cg_diag_sha_stats(0, None)
n = int(first[-1])
lens = np.sort(out[: 48 * n].cpu().numpy().view(ca.DESC_DTYPE)["length"].astype(np.int64))[::-1]
blocks = (lens + 72) // 64

wg = buf.reshape(-1, 8)
bases, sizes, kinds = [], [], []
for b in range(nq + npair + n1):
    if b < nq:
        bases.append(8 * b), sizes.append(8), kinds.append("quad")
    elif b < nq + npair:
        bases.append(8 * nq + 32 * (b - nq)), sizes.append(32), kinds.append("pair")
    else:
        bases.append(8 * nq + 32 * npair + 64 * (b - nq - npair)), sizes.append(64), kinds.append("lane")
used = [b for b in range(len(bases)) if bases[b] < n]
t0 = min(int(wg[b, 4]) for b in used)


def loc(v):
    v = int(v)
    hw, xcc = v & 0xffffffff, v >> 32
    return {"xcc": xcc & 0xf, "se": (hw >> 13) & 7, "sh": (hw >> 12) & 1, "cu": (hw >> 8) & 15, "simd": (hw >> 4) & 3}


def cu_key(L):
    return (L["xcc"], L["se"], L["sh"], L["cu"])


recs = []
for b in used:
    nb = int(blocks[bases[b]])
    c, p = loc(wg[b, 6]), loc(wg[b, 7])
    recs.append({"wg": b, "kind": kinds[b], "blocks": nb, "start_us": (int(wg[b, 4]) - t0) / 100.0,
                 "end_us": (int(wg[b, 5]) - t0) / 100.0, "cyc_per_round": float(wg[b, 3]) / max(nb * 64, 1),
                 "cons": c, "prod": p})
end = max(r["end_us"] for r in recs)
last = max(recs, key=lambda r: r["end_us"])
res = {"digest_ms": round(st[4], 3), "chunks": n, "tiers": {"quad": nq, "pair": npair, "one_lane": n1, "pad": pad},
       "stage_end_us": end, "last_wg": {k: last[k] for k in ("wg", "kind", "blocks", "start_us", "end_us",
                                                              "cyc_per_round")}}
for kind in ("quad", "pair", "lane"):
    rs = [r for r in recs if r["kind"] == kind]
    if not rs:
        continue
    cpr = np.array([r["cyc_per_round"] for r in rs])
    res[kind] = {"wgs": len(rs), "max_end_us": max(r["end_us"] for r in rs),
                 "max_start_us": max(r["start_us"] for r in rs),
                 "cyc_per_round_of_longest": {"median": round(float(np.median(cpr)), 2),
                                              "max": round(float(cpr.max()), 2),
                                              "min": round(float(cpr.min()), 2)}}
# sharing: other workgroups' waves on a quad consumer's CU / SIMD while it ran
share = []
for q in (r for r in recs if r["kind"] == "quad"):
    same_cu = same_simd = 0
    for r in recs:
        if r is q or r["start_us"] >= q["end_us"] or r["end_us"] <= q["start_us"]:
            continue
        for w in (r["cons"], r["prod"]):
            if cu_key(w) == cu_key(q["cons"]):
                same_cu += 1
                same_simd += w["simd"] == q["cons"]["simd"]
    share.append({"wg": q["wg"], "blocks": q["blocks"], "cyc_per_round": round(q["cyc_per_round"], 2),
                  "end_us": q["end_us"], "other_waves_on_cu": same_cu, "other_waves_on_simd": same_simd,
                  "own_producer_same_simd": q["prod"]["simd"] == q["cons"]["simd"] and
                  cu_key(q["prod"]) == cu_key(q["cons"])})
res["quad_sharing"] = share[:64]
# lanes per SIMD over the stage: how many distinct CUs were used
res["cus_used"] = len({cu_key(r["cons"]) for r in recs} | {cu_key(r["prod"]) for r in recs})
print(json.dumps(res))

"""Diagnostic: aggregate rate of K config-2 batches in flight (bench.py's `concurrent`
measurement) by SHA-256 workgroup tiers: the product's latency tiers (quads and pairs
for the longest chunks) vs one lane per chunk everywhere (cg_test_sha_quad_max /
cg_test_sha_split_max = 0), which spends 5x fewer lane-instructions per round -- with the
digests of concurrent callers merged (the product) and with one launch per batch."""
import os
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("CHUNKER_AMD_DIAG_HW_QUEUES", "16")
import argparse  # noqa: E402
import json  # noqa: E402
import sys  # noqa: E402

sys.path.insert(0, ".")
import torch  # noqa: E402

import bench  # noqa: E402
import chunker_amd as ca  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--concurrent", default="1,8,32")
ap.add_argument("--zeros", action="store_true")
ap.add_argument("--concurrent-reps", type=int, default=3)
args = ap.parse_args()
n_per, nar_bytes, params, algo, _ = bench.CONFIGS["c2"]
res = {"hw_queues": os.environ["GPU_MAX_HW_QUEUES"]}
for coal in (1, 0):
    old_c = ca.lib.cg_test_coalesce(coal)
    for name, q, p in [("latency_tiers", 256, 256), ("one_lane", 0, 0), ("pairs_only", 0, 256)]:
        oq, op = ca.lib.cg_test_sha_quad_max(q), ca.lib.cg_test_sha_split_max(p)
        try:
            res[f"{name}{'' if coal else '_per_batch'}"] = bench.concurrent_rates(ca, torch, args, n_per, nar_bytes,
                                                                                 params, algo)
        finally:
            ca.lib.cg_test_sha_quad_max(oq)
            ca.lib.cg_test_sha_split_max(op)
    ca.lib.cg_test_coalesce(old_c)
print(json.dumps(res))

"""One summary row of a bench line (depth A/B sessions): config, depth, value, ms/step,
batch latency p50/p99, digest ms, overlap."""
import json
import sys

d = json.load(open(sys.argv[1]))
lat = d.get("batch_latency_ms", {})
print(sys.argv[2], sys.argv[3], d["value"], d["ms_per_step"], lat.get("p50"), lat.get("p99"),
      d["stages_ms"]["digest_timed"], d["overlap"])

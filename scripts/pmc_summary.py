"""Summarise rocprofv3 --pmc passes (scripts/gpu_pmc.sh) into per-kernel averages per
dispatch.  FETCH_SIZE / WRITE_SIZE are in KiB; per MI355X_MICROARCH.md §HBM,
FETCH_SIZE reads half the bytes of wide (16 B/lane) coalesced streaming loads on
gfx950, so `fetch_bytes_x2` doubles it; other access widths are uncalibrated."""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
tag = sys.argv[2] if len(sys.argv) > 2 else "pmc"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob(f"{root}/{tag}_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, d in acc.items():
    row = {c: sum(v) / len(v) for c, v in d.items()}
    if "FETCH_SIZE" in row:
        row["fetch_bytes"] = row["FETCH_SIZE"] * 1024
        row["fetch_bytes_x2"] = row["FETCH_SIZE"] * 2048
    if "WRITE_SIZE" in row:
        row["write_bytes"] = row["WRITE_SIZE"] * 1024
    out[k] = {c: round(v, 1) for c, v in row.items()}
print(json.dumps(out, indent=1))

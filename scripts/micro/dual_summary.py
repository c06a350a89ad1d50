"""Summarise a rocprofv3 --pmc pass over scripts/micro/_bin/issue_rates (counters
SQ_ACTIVE_INST_VALU2, SQ_INSTS_VALU): per kernel and grid size (w = waves per SIMD =
grid / (256 CUs x 256 threads)), summed over dispatches, the share of VALU instructions
issued two per quad-cycle, dual_frac = 2 x VALU2 / INSTS_VALU."""
import collections
import csv
import glob
import json
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
for path in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
        acc[(name, grid)][r["Counter_Name"]] += float(r["Counter_Value"])
rows = []
for (name, grid), d in sorted(acc.items()):
    insts, v2 = d.get("SQ_INSTS_VALU", 0.0), d.get("SQ_ACTIVE_INST_VALU2", 0.0)
    rows.append({"kernel": name, "w": round(grid / (256 * 256), 2), "insts_valu": insts, "valu2": v2,
                 "dual_frac": round(2 * v2 / insts, 4) if insts else None})
print(json.dumps({"what": "2 x SQ_ACTIVE_INST_VALU2 / SQ_INSTS_VALU per kernel and waves per SIMD", "rows": rows},
                 indent=1))

#!/bin/bash
# A/B kernel traces: bench.py --config $CFG under rocprofv3 --kernel-trace --stats, current build
# vs chunker_amd/libchunker_amd_prev.so, alternating; prints per-kernel average microseconds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c3}
TAG=${TAG:-abt}
P=$R/chunker_amd/libchunker_amd_prev.so
for i in 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_new_$i" -o run --output-format csv -- python3 "$R/bench.py" --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-concurrent > gpurun_out/${TAG}_new_$i.log 2>&1 || exit $?
  CHUNKER_AMD_LIB=$P timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prev_$i" -o run --output-format csv -- python3 "$R/bench.py" --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-concurrent > gpurun_out/${TAG}_prev_$i.log 2>&1 || exit $?
done
python3 - "$TAG" <<'PY'
import csv, glob, json, sys
tag = sys.argv[1]
for run in sorted(glob.glob(f"gpurun_out/{tag}_*_[12]")):
    f = glob.glob(run + "/**/run_kernel_stats.csv", recursive=True) or glob.glob(run + "/run_kernel_stats.csv")
    rows = list(csv.DictReader(open(f[0])))
    top = {r["Name"].split("(")[0].replace("void ", "")[:28]: round(float(r["AverageNs"]) / 1e3, 2) for r in rows[:9]}
    line = open(run + ".log").read().strip().splitlines()[-1]
    try:
        v = json.loads(line)["value"]
    except Exception:
        v = None
    print(run, v, json.dumps(top))
PY

#!/bin/bash
# Round 4 session G: product scan choice (persistent from 4 GiB), coalescer with one set and
# an adaptive group target, K = 32 kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/r04g_pytest_fast.log 2>&1 || { tail -40 gpurun_out/r04g_pytest_fast.log; exit 1; }
tail -2 gpurun_out/r04g_pytest_fast.log
timeout -k 10 300 python -u scripts/scan_ab.py --configs c2,c4,c5 --reps 5 --kernels 0,1,2 > gpurun_out/r04g_scan_ab.json 2> gpurun_out/r04g_scan_ab.err || { tail -5 gpurun_out/r04g_scan_ab.err; exit 1; }
timeout -k 10 300 python bench.py --concurrent-only --concurrent-reps 6 > gpurun_out/r04g_conc_coal1.json 2> gpurun_out/r04g_conc_coal1.err || exit 1
CHUNKER_AMD_COAL_SETS=2 timeout -k 10 300 python bench.py --concurrent-only --concurrent-reps 6 > gpurun_out/r04g_conc_coal2.json 2> gpurun_out/r04g_conc_coal2.err || exit 1
timeout -k 10 300 python bench.py --concurrent-only --concurrent-reps 6 --no-coalesce > gpurun_out/r04g_conc_nocoal.json 2> gpurun_out/r04g_conc_nocoal.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04g_k32 -o run --output-format csv -- python3 bench.py --concurrent-only --concurrent 32 --concurrent-reps 3 > gpurun_out/r04g_k32.log 2>&1 || { tail -5 gpurun_out/r04g_k32.log; exit 1; }
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r04g_scan_ab*.json")):
    d=json.loads(open(f).read())
    print(f.split("/")[-1], {k:v["ms"] for k,v in d.items() if isinstance(v,dict)})
PY
cat gpurun_out/r04g_conc_coal1.json gpurun_out/r04g_conc_coal2.json gpurun_out/r04g_conc_nocoal.json
find gpurun_out/r04g_k32 -name "*kernel_stats.csv" | head -1 | xargs head -12 | cut -c1-200
echo "rc=0"

#!/bin/bash
# Round 3 session Y: asynchronous device batches (cg_chunk_batch_device_async / cg_batch_wait)
# and bench.py's queued steps -- the parity suite, then configs 2 and 3 (kernel trace of c3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m "gpu and not slow" tests > gpurun_out/r03_y_tests.log 2>&1 || { tail -30 gpurun_out/r03_y_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r03_y_tests.log)"
for c in c3 c2 c3; do
  timeout -k 10 200 python3 bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-concurrent > gpurun_out/r03_y_$c.json 2> gpurun_out/r03_y_$c.err || { tail -3 gpurun_out/r03_y_$c.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['ms_per_step'],d['stages_ms'])" gpurun_out/r03_y_$c.json $c
  cat gpurun_out/r03_y_$c.json >> gpurun_out/r03_y_all.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r03_y_c3" -o run --output-format csv -- python3 "$R/bench.py" --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-concurrent > gpurun_out/prof_r03_y_c3.log 2>&1 && echo "rocprof ok"
rc=$?; echo "rc=$rc"; exit $rc

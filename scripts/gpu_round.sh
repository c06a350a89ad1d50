#!/bin/bash
# One GPU session: parity tests, bench lines c2/c3/c4, end-to-end host rate,
# rocprofv3 kernel-trace summaries for c2 and c3.  Every GPU step has its own time
# limit; steps are chained with && so a failure stops the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
timeout -k 10 700 python -u -m pytest tests/ -x -q -m "gpu and not slow" --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
 && echo "pytest ok" \
 && timeout -k 10 200 python bench.py --config c2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err && cat gpurun_out/bench_c2.json \
 && timeout -k 10 200 python bench.py --config c3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err && cat gpurun_out/bench_c3.json \
 && timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --cpu-sample-nars 1 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err && cat gpurun_out/bench_c4.json \
 && timeout -k 10 200 python scripts/e2e_bench.py > gpurun_out/e2e_c2.json 2> gpurun_out/e2e.err && cat gpurun_out/e2e_c2.json \
 && timeout -k 10 200 python scripts/e2e_bench.py --algo 0 > gpurun_out/e2e_c3.json 2>> gpurun_out/e2e.err && cat gpurun_out/e2e_c3.json \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_c2" -o run --output-format csv -- python3 "$R/bench.py" --config c2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${TAG}_c2.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_c3" -o run --output-format csv -- python3 "$R/bench.py" --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${TAG}_c3.log 2>&1 \
 && echo "rocprof ok"
rc=$?
echo "rc=$rc"
tail -3 gpurun_out/pytest_gpu.log
exit $rc

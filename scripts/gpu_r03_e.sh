#!/bin/bash
# Round 3 session E: GPU tests (fast), the streaming rates (lazy arena), the default
# bench line.  Every GPU step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -v -m "gpu and not slow" --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
prc=$?
echo "pytest fast rc=$prc"; tail -2 gpurun_out/pytest_gpu.log; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head
[ $prc -le 1 ] \
 && timeout -k 10 400 python -u scripts/stream_bench.py > gpurun_out/stream_bench.json 2> gpurun_out/stream_bench.err && cat gpurun_out/stream_bench.json \
 && timeout -k 10 400 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err && cat gpurun_out/bench_c2.json
rc=$?
echo "rc=$rc"
exit $rc

#!/bin/bash
# Streaming + concurrency session: stream parity tests, scripts/stream_bench.py, and a
# rocprofv3 kernel trace of K = 8 config-2 batches in flight (bench.py --concurrent-only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robust.py -x -v -k "stream or push or concurrent or spin" --timeout 200 --timeout-method thread > gpurun_out/pytest_stream.log 2>&1 \
 && echo "pytest ok" \
 && timeout -k 10 500 python -u scripts/stream_bench.py > gpurun_out/stream_${TAG}.json 2> gpurun_out/stream.err && cat gpurun_out/stream_${TAG}.json \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_conc" -o run --output-format csv -- python3 "$R/bench.py" --concurrent-only --concurrent 8 > gpurun_out/prof_${TAG}_conc.log 2>&1 \
 && tail -1 gpurun_out/prof_${TAG}_conc.log && echo "rocprof ok"
rc=$?
echo "rc=$rc"
tail -5 gpurun_out/pytest_stream.log
exit $rc

#!/bin/bash
# Round 3 session I: staged (asynchronous) stream push -- stream tests, stream bench, GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stream.py tests/test_gpu_parity.py > gpurun_out/r03_i_stream_tests.log 2>&1 \
 && echo "stream tests ok" \
 && timeout -k 10 300 python3 scripts/stream_bench.py > gpurun_out/r03_i_stream_bench.json 2> gpurun_out/r03_i_stream_bench.err \
 && echo "stream bench ok" && cat gpurun_out/r03_i_stream_bench.json \
 && timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r03_i_pytest_gpu.log 2>&1 \
 && echo "gpu suite ok" && tail -2 gpurun_out/r03_i_pytest_gpu.log
rc=$?
tail -15 gpurun_out/r03_i_stream_tests.log
echo "rc=$rc"
exit $rc

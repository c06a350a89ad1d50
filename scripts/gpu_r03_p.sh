#!/bin/bash
# Round 3 session P: stream group cap + 2 GiB default budget -- tests, grid, stream bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stream.py tests/test_gpu_parity.py > gpurun_out/r03_p_tests.log 2>&1 \
 && GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python3 scripts/diag_stream_push.py --budgets 512,1024,2048,4096 > gpurun_out/r03_p_new16.json 2>gpurun_out/r03_p_new16.err \
 && GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python3 scripts/diag_stream_push.py --budgets 512,1024,2048,4096 > gpurun_out/r03_p_new4.json 2>gpurun_out/r03_p_new4.err \
 && GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python3 scripts/diag_stream_push.py --gib 4 --budgets 1024,2048,4096 > gpurun_out/r03_p_new16_4g.json 2>gpurun_out/r03_p_new16_4g.err \
 && GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python3 scripts/diag_stream_push.py --gib 4 --budgets 1024,2048,4096 > gpurun_out/r03_p_new4_4g.json 2>gpurun_out/r03_p_new4_4g.err \
 && timeout -k 10 300 python3 scripts/stream_bench.py > gpurun_out/r03_p_stream_bench.json 2> gpurun_out/r03_p_stream_bench.err
rc=$?; tail -2 gpurun_out/r03_p_tests.log; cat gpurun_out/r03_p_stream_bench.json; echo "rc=$rc"; exit $rc

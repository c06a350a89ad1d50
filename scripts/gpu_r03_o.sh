#!/bin/bash
# Round 3 session O: stream lanes without hipFree stalls (A/B against the previous build), 16 and 4 HW queues.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
P=$PWD/chunker_amd/libchunker_amd_prev.so
timeout -k 10 120 python3 scripts/diag_alloc.py > gpurun_out/r03_o_alloc.json 2>gpurun_out/r03_o_alloc.err \
 && GPU_MAX_HW_QUEUES=16 CHUNKER_AMD_LIB=$P timeout -k 10 300 python3 scripts/diag_stream_push.py --budgets 512,1024,2048,4096 > gpurun_out/r03_o_prev16.json 2>gpurun_out/r03_o_prev16.err \
 && GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python3 scripts/diag_stream_push.py --budgets 512,1024,2048,4096 > gpurun_out/r03_o_new4.json 2>gpurun_out/r03_o_new4.err \
 && GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python3 scripts/diag_stream_push.py --gib 4 --budgets 1024,2048,4096 --group-caps 0,256 > gpurun_out/r03_o_new16_4g.json 2>gpurun_out/r03_o_new16_4g.err \
 && timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stream.py tests/test_gpu_parity.py > gpurun_out/r03_o_tests.log 2>&1
rc=$?; cat gpurun_out/r03_o_alloc.json; tail -2 gpurun_out/r03_o_tests.log; echo "rc=$rc"; exit $rc

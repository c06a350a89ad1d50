#!/bin/bash
# Round 3 session Q: stream digest lanes at 4 HW queues (does the third lane share the boundary stream's queue?).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python3 scripts/diag_stream_push.py --budgets 1024,2048,4096 --lanes 2,3 --group-caps 0,1048576 > gpurun_out/r03_q_q4.json 2>gpurun_out/r03_q_q4.err \
 && GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python3 scripts/diag_stream_push.py --gib 4 --budgets 2048,4096 --lanes 2,3 --group-caps 0,1048576 > gpurun_out/r03_q_q4_4g.json 2>gpurun_out/r03_q_q4_4g.err \
 && GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python3 scripts/diag_stream_push.py --gib 4 --budgets 2048,4096 --lanes 8,14 > gpurun_out/r03_q_q16_4g.json 2>gpurun_out/r03_q_q16_4g.err \
 && GPU_MAX_HW_QUEUES=4 timeout -k 10 200 rocprofv3 --kernel-trace -d $PWD/gpurun_out/r03_q_trace -o run --output-format csv -- python3 scripts/diag_stream_push.py --budgets 2048 > gpurun_out/r03_q_trace.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc

#!/bin/bash
# Round 3 session N: stream shape grid (group size cap, lanes, eager launch, budget) at 16 and 4 HW queues.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python3 scripts/diag_stream_push.py --budgets 512,1024,2048,4096 --group-caps 0,64 --lanes 0,15 --eager 0,1 > gpurun_out/r03_n_grid1.json 2>gpurun_out/r03_n_grid1.err \
 && GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python3 scripts/diag_stream_push.py --gib 4 --budgets 1024,2048,4096 --eager 0,1 > gpurun_out/r03_n_grid4.json 2>gpurun_out/r03_n_grid4.err \
 && GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python3 scripts/diag_stream_push.py --budgets 512,1024,2048,4096 --eager 0,1 > gpurun_out/r03_n_grid1_q4.json 2>gpurun_out/r03_n_grid1_q4.err \
 && GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python3 scripts/diag_stream_push.py --gib 4 --budgets 1024,2048,4096 --eager 0,1 > gpurun_out/r03_n_grid4_q4.json 2>gpurun_out/r03_n_grid4_q4.err
rc=$?; echo "rc=$rc"; exit $rc

#!/bin/bash
# Round 3, first session: the N > 1 path rehearsed on the one-GPU box (2 ranks over
# gloo, rank-0 check of the gathered batch), the dist GPU tests, config-4 bench with the
# exported digest tiers, and the host's CPU share.  Every GPU step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
{ echo "nproc=$(nproc) affinity=$(python3 -c 'import os; print(len(os.sched_getaffinity(0)))') OMP=$OMP_NUM_THREADS MAX_JOBS=$MAX_JOBS";
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; } > gpurun_out/cpuinfo.txt
timeout -k 10 400 python -u -m pytest tests/test_dist.py tests/test_gpu_stream.py -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1
prc=$?
echo "dist+stream tests rc=$prc"
# test failures (rc 1) are read afterwards; a crash, abort or time limit ends the session here
[ $prc -le 1 ] \
 && timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline --no-concurrent > gpurun_out/bench_g2_gloo.json 2> gpurun_out/bench_g2_gloo.err \
 && cat gpurun_out/bench_g2_gloo.json \
 && timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-concurrent > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err \
 && cat gpurun_out/bench_c4.json \
 && timeout -k 10 200 python -u scripts/diag_sha_place.py > gpurun_out/diag_sha_place_c4.json 2> gpurun_out/diag_sha_place.err \
 && echo "diag place ok" \
 && timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -v -k config4 --timeout 280 --timeout-method thread > gpurun_out/pytest_c4.log 2>&1 \
 && echo "c4 test ok" \
 && timeout -k 10 300 python bench.py --no-cpu-baseline --concurrent 8 --e2e 1,4,8 > gpurun_out/bench_c2_e2e.json 2> gpurun_out/bench_c2_e2e.err \
 && cat gpurun_out/bench_c2_e2e.json
rc=$?
echo "rc=$rc"
cat gpurun_out/cpuinfo.txt
tail -3 gpurun_out/pytest_dist.log
tail -3 gpurun_out/pytest_c4.log 2>/dev/null
exit $rc

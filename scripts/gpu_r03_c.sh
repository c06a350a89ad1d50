#!/bin/bash
# Round 3 session C: SHA-256 tier sweeps on the config-4 and config-5 shapes, and the
# e2e in-flight rates with 4 reps per thread.  Every GPU step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_configs.py -v -m gpu -k "blake3 or b3 or B3 or stream or config3" --timeout 200 --timeout-method thread > gpurun_out/pytest_b3.log 2>&1
prc=$?
echo "blake3/stream tests rc=$prc"; tail -3 gpurun_out/pytest_b3.log
[ $prc -le 1 ] \
 && timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-concurrent > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err && cat gpurun_out/bench_c3.json \
 && timeout -k 10 300 python -u scripts/diag_sha_tiers.py --quad-max 256 --pairs 64,96,128,160,192 --fill 48,64,96,128 > gpurun_out/tiers_c4.json 2> gpurun_out/tiers_c4.err && cat gpurun_out/tiers_c4.json \
 && timeout -k 10 300 python -u scripts/diag_sha_tiers.py --params 262144,1048576,4194304 --quad-max 8,16,32,64,128,256 --pairs 32,64,128,256 --fill 32 > gpurun_out/tiers_c5.json 2> gpurun_out/tiers_c5.err && cat gpurun_out/tiers_c5.json \
 && timeout -k 10 300 python bench.py --no-cpu-baseline --concurrent 8 --e2e 4,8,16 > gpurun_out/bench_e2e.json 2> gpurun_out/bench_e2e.err && cat gpurun_out/bench_e2e.json
rc=$?
echo "rc=$rc"
exit $rc

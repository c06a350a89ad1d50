#!/bin/bash
# Round 3 session C: SHA-256 tier sweeps on the config-4 and config-5 shapes, and the
# e2e in-flight rates with 4 reps per thread.  Every GPU step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/diag_sha_tiers.py --quad-max 256 --pairs 64,96,128,160,192 --fill 48,64,96,128 > gpurun_out/tiers_c4.json 2> gpurun_out/tiers_c4.err && cat gpurun_out/tiers_c4.json \
 && timeout -k 10 300 python -u scripts/diag_sha_tiers.py --params 262144,1048576,4194304 --quad-max 8,16,32,64,128,256 --pairs 32,64,128,256 --fill 32 > gpurun_out/tiers_c5.json 2> gpurun_out/tiers_c5.err && cat gpurun_out/tiers_c5.json \
 && timeout -k 10 300 python bench.py --no-cpu-baseline --concurrent 8 --e2e 4,8,16 > gpurun_out/bench_e2e.json 2> gpurun_out/bench_e2e.err && cat gpurun_out/bench_e2e.json
rc=$?
echo "rc=$rc"
exit $rc

#!/bin/bash
# Round 3 session BA: config 4 / config 5 digest by quad / pair tier sizes, re-run now that
# the quad and pair round code is aligned (the fills were tuned at 41.8 / 46.5 clocks).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python3 scripts/diag_sha_tiers.py --fill 32,48,64,96 --pairs 64,128,192 > gpurun_out/r03_ba_tiers_c4.json 2> gpurun_out/r03_ba_tiers_c4.err || { tail -5 gpurun_out/r03_ba_tiers_c4.err; exit 1; }
cat gpurun_out/r03_ba_tiers_c4.json
timeout -k 10 500 python3 scripts/diag_sha_tiers.py --fill 32,64,128 --pairs 64,128,256 --params 262144,1048576,4194304 > gpurun_out/r03_ba_tiers_c5.json 2> gpurun_out/r03_ba_tiers_c5.err || { tail -5 gpurun_out/r03_ba_tiers_c5.err; exit 1; }
cat gpurun_out/r03_ba_tiers_c5.json
echo "rc=0"

#!/bin/bash
# Round 3 session AH: k_walk phase clocks on the config 4 / 5 / 2 shapes (diagnostics build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/diag_walk.py > gpurun_out/r03_ah_walk.json 2> gpurun_out/r03_ah_walk.err
rc=$?; cat gpurun_out/r03_ah_walk.json; tail -3 gpurun_out/r03_ah_walk.err; echo "rc=$rc"; exit $rc

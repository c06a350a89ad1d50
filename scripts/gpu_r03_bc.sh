#!/bin/bash
# Round 3 session BC: where config 4's digest time goes with the aligned round code
# (per-workgroup placement and tier end times, diagnostics build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/diag_sha_place.py > gpurun_out/r03_bc_place_c4.json 2> gpurun_out/r03_bc_place.err || { tail -5 gpurun_out/r03_bc_place.err; exit 1; }
cat gpurun_out/r03_bc_place_c4.json
echo "rc=0"

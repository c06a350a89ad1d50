#!/bin/bash
# Round 3 session AA: 16 GiB scan forms (config-5 shape): product k_scan_flat32<2, nt> vs
# a 4-row ring (mode 21) and cached loads (mode 22), and segments-per-wave caps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 scripts/diag_scan.py --variants 0 --modes 21,22 --mode-variant 5 --configs c5full,c4full --no-pattern --hash 1 --spw 0,16,64 > gpurun_out/r03_aa_scan.json 2> gpurun_out/r03_aa_scan.err
rc=$?; tail -3 gpurun_out/r03_aa_scan.err; cat gpurun_out/r03_aa_scan.json; echo "rc=$rc"; exit $rc

#!/bin/bash
# Round 3 session AB: SHA-256 consumer cycles per round on config 2 with the producer
# working (mode 0), without producer work (mode 1) and without the next-block wait (mode 2);
# lone-wave round cost and clock (diag_sha.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/diag_sha_stats.py c2 c2_mode1 c2_mode2 c2_again > gpurun_out/r03_ab_sha_stats.json 2> gpurun_out/r03_ab_sha_stats.err \
 && timeout -k 10 300 python3 scripts/diag_sha.py > gpurun_out/r03_ab_sha_rounds.json 2> gpurun_out/r03_ab_sha_rounds.err
rc=$?; cat gpurun_out/r03_ab_sha_stats.json gpurun_out/r03_ab_sha_rounds.json; tail -3 gpurun_out/r03_ab_sha_stats.err; echo "rc=$rc"; exit $rc

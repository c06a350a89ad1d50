#!/bin/bash
# Scan stage with and without a MALL flush before each timed scan (SHA-256 pipeline),
# 1 GiB (config 2) and 16 GiB (config 5 shard) batches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/diag_scan.py --variants 0 --modes "" --configs c2,c5one --no-pattern --hash 1 > gpurun_out/scan_mall_warm.json 2>/dev/null \
 && timeout -k 10 300 python -u scripts/diag_scan.py --variants 0 --modes "" --configs c2,c5one --no-pattern --hash 1 --flush > gpurun_out/scan_mall_flush.json 2>/dev/null \
 && timeout -k 10 300 python -u scripts/diag_scan.py --variants 0 --modes "" --configs c5full --no-pattern --hash 1 > gpurun_out/scan_mall_c5.json 2>/dev/null
rc=$?
cat gpurun_out/scan_mall_warm.json gpurun_out/scan_mall_flush.json gpurun_out/scan_mall_c5.json
exit $rc

#!/bin/bash
# Round 3 session AC: robustness tests (async batches from threads), then PMC passes for
# configs 2 and 3 on the queued-batch code (bench.py's traffic figures).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_robust.py > gpurun_out/r03_ac_robust.log 2>&1 || { tail -30 gpurun_out/r03_ac_robust.log; exit 1; }
echo "robust: $(tail -1 gpurun_out/r03_ac_robust.log)"
CFG=c3 TAG=r03_v22_pmc_c3 bash scripts/gpu_pmc.sh && python3 scripts/pmc_summary.py gpurun_out r03_v22_pmc_c3 > gpurun_out/r03_v22_pmc_c3.json \
 && CFG=c2 TAG=r03_v22_pmc_c2 bash scripts/gpu_pmc.sh && python3 scripts/pmc_summary.py gpurun_out r03_v22_pmc_c2 > gpurun_out/r03_v22_pmc_c2.json
rc=$?; echo "rc=$rc"; exit $rc

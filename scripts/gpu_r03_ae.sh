#!/bin/bash
# Round 3 session AE: randomized device-entry parity sweep (tests/test_gpu_fuzz.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m "gpu and slow" tests/test_gpu_fuzz.py > gpurun_out/r03_ae_fuzz.log 2>&1
rc=$?; tail -5 gpurun_out/r03_ae_fuzz.log; echo "rc=$rc"; exit $rc

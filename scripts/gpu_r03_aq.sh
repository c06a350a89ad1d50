#!/bin/bash
# Round 3 session AQ: the randomized device-batch parity sweep widened to 640 seeds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CHUNKER_AMD_FUZZ_SEEDS=640 timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fuzz.py > gpurun_out/r03_aq_fuzz.log 2>&1
rc=$?; tail -3 gpurun_out/r03_aq_fuzz.log; echo "rc=$rc"; exit $rc

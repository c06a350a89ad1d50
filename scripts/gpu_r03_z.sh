#!/bin/bash
# Round 3 session Z: configs 3 / 4 / 5 bench lines (with the CPU baseline) and the Node::put
# (CAS) bench on the queued-batch code; c3 kernel trace via gpu_configs_bench.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r03_v19 bash scripts/gpu_configs_bench.sh \
 && timeout -k 10 300 python3 scripts/cas_bench.py --config c2 > gpurun_out/r03_z_cas_c2.json 2> gpurun_out/r03_z_cas_c2.err && cat gpurun_out/r03_z_cas_c2.json
rc=$?; echo "rc=$rc"; exit $rc

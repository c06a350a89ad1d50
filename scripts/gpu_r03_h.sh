#!/bin/bash
# Round 3 session H: PMC passes (traffic for bench.py's roofline) for configs 2 and 3 on
# the current kernels, and kernel-trace summaries of the c2 / c4 bench commands.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=c2 TAG=r03_pmc_c2 bash scripts/gpu_pmc.sh && python3 scripts/pmc_summary.py gpurun_out r03_pmc_c2 > gpurun_out/r03_v8_pmc_c2.json \
 && CFG=c3 TAG=r03_pmc_c3 bash scripts/gpu_pmc.sh && python3 scripts/pmc_summary.py gpurun_out r03_pmc_c3 > gpurun_out/r03_v8_pmc_c3.json \
 && CFG=c4 TAG=r03_pmc_c4 bash scripts/gpu_pmc.sh && python3 scripts/pmc_summary.py gpurun_out r03_pmc_c4 > gpurun_out/r03_v8_pmc_c4.json \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r03_h_c2" -o run --output-format csv -- python3 "$R/bench.py" --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-concurrent > gpurun_out/prof_r03_h_c2.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r03_h_c4" -o run --output-format csv -- python3 "$R/bench.py" --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-concurrent > gpurun_out/prof_r03_h_c4.log 2>&1 \
 && echo "profiles ok"
rc=$?
echo "rc=$rc"
exit $rc

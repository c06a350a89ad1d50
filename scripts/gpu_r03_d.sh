#!/bin/bash
# Round 3 session D: config-4 tiers (64 quads / 128 pairs when the batch fills the GPU),
# BLAKE3 back to the separate top-fold kernel, and where the host-to-host rate goes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -v -m gpu -k "sha or config4 or blake3 or config3" --timeout 300 --timeout-method thread > gpurun_out/pytest_d.log 2>&1
prc=$?
echo "tests rc=$prc"; tail -3 gpurun_out/pytest_d.log
[ $prc -le 1 ] \
 && timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-concurrent > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err && cat gpurun_out/bench_c4.json \
 && timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-concurrent > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err && cat gpurun_out/bench_c3.json \
 && timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-concurrent > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err && cat gpurun_out/bench_c5.json \
 && timeout -k 10 400 python -u scripts/diag_e2e.py > gpurun_out/diag_e2e.json 2> gpurun_out/diag_e2e.err && cat gpurun_out/diag_e2e.json
rc=$?
echo "rc=$rc"
exit $rc

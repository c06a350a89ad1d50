#!/bin/bash
# Round 3 session F: K1 scan with buffer-resource row loads -- parity (every scan path and
# the full-size configs), then the scan stage on configs 2 / 3 / 4 / 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_tables.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_f.log 2>&1
prc=$?
echo "tests rc=$prc"; tail -2 gpurun_out/pytest_f.log; grep -E "FAILED|ERROR" gpurun_out/pytest_f.log | head
[ $prc -le 1 ] \
 && timeout -k 10 300 python bench.py --no-cpu-baseline --no-concurrent > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err && cat gpurun_out/bench_c2.json \
 && timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-concurrent > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err && cat gpurun_out/bench_c3.json \
 && timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --no-concurrent > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err && cat gpurun_out/bench_c4.json \
 && timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-concurrent > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err && cat gpurun_out/bench_c5.json
rc=$?
echo "rc=$rc"
exit $rc

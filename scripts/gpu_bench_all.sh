#!/bin/bash
# Parity subset + bench lines for configs c2, c3, c4 (each GPU step time-limited, chained with &&).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m "gpu and not slow" ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 \
 && echo "pytest ok" \
 && timeout -k 10 300 python bench.py --config c2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err && cat gpurun_out/bench_c2.json \
 && timeout -k 10 300 python bench.py --config c3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err && cat gpurun_out/bench_c3.json \
 && timeout -k 10 400 python bench.py --config c4 --steps 3 --warmup 1 --cpu-sample-nars 1 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err && cat gpurun_out/bench_c4.json
rc=$?
echo "rc=$rc"
tail -5 gpurun_out/pytest_gpu.log
exit $rc

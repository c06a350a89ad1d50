#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; steps are chained with && so a fault stops the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
TAG=${TAG:-r01}
MARK="gpu and not slow"; [ -n "$FULL" ] && MARK="gpu"
timeout -k 10 900 python -m pytest tests/ -x -q -m "$MARK" ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 \
 && echo "pytest ok" \
 && timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err \
 && echo "bench ok" && cat gpurun_out/bench.json \
 && export TMPDIR=/tmp \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof_${TAG}.log 2>&1 \
 && echo "rocprof ok"
rc=$?
echo "rc=$rc"
tail -15 gpurun_out/pytest_gpu.log
exit $rc

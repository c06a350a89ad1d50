#!/bin/bash
# Bench lines for configs c3, c4, c5 (c2 is gpu_round.sh's) plus a kernel trace of c3,
# every GPU step time-limited and chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
timeout -k 10 300 python bench.py --config c3 --no-concurrent > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err && cat gpurun_out/bench_c3.json \
 && timeout -k 10 400 python bench.py --config c4 --steps 3 --warmup 1 --no-concurrent > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err && cat gpurun_out/bench_c4.json \
 && timeout -k 10 400 python bench.py --config c5 --steps 3 --warmup 1 --no-concurrent > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err && cat gpurun_out/bench_c5.json \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_c3" -o run --output-format csv -- python3 "$R/bench.py" --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-concurrent > gpurun_out/prof_${TAG}_c3.log 2>&1 \
 && echo "rocprof ok"
rc=$?
echo "rc=$rc"
exit $rc

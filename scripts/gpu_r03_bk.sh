#!/bin/bash
# Round 3 session BK: full validation on HEAD (gpu_round.sh: fast + slow GPU tests, smoke,
# default bench line, c2 kernel trace), then the c3 / c4 / c5 bench lines and a c3 kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r03_v50 bash scripts/gpu_round.sh \
 && for cfg in c3 c4 c5; do timeout -k 10 400 python3 bench.py --config $cfg --steps 20 --no-concurrent > gpurun_out/r03_v50_${cfg}_bench.json 2> gpurun_out/r03_v50_${cfg}_bench.err || exit 1; tail -1 gpurun_out/r03_v50_${cfg}_bench.json | cut -c1-300; done \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r03_v50_c3" -o run --output-format csv -- python3 "$R/bench.py" --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-concurrent --e2e '' > gpurun_out/prof_r03_v50_c3.log 2>&1 \
 && echo "c3 rocprof ok"
rc=$?; echo "rc=$rc"; exit $rc

#!/bin/bash
# Round 3 session G: where a ChunkStream's time goes, the BLAKE3 load share (diag modes
# 0 / 1), and a config-3 kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/stream_profile.py > gpurun_out/stream_profile.txt 2>&1 && tail -40 gpurun_out/stream_profile.txt \
 && timeout -k 10 200 python -u scripts/diag_b3.py 0,1,0,1 > gpurun_out/diag_b3.json 2> gpurun_out/diag_b3.err && cat gpurun_out/diag_b3.json \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r03_g_c3" -o run --output-format csv -- python3 "$R/bench.py" --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-concurrent > gpurun_out/prof_r03_g_c3.log 2>&1 \
 && echo "rocprof ok" && head -12 gpurun_out/prof_r03_g_c3/run_kernel_stats.csv | cut -c1-160
rc=$?
echo "rc=$rc"
exit $rc

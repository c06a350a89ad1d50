#!/bin/bash
# Round 3 session B: the whole GPU suite (fast, then slow), smoke, the default bench line
# (cpu_baseline, concurrent, e2e), config 3, the SHA-256 tier sweep on the config-4 shape,
# and a kernel-trace profile of config 2.  Every GPU step has its own time limit; a crash,
# abort or time limit ends the session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03_b}
timeout -k 10 600 python -u -m pytest tests/ -v -m "gpu and not slow" --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
prc=$?
echo "pytest fast rc=$prc"
[ $prc -le 1 ] \
 && timeout -k 10 700 python -u -m pytest tests/ -v -m "gpu and slow" --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_slow.log 2>&1
prc=$?
echo "pytest slow rc=$prc"
[ $prc -le 1 ] \
 && timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && cat gpurun_out/smoke.log \
 && timeout -k 10 400 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err && cat gpurun_out/bench_c2.json \
 && timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-concurrent > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err && cat gpurun_out/bench_c3.json \
 && timeout -k 10 300 python -u scripts/diag_sha_tiers.py --fill 16,32,48,64 --pairs 128,256,384 > gpurun_out/diag_sha_tiers.json 2> gpurun_out/diag_sha_tiers.err && cat gpurun_out/diag_sha_tiers.json \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_c2" -o run --output-format csv -- python3 "$R/bench.py" --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-concurrent > gpurun_out/prof_${TAG}_c2.log 2>&1 \
 && echo "rocprof ok"
rc=$?
echo "rc=$rc"
tail -3 gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu_slow.log 2>/dev/null
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu*.log | head -20
exit $rc

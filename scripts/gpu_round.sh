#!/bin/bash
# One GPU session: parity tests (fast, then the full-size config tests), smoke, the
# default bench line (with cpu_baseline and the in-flight `concurrent` rates), and a
# rocprofv3 kernel-trace summary of the c2 bench; DIAG=1 adds the scan-variant A/B
# (diagnostics library), PMC=1 the counter passes for bench.py's `traffic`.  Every GPU step has its own time
# limit; steps are chained with && so a failure stops the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
timeout -k 10 600 python -u -m pytest tests/ -x -v -m "gpu and not slow" --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
 && echo "pytest fast ok" \
 && timeout -k 10 700 python -u -m pytest tests/ -x -v -m "gpu and slow" --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_slow.log 2>&1 \
 && echo "pytest slow ok" \
 && timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && cat gpurun_out/smoke.log \
 && timeout -k 10 400 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err && cat gpurun_out/bench_c2.json \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_c2" -o run --output-format csv -- python3 "$R/bench.py" --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-concurrent > gpurun_out/prof_${TAG}_c2.log 2>&1 \
 && echo "rocprof ok" \
 && { [ -z "$DIAG" ] || { timeout -k 10 300 python -u scripts/diag_scan.py --modes "" > gpurun_out/diag_scan_${TAG}.json 2> gpurun_out/diag_scan.err && cat gpurun_out/diag_scan_${TAG}.json; }; } \
 && { [ -z "$PMC" ] || { CFG=c2 TAG=${TAG}_pmc bash scripts/gpu_pmc.sh && python3 scripts/pmc_summary.py gpurun_out ${TAG}_pmc > gpurun_out/${TAG}_pmc_c2.json; }; }
rc=$?
echo "rc=$rc"
tail -3 gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu_slow.log 2>/dev/null
exit $rc

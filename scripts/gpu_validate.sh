#!/bin/bash
# One validation session on the GPU box (folds the per-session scripts of rounds 1-4):
#   STEPS="tests slow smoke bench configs trace conc scan" TAG=r04_v8 bash scripts/gpu_validate.sh
# Steps, run in the order given (default: all but conc and scan):
#   tests    pytest -m "gpu and not slow"        slow    pytest -m "gpu and slow"
#   smoke    __graft_entry__.smoke()             bench   the default bench line (config 2, everything on)
#   configs  bench lines for c3, c4, c5 (20 steps; cpu baseline and clock included)
#   trace    rocprofv3 --kernel-trace --stats of the c2-c5 bench commands (no concurrent leg)
#   conc     the in-flight measurement alone, coalesced and per-batch digests (6 reps)
#   scan     K1 A/B: product / one-shot / persistent (scripts/scan_ab.py)
# Outputs: gpurun_out/${TAG}_*.  Every GPU step has its own time limit; the first failure
# ends the script (no step is retried).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-validate}
STEPS=${STEPS:-"tests slow smoke bench configs trace"}
o=gpurun_out/$TAG
fail() { echo "step $1 failed"; tail -30 "$2"; exit 1; }
for s in $STEPS; do
  case $s in
  tests) timeout -k 10 900 python -u -m pytest tests/ -x -v -m "gpu and not slow" --timeout 300 --timeout-method thread > ${o}_pytest_fast.log 2>&1 || fail tests ${o}_pytest_fast.log
         tail -1 ${o}_pytest_fast.log ;;
  slow)  timeout -k 10 1000 python -u -m pytest tests/ -x -v -m "gpu and slow" --timeout 400 --timeout-method thread > ${o}_pytest_slow.log 2>&1 || fail slow ${o}_pytest_slow.log
         tail -1 ${o}_pytest_slow.log ;;
  smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > ${o}_smoke.log 2>&1 || fail smoke ${o}_smoke.log
         tail -2 ${o}_smoke.log ;;
  bench) timeout -k 10 600 python bench.py --steps 20 --warmup 5 > ${o}_bench_c2.json 2> ${o}_bench_c2.err || fail bench ${o}_bench_c2.err
         cut -c1-300 ${o}_bench_c2.json ;;
  configs)
         for c in c3 c4 c5; do
           timeout -k 10 600 python bench.py --config $c --steps 20 --warmup 3 --no-concurrent --e2e '' --drop-in '' > ${o}_bench_$c.json 2> ${o}_bench_$c.err || fail "bench $c" ${o}_bench_$c.err
           cut -c1-300 ${o}_bench_$c.json
         done ;;
  trace)
         for c in c2 c3 c4 c5; do
           timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/${o}_trace_$c" -o run --output-format csv -- python3 "$R/bench.py" --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-concurrent --no-clock --e2e '' --drop-in '' > ${o}_trace_$c.log 2>&1 || fail "trace $c" ${o}_trace_$c.log
           echo "trace $c ok"
         done ;;
  conc)  timeout -k 10 400 python bench.py --concurrent-only --concurrent-reps 6 > ${o}_conc_coal.json 2> ${o}_conc_coal.err || fail conc ${o}_conc_coal.err
         timeout -k 10 400 python bench.py --concurrent-only --concurrent-reps 6 --no-coalesce > ${o}_conc_nocoal.json 2> ${o}_conc_nocoal.err || fail conc ${o}_conc_nocoal.err
         cat ${o}_conc_coal.json ${o}_conc_nocoal.json ;;
  scan)  timeout -k 10 300 python -u scripts/scan_ab.py --configs c2,c4,c5 --reps 5 --kernels 0,1,2 > ${o}_scan_ab.json 2> ${o}_scan_ab.err || fail scan ${o}_scan_ab.err
         cut -c1-600 ${o}_scan_ab.json ;;
  *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "rc=0"

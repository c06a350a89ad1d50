# round 6 v20: BLAKE3 leaves holding the last 128-byte line in registers (CG_B3_HOLD_TAIL=1,
# chunker_amd/_ab/libchunker_amd_b3hold.so) against the product (aligned segments through LDS):
# parity with the variant, c3 A/B (same box, alternating), kernel trace and FETCH_SIZE of each
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=gpurun_out/r06_v20_summary.txt
V=$R/chunker_amd/_ab/libchunker_amd_b3hold.so
CHUNKER_AMD_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -k "blake3 or b3 or spans or config3" --timeout 300 --timeout-method thread -m gpu > gpurun_out/r06_v20_pytest_b3hold.txt 2>&1 || { echo "variant tests failed"; tail -30 gpurun_out/r06_v20_pytest_b3hold.txt; exit 1; }
tail -1 gpurun_out/r06_v20_pytest_b3hold.txt >> $S
B="--config c3 --steps 20 --warmup 3 --no-concurrent --e2e= --drop-in= --no-cpu-baseline --no-clock"
for rep in 1 2; do
  for lib in head b3hold; do
    if [ $lib = head ]; then L=""; else L=$V; fi
    CHUNKER_AMD_LIB=$L timeout -k 10 300 python -u bench.py $B > gpurun_out/r06_v20_c3_${lib}_$rep.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r06_v20_c3_${lib}_$rep.json'));print('c3 $lib', d['value'], d['stages_ms'])" >> $S
  done
done
for lib in head b3hold; do
  if [ $lib = head ]; then L=""; else L=$V; fi
  CHUNKER_AMD_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r06_v20_trace_$lib" -o run --output-format csv -- python3 "$R/bench.py" --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-concurrent --no-clock --e2e= --drop-in= > gpurun_out/r06_v20_trace_$lib.log 2>&1 || exit $?
  CHUNKER_AMD_LIB=$L timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/r06_v20_pmc_$lib" -o run --output-format csv -- python3 "$R/bench.py" --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-concurrent --no-clock --e2e= --drop-in= --no-stage-profile > gpurun_out/r06_v20_pmc_$lib.log 2>&1 || exit $?
done
cat $S

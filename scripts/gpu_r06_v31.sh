# round 6 v31: lean persistent scan (>= 4 GiB batches) in the pipeline: parity with the lean
# scans forced everywhere (one-shot and persistent), then c4 / c5 (lean vs forced off) and c2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=gpurun_out/r06_v31_summary.txt
CHUNKER_AMD_SCAN_LEAN=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_pipeline.py -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/r06_v31_pytest_lean.txt 2>&1 || { echo "lean tests failed"; tail -30 gpurun_out/r06_v31_pytest_lean.txt; exit 1; }
tail -1 gpurun_out/r06_v31_pytest_lean.txt >> $S
B="--steps 20 --warmup 5 --no-concurrent --e2e= --drop-in= --no-cpu-baseline --no-clock"
for rep in 1 2; do for c in c5 c4; do for lean in def 0; do
  if [ $lean = def ]; then E=""; else E="CHUNKER_AMD_SCAN_LEAN=0"; fi
  env $E timeout -k 10 300 python -u bench.py --config $c $B > gpurun_out/r06_v31_${c}_$lean.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_v31_${c}_$lean.json'));p=d['pipeline'];print('$c lean=$lean', d['value'], 'steady', p['steady_window']['GiBps'], 'launch', d['roofline']['launch']['ms'], 'p50', d['batch_latency_ms']['p50'])" >> $S
done; done; done
timeout -k 10 300 python -u bench.py $B > gpurun_out/r06_v31_c2.json 2>/dev/null || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/r06_v31_c2.json'));p=d['pipeline'];print('c2', d['value'], 'steady', p['steady_window']['GiBps'], 'launch', d['roofline']['launch']['ms'], 'p50', d['batch_latency_ms']['p50'])" >> $S
cat $S

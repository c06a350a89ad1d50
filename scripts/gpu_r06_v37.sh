# round 6 v37: lane staggering (k_pipe_stagger / k_pipe_end) with four lanes and two boundary
# streams: tests, then bench lines (value = one 20-step window vs the 4 x lanes group steady
# window), stagger on and off
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=gpurun_out/r06_v37_summary.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q -m gpu -k "pipeline" --timeout 400 --timeout-method thread > gpurun_out/r06_v37_pytest.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06_v37_pytest.txt; exit 1; }
tail -1 gpurun_out/r06_v37_pytest.txt >> $S
B="--steps 20 --warmup 5 --no-concurrent --e2e= --drop-in= --no-cpu-baseline --no-clock"
for rep in 1 2 3; do for st in 1 0; do
  if [ $st = 0 ] && [ $rep = 3 ]; then continue; fi
  CHUNKER_AMD_PIPE_STAGGER=$st timeout -k 10 300 python -u bench.py $B > gpurun_out/r06_v37_c2_s${st}_$rep.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_v37_c2_s${st}_$rep.json'));p=d['pipeline'];print('c2 stagger=$st', d['value'], 'steady', p['steady_window']['GiBps'], 'settle', p['settle_GiBps'], 'launch', d['roofline']['launch']['ms'], 'p50', d['batch_latency_ms']['p50'])" >> $S
done; done
for c in c4 c5; do
  timeout -k 10 300 python -u bench.py --config $c $B > gpurun_out/r06_v37_$c.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_v37_$c.json'));p=d['pipeline'];print('$c', d['value'], 'steady', p['steady_window']['GiBps'], 'launch', d['roofline']['launch']['ms'], 'p50', d['batch_latency_ms']['p50'])" >> $S
done
cat $S

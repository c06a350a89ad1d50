# round 6 v30: the lean boundary-stream scan as the product (pipeline only) with three digest
# lanes: parity, c2 sweep of group x lanes, default bench lines c2 / c4 / c5 at 2 and 3 lanes
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=gpurun_out/r06_v30_summary.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/r06_v30_pytest.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06_v30_pytest.txt; exit 1; }
tail -1 gpurun_out/r06_v30_pytest.txt >> $S
timeout -k 10 400 python -u scripts/pipe_bench.py --config c2 --sweep 20x3,24x3,16x3,12x3,20x2 --steps 120 --profile > gpurun_out/r06_v30_c2_sweep.jsonl 2>/dev/null || exit $?
python3 -c "
import json
for l in open('gpurun_out/r06_v30_c2_sweep.jsonl'):
    d=json.loads(l)
    if 'group' in d: print('c2 sweep', d['group'], d['lanes'], d['GiBps'], d['stats'].get('digest_ms_mean'), d.get('lat_p50_ms'))" >> $S
B="--steps 20 --warmup 5 --no-concurrent --e2e= --drop-in= --no-cpu-baseline --no-clock"
for c in c2 c4 c5; do for L in 3 2; do
  timeout -k 10 300 python -u bench.py --config $c --lanes $L $B > gpurun_out/r06_v30_${c}_L$L.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_v30_${c}_L$L.json'));p=d['pipeline'];print('$c lanes=$L', d['value'], 'steady', p['steady_window']['GiBps'], 'launch', d['roofline']['launch']['ms'], 'p50', d['batch_latency_ms']['p50'], 'scan', d['stages_ms']['scan'])" >> $S
done; done
cat $S

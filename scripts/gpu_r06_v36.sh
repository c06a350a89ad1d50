# round 6 v36: the product with two boundary streams and four lanes for SHA-256 batches under
# 4 GiB (one boundary stream, three lanes from 4 GiB): pipeline + parity tests, bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=gpurun_out/r06_v36_summary.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/r06_v36_pytest.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06_v36_pytest.txt; exit 1; }
tail -1 gpurun_out/r06_v36_pytest.txt >> $S
B="--steps 20 --warmup 5 --no-concurrent --e2e= --drop-in= --no-cpu-baseline --no-clock"
for rep in 1 2; do for c in c2 c4 c5 c3; do
  timeout -k 10 300 python -u bench.py --config $c $B > gpurun_out/r06_v36_${c}_$rep.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_v36_${c}_$rep.json'));p=d['pipeline'];print('$c', d['value'], 'steady', (p.get('steady_window') or {}).get('GiBps'), 'group/lanes/depth', p['group'], p['lanes'], p['depth'], 'launch', d['roofline'].get('launch',{}).get('ms'), 'p50', d['batch_latency_ms']['p50'])" >> $S
done; done
timeout -k 10 400 python -u bench.py $B --dist-force > gpurun_out/r06_v36_dist.json 2> gpurun_out/r06_v36_dist.err || exit $?
python3 -c "import json;d=[json.loads(l) for l in open('gpurun_out/r06_v36_dist.json') if l.startswith('{')][-1];p=d['pipeline'];print('dist-force', d['value'], 'steady', p['steady_window']['GiBps'], 'p50', d['batch_latency_ms']['p50'], d.get('gather_check'))" >> $S
cat $S

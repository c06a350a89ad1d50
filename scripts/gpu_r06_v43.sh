# round 6 v43: BLAKE3 pipelines on three boundary streams, depth 8: GPU tests, c3 and c2 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=gpurun_out/r06_v43_summary.txt
timeout -k 10 600 python -u -m pytest tests/ -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/r06_v43_pytest.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06_v43_pytest.txt; exit 1; }
tail -1 gpurun_out/r06_v43_pytest.txt >> $S
B="--steps 20 --warmup 5 --no-concurrent --e2e= --drop-in= --no-cpu-baseline --no-clock"
for rep in 1 2; do for c in c3 c2; do
  timeout -k 10 300 python -u bench.py --config $c $B > gpurun_out/r06_v43_${c}_$rep.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_v43_${c}_$rep.json'));p=d['pipeline'];print('$c', d['value'], 'steady', (p.get('steady_window') or {}).get('GiBps'), 'depth', p['depth'], 'p50', d['batch_latency_ms']['p50'])" >> $S
done; done
cat $S

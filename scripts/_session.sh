cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v31
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_robust.py -m gpu > gpurun_out/${T}_robust.log 2>&1 || { tail -30 gpurun_out/${T}_robust.log; exit 1; }
tail -1 gpurun_out/${T}_robust.log
for rep in 1 2; do
timeout -k 10 400 python -u bench.py --concurrent-only --concurrent 8,12,16,32 --concurrent-reps 6 > gpurun_out/${T}_conc_$rep.json 2> gpurun_out/${T}_conc_$rep.err || exit 1
python3 -c "
import json;d=json.load(open('gpurun_out/${T}_conc_$rep.json'))['concurrent']
for k in ('K8','K12','K16','K32'):
    x=d[k+'_detail'];print(k, d[k], 'merged', x['merged']['GiBps'], x['merged']['p50'], x['merged']['p99'], x['merged']['coalescer']['groups'], 'per_batch', x['per_batch']['GiBps'], x['per_batch']['p50'], x['per_batch']['p99'])
"
done

# round 6 v12: the driver's default bench line (all legs), --dist-force, c3 / c4 / c5 lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
( time timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_v12_bench_c2_full.json 2> gpurun_out/r06_v12_bench_c2_full.err ) 2> gpurun_out/r06_v12_time.txt || exit $?
B="--steps 20 --warmup 5 --no-concurrent --drop-in= --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $B --dist-force > gpurun_out/r06_v12_bench_c2_dist.json 2> gpurun_out/r06_v12_bench_c2_dist.err || exit $?
timeout -k 10 300 python -u bench.py $B > gpurun_out/r06_v12_bench_c2_lean.json 2>/dev/null || exit $?
for c in c3 c4 c5; do
  timeout -k 10 300 python -u bench.py --config $c $B > gpurun_out/r06_v12_bench_$c.json 2> gpurun_out/r06_v12_bench_$c.err || exit $?
done
for f in c2_full c2_dist c2_lean c3 c4 c5; do python3 -c "
import json;d=json.load(open('gpurun_out/r06_v12_bench_$f.json'));p=d['pipeline'];print('$f', d['value'], p['group'], p['lanes'], p['depth'], p['steady_window']['GiBps'], d['batch_latency_ms']['p50'], d['roofline']['launch'], d.get('gather_check'))"; done > gpurun_out/r06_v12_summary.txt
cat gpurun_out/r06_v12_summary.txt gpurun_out/r06_v12_time.txt

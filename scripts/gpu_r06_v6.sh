# round 6 v6: pipeline/multi tests; steady-state bench (group end to group end), lanes 2 vs 3, repeated
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_pipeline.py -v --timeout 300 --timeout-method thread > gpurun_out/r06_v6_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for L in 2 3 2 3; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-concurrent --drop-in '' --no-cpu-baseline --no-clock --lanes $L > gpurun_out/r06_v6_bench_c2_L$L.json 2> gpurun_out/r06_v6_bench_c2_L$L.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/r06_v6_bench_c2_L$L.json'));print('L$L', d['value'], d['pipeline'], d['batch_latency_ms'], d['roofline']['launch'])" >> gpurun_out/r06_v6_bench_summary.txt
done

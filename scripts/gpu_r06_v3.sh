# round 6 v3: pipeline GPU tests, (group x lanes) sweep, short bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_v3_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u scripts/pipe_bench.py --config c2 --sweep 16x2,24x2,32x2,12x3,16x3,20x3,32x1,48x1 --steps 96 --profile > gpurun_out/r06_v3_pipe_c2.jsonl 2> gpurun_out/r06_v3_pipe_c2.err || exit $?
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-concurrent --drop-in '' --no-cpu-baseline > gpurun_out/r06_v3_bench_c2.json 2> gpurun_out/r06_v3_bench_c2.err
echo "bench rc=$?"

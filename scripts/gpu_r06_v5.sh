# round 6 v5: pipeline + multi-device tests, pipeline parity tests, bench (steady state), sweep
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_pipeline.py "tests/test_gpu_parity.py::test_batch_pipeline_matches_sync" "tests/test_gpu_parity.py::test_async_after_inputs_ready_matches_sync" "tests/test_gpu_parity.py::test_async_batches_match_sync" -v --timeout 300 --timeout-method thread > gpurun_out/r06_v5_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-concurrent --drop-in '' --no-cpu-baseline > gpurun_out/r06_v5_bench_c2.json 2> gpurun_out/r06_v5_bench_c2.err || exit $?
timeout -k 10 400 python -u scripts/pipe_bench.py --config c2 --sweep 24x2,16x3,20x2,28x2 --steps 96 --profile > gpurun_out/r06_v5_pipe_c2.jsonl 2> gpurun_out/r06_v5_pipe_c2.err

cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v46
CHUNKER_AMD_FUZZ_SEEDS=640 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fuzz.py -m gpu > gpurun_out/${T}_fuzz640.log 2>&1 || { tail -30 gpurun_out/${T}_fuzz640.log; exit 1; }
tail -1 gpurun_out/${T}_fuzz640.log
f=gpurun_out/${T}_c2_soak
timeout -k 10 300 python -u bench.py --config c2 --steps 1000 --warmup 5 --no-cpu-baseline --no-concurrent --drop-in '' --e2e '' --no-clock > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
python3 scripts/depth_row.py $f.json c2 "1000 steps"

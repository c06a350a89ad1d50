cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v10
CONFIGS="c2 c3" TAG=$T bash scripts/gpu_pmc_all.sh || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --dist-force --steps 10 --warmup 3 --no-cpu-baseline --no-concurrent --e2e '' --drop-in '' --no-clock > gpurun_out/${T}_bench_c2_dist.json 2> gpurun_out/${T}_bench_c2_dist.err || { tail -20 gpurun_out/${T}_bench_c2_dist.err; exit 1; }
cut -c1-400 gpurun_out/${T}_bench_c2_dist.json
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --steps 4 --warmup 1 --no-cpu-baseline --no-concurrent --e2e '' --drop-in '' --no-clock > gpurun_out/${T}_bench_g2_gloo.json 2> gpurun_out/${T}_bench_g2_gloo.err || { tail -20 gpurun_out/${T}_bench_g2_gloo.err; exit 1; }
cut -c1-400 gpurun_out/${T}_bench_g2_gloo.json; grep -o '"gather_check".*' gpurun_out/${T}_bench_g2_gloo.json | cut -c1-200
timeout -k 10 300 python -u -m pytest tests/test_dist.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_dist.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_dist.log; exit 1; }
tail -1 gpurun_out/${T}_pytest_dist.log
echo done

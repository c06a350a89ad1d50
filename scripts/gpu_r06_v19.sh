# round 6 v19: BLAKE3 leaves with the aligned-segment LDS ring as the product: fast GPU suite,
# c3 bench lines, PMC passes for config 3 (traffic source of the c3 bench line)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/ -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/r06_v19_pytest_fast.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06_v19_pytest_fast.log; exit 1; }
tail -1 gpurun_out/r06_v19_pytest_fast.log
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-concurrent --e2e= --drop-in= > gpurun_out/r06_v19_bench_c3_$rep.json 2>/dev/null || exit $?
  cut -c1-200 gpurun_out/r06_v19_bench_c3_$rep.json
done
CFG=c3 TAG=r06_v19_pmc_c3 bash scripts/gpu_pmc.sh || exit $?
python3 scripts/pmc_summary.py gpurun_out r06_v19_pmc_c3 > gpurun_out/r06_v19_pmc_c3.json
python3 -c "
import json
d=json.load(open('gpurun_out/r06_v19_pmc_c3.json'))
for k,v in d.items():
    if 'b3' in k or 'scan' in k: print(k, v.get('fetch_bytes_x2'), v.get('SQ_INSTS_VALU'), v.get('SQ_WAVES'))"

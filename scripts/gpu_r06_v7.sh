# round 6 v7: SHA ring 34 KiB (two one-lane slots, early release) -- parity first; then
# occupancy A/B on c4 / c5 / c2 pipeline; --dist-force; c3
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robust.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread -m "gpu and not slow" > gpurun_out/r06_v7_pytest.txt 2>&1
rc=$?
tail -5 gpurun_out/r06_v7_pytest.txt
if [ $rc -ne 0 ]; then exit $rc; fi
B="--steps 20 --warmup 5 --no-concurrent --drop-in= --no-cpu-baseline --no-clock --no-stage-profile"
for occ in 2,2 4,4 2,4 3,3; do
  for cfg in c4 c5; do
    timeout -k 10 300 python -u bench.py --config $cfg $B --sha-occ $occ > gpurun_out/r06_v7_bench_${cfg}_occ${occ/,/_}.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r06_v7_bench_${cfg}_occ${occ/,/_}.json'));print('$cfg occ $occ', d['value'], d['pipeline']['steady_window']['GiBps'], d['roofline']['launch'])" >> gpurun_out/r06_v7_summary.txt
  done
  timeout -k 10 300 python -u bench.py $B --sha-occ $occ > gpurun_out/r06_v7_bench_c2_occ${occ/,/_}.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_v7_bench_c2_occ${occ/,/_}.json'));print('c2 occ $occ', d['value'], d['pipeline']['steady_window']['GiBps'], d['roofline']['launch'])" >> gpurun_out/r06_v7_summary.txt
done
cat gpurun_out/r06_v7_summary.txt

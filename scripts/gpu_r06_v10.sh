# round 6 v10: fused one-lane SHA-256 tier for GPU-filling launches -- parity, then c4 / c5 A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "fused or workgroup_kinds or latency_tiers or descriptors_match or spans or randomized" > gpurun_out/r06_v10_pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r06_v10_pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "config4 or config5" > gpurun_out/r06_v10_pytest_cfg.txt 2>&1
rc=$?; tail -3 gpurun_out/r06_v10_pytest_cfg.txt; [ $rc -ne 0 ] && exit $rc
B="--steps 20 --warmup 5 --no-concurrent --drop-in= --no-cpu-baseline --no-clock --no-stage-profile"
for v in "0 2,2" "1 2,2" "1 2,3" "1 2,4"; do
  set -- $v
  for cfg in c4 c5; do
    f=gpurun_out/r06_v10_${cfg}_f$1_occ${2/,/_}.json
    timeout -k 10 300 python -u bench.py --config $cfg $B --sha-fused $1 --sha-occ $2 > $f 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('$f'));print('$cfg fused $1 occ $2', d['value'], d['pipeline']['steady_window']['GiBps'], d['roofline']['launch']['ms'])" >> gpurun_out/r06_v10_summary.txt
  done
done
cat gpurun_out/r06_v10_summary.txt

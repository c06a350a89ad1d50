# round 6 v11: same-box A/B -- c4 / c5 group 1 vs 2, fused one-lane tier on / off (2 workgroups per CU)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
B="--steps 20 --warmup 5 --no-concurrent --drop-in= --no-cpu-baseline --no-clock --no-stage-profile --sha-occ 2,2"
for rep in 1 2; do
for v in "c4 1 0" "c4 1 1" "c4 2 0" "c4 2 1" "c5 1 0" "c5 2 0" "c5 2 1" "c5 4 0"; do
  set -- $v
  f=gpurun_out/r06_v11_${1}_g$2_f$3_r$rep.json
  timeout -k 10 300 python -u bench.py --config $1 $B --group $2 --sha-fused $3 > $f 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('$f'));print('$1 group $2 fused $3', d['value'], d['pipeline']['steady_window']['GiBps'], d['roofline']['launch']['ms'])" >> gpurun_out/r06_v11_summary.txt
done
done
cat gpurun_out/r06_v11_summary.txt

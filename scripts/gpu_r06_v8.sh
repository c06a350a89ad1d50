# round 6 v8: one-lane ring A/B (4 slots = round 5 / 3 slots + early release = product / 2 slots)
# x workgroups per CU, on c4 / c5 / c2 (pipeline)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
B="--steps 20 --warmup 5 --no-concurrent --drop-in= --no-cpu-baseline --no-clock --no-stage-profile"
run() {  # lib occ cfg
  local lib=$1 occ=$2 cfg=$3 f=gpurun_out/r06_v8_${1}_${3}_occ${2/,/_}.json
  if [ "$lib" = ring3 ]; then L=""; else L=chunker_amd/_ab/libchunker_amd_$lib.so; fi
  CHUNKER_AMD_LIB=$L timeout -k 10 300 python -u bench.py --config $cfg $B --sha-occ $occ > $f 2>/dev/null || return $?
  python3 -c "import json;d=json.load(open('$f'));print('$lib $cfg occ $occ', d['value'], d['pipeline']['steady_window']['GiBps'], d['pipeline']['group'], d['roofline']['launch']['ms'])" >> gpurun_out/r06_v8_summary.txt
}
for cfg in c4 c2 c5; do
  run ring4 2,2 $cfg || exit $?
  run ring3 2,2 $cfg || exit $?
  run ring3 3,3 $cfg || exit $?
  run ring2 4,4 $cfg || exit $?
done
cat gpurun_out/r06_v8_summary.txt

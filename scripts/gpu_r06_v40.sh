# round 6 v40: lane staggering on / off at three lanes, same box, alternating: c4, c5, c2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=gpurun_out/r06_v40_summary.txt
B="--steps 20 --warmup 5 --no-concurrent --e2e= --drop-in= --no-cpu-baseline --no-clock --no-stage-profile"
for rep in 1 2; do for c in c4 c5 c2; do for st in 1 0; do
  CHUNKER_AMD_PIPE_STAGGER=$st timeout -k 10 300 python -u bench.py --config $c $B > gpurun_out/r06_v40_${c}_s${st}_$rep.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_v40_${c}_s${st}_$rep.json'));p=d['pipeline'];print('$c stagger=$st', d['value'], 'steady', p['steady_window']['GiBps'], 'settle', p['settle_GiBps'], 'launch', d['roofline']['launch']['ms'])" >> $S
done; done; done
cat $S

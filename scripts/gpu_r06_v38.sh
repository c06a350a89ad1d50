# round 6 v38: with a longer settle (>= 4 x lanes groups): does the 20-step value of four
# staggered lanes land near the steady window?  Against three lanes / one boundary stream.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=gpurun_out/r06_v38_summary.txt
B="--steps 20 --warmup 5 --no-concurrent --e2e= --drop-in= --no-cpu-baseline --no-clock"
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench.py $B > gpurun_out/r06_v38_c2_L4_$rep.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_v38_c2_L4_$rep.json'));p=d['pipeline'];print('c2 4 lanes 2 bstreams', d['value'], 'steady', p['steady_window']['GiBps'], 'settle', p['settle_steps'], p['settle_GiBps'], 'p50', d['batch_latency_ms']['p50'])" >> $S
  CHUNKER_AMD_PIPE_BSTREAMS=1 timeout -k 10 300 python -u bench.py $B --lanes 3 > gpurun_out/r06_v38_c2_L3_$rep.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_v38_c2_L3_$rep.json'));p=d['pipeline'];print('c2 3 lanes 1 bstream', d['value'], 'steady', p['steady_window']['GiBps'], 'settle', p['settle_steps'], p['settle_GiBps'], 'p50', d['batch_latency_ms']['p50'])" >> $S
done
cat $S

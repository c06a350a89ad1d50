# round 6 v42: BLAKE3 batches on one / two / three boundary streams (consecutive batches then
# overlap: the next scan beside the current digest), same box, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=gpurun_out/r06_v42_summary.txt
B="--config c3 --steps 20 --warmup 3 --no-concurrent --e2e= --drop-in= --no-cpu-baseline --no-clock --no-stage-profile"
for rep in 1 2 3; do for nb in 1 2 3; do
  CHUNKER_AMD_PIPE_BSTREAMS=$nb timeout -k 10 300 python -u bench.py $B --depth 8 > gpurun_out/r06_v42_c3_b${nb}_$rep.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_v42_c3_b${nb}_$rep.json'));p=d['pipeline'];print('c3 bstreams=$nb', d['value'], 'steady', (p.get('steady_window') or {}).get('GiBps'), 'p50', d['batch_latency_ms']['p50'])" >> $S
done; done
cat $S

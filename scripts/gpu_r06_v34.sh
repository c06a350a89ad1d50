# round 6 v34: the N > 1 path at one nccl rank (--dist-force) with the three-lane pipeline and
# lean boundary scans, against the one-rank line on the same box; then 4 lanes with the
# lanes in HIP's low-priority pool (CHUNKER_AMD_PIPE_STREAMS=split)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=gpurun_out/r06_v34_summary.txt
B="--steps 20 --warmup 5 --no-concurrent --e2e= --drop-in= --no-cpu-baseline --no-clock"
for rep in 1 2; do
  timeout -k 10 400 python -u bench.py $B > gpurun_out/r06_v34_one_$rep.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_v34_one_$rep.json'));p=d['pipeline'];print('one rank', d['value'], 'steady', p['steady_window']['GiBps'], 'p50', d['batch_latency_ms']['p50'])" >> $S
  timeout -k 10 400 python -u bench.py $B --dist-force > gpurun_out/r06_v34_dist_$rep.json 2> gpurun_out/r06_v34_dist_$rep.err || exit $?
  python3 -c "import json;d=[json.loads(l) for l in open('gpurun_out/r06_v34_dist_$rep.json') if l.startswith('{')][-1];p=d['pipeline'];print('dist-force', d['value'], 'steady', p['steady_window']['GiBps'], 'p50', d['batch_latency_ms']['p50'], d.get('gather_check'))" >> $S
done
CHUNKER_AMD_PIPE_STREAMS=split timeout -k 10 400 python -u scripts/pipe_bench.py --config c2 --sweep 20x3,20x4,24x4,16x4 --steps 120 --profile > gpurun_out/r06_v34_split.jsonl 2>/dev/null || exit $?
python3 -c "
import json
for l in open('gpurun_out/r06_v34_split.jsonl'):
    d=json.loads(l)
    if 'group' in d: print('split', d['group'], d['lanes'], d['GiBps'], d['stats'].get('digest_ms_mean'), d.get('lat_p50_ms'))" >> $S
cat $S

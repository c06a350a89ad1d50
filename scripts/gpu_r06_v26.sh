# round 6 v26: is it the merged launch's empty workgroups?  The grid is sized from the members'
# capacity (~87 k chunks for 20 config-2 batches, ~20 k real): ~1,000 workgroups that exit at
# once but each needs a 70 KiB slot, churning through every slot a finishing workgroup frees --
# the scans of the next group wait behind them.  A/B: grid from 1.4x the expected count
# (CHUNKER_AMD_PIPE_TIGHT=1, checked against the per-batch entry) vs capacity, same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=gpurun_out/r06_v26_summary.txt
CHUNKER_AMD_PIPE_TIGHT=1 timeout -k 10 300 python -u scripts/pipe_bench.py --config c2 --sweep 20x2 --steps 40 --check > gpurun_out/r06_v26_check.jsonl 2>&1 || { tail -20 gpurun_out/r06_v26_check.jsonl; exit 1; }
grep -o '"check": {[^}]*}' gpurun_out/r06_v26_check.jsonl >> $S
for rep in 1 2; do
  for t in 0 1; do
    CHUNKER_AMD_PIPE_TIGHT=$t timeout -k 10 300 python -u scripts/pipe_bench.py --config c2 --sweep 20x2,20x3,24x2 --steps 60 --profile > gpurun_out/r06_v26_t$t.jsonl 2>/dev/null || exit $?
    python3 -c "
import json
for l in open('gpurun_out/r06_v26_t$t.jsonl'):
    d=json.loads(l)
    if 'group' in d: print('c2 tight=$t', d['group'], d['lanes'], d['GiBps'], d['stats'].get('digest_ms_mean'), d.get('lat_p50_ms'))" >> $S
  done
done
cat $S
CHUNKER_AMD_PIPE_TIGHT=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r06_v26_trace" -o run --output-format csv -- python3 "$R/scripts/pipe_bench.py" --config c2 --sweep 20x3 --steps 60 --profile > gpurun_out/r06_v26_trace.jsonl 2> gpurun_out/r06_v26_trace.err || exit $?
python3 - <<'PY'
import csv, glob, collections
import numpy as np
f = glob.glob('gpurun_out/r06_v26_trace/*kernel_trace.csv')[0]
byk = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    byk[r['Kernel_Name'].split('(')[0].replace('void ', '')].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
for n, v in sorted(byk.items(), key=lambda x: -sum(x[1]))[:4]:
    v = np.array(v); print('tight trace', n[:44], len(v), 'mean %.3f p50 %.3f max %.3f' % (v.mean(), np.median(v), v.max()))
PY

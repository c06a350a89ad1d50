# round 6 v23: the boundary stream's scans wait for CU slots under the merged SHA-256 launches
# (k_scan_flat32 0.2 ms alone, mean 1.5 / max 27 ms in the pipeline: 68 KiB of LDS does not fit
# beside two 70 KiB digest workgroups).  A/B: boundary stream high priority + digest lanes low
# priority ("split") against all high priority, same box, alternating; kernel trace of split.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=gpurun_out/r06_v23_summary.txt
for rep in 1 2; do
  for kind in high split; do
    CHUNKER_AMD_PIPE_STREAMS=$kind timeout -k 10 300 python -u scripts/pipe_bench.py --config c2 --sweep 20x2,20x3,24x2 --steps 60 --profile > gpurun_out/r06_v23_$kind.jsonl 2>/dev/null || exit $?
    python3 -c "
import json
for l in open('gpurun_out/r06_v23_$kind.jsonl'):
    d=json.loads(l)
    if 'group' in d: print('$kind', d['group'], d['lanes'], d['GiBps'], d['stats'].get('digest_ms_mean'), d.get('lat_p50_ms'))" >> $S
  done
done
cat $S
CHUNKER_AMD_PIPE_STREAMS=split timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r06_v23_trace" -o run --output-format csv -- python3 "$R/scripts/pipe_bench.py" --config c2 --sweep 20x2 --steps 60 --profile > gpurun_out/r06_v23_trace.jsonl 2> gpurun_out/r06_v23_trace.err || exit $?
python3 - <<'PY'
import csv, glob, collections
import numpy as np
f = glob.glob('gpurun_out/r06_v23_trace/*kernel_trace.csv')[0]
byk = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    byk[r['Kernel_Name'].split('(')[0].replace('void ', '')].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
for n, v in sorted(byk.items(), key=lambda x: -sum(x[1]))[:5]:
    v = np.array(v); print('split trace', n[:40], len(v), 'mean %.3f p50 %.3f max %.3f' % (v.mean(), np.median(v), v.max()))
PY

# round 6 v22: why a third digest lane does not add throughput at 4 hardware queues:
# (1) how many high- / low-priority streams get a hardware queue of their own (4, 5 streams),
# (2) kernel trace of the config-2 pipeline at 20 x 3 (per-lane launch gaps vs stretch)
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06_v22_queue_probe.txt
for k in 1 2; do for n in 3 4 5 6; do
  timeout -k 5 30 scripts/micro/_bin/queue_probe $k $n 0 40 0 | tail -1 >> $O || exit $?
done; done
cat $O
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r06_v22_trace" -o run --output-format csv -- python3 "$R/scripts/pipe_bench.py" --config c2 --sweep 20x3,20x2 --steps 60 --profile > gpurun_out/r06_v22_pipe.jsonl 2> gpurun_out/r06_v22_pipe.err || exit $?
python3 - <<'PY'
import csv, glob, json
for l in open('gpurun_out/r06_v22_pipe.jsonl'):
    d = json.loads(l)
    if 'group' in d:
        print('run', d['group'], d['lanes'], d['GiBps'], d['stats'].get('digest_ms_mean'))
f = glob.glob('gpurun_out/r06_v22_trace/*kernel_trace.csv')[0]
rows = [r for r in csv.DictReader(open(f)) if 'k_sha256' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
t0 = int(rows[0]['Start_Timestamp'])
last = {}
for r in rows:
    s = (int(r['Start_Timestamp']) - t0) / 1e6; e = (int(r['End_Timestamp']) - t0) / 1e6
    q = r.get('Queue_Id'); gap = s - last.get(q, s); last[q] = e
    print(round(s, 1), round(e, 1), 'dur', round(e - s, 1), 'queue', q, 'stream', r.get('Stream_Id'), 'gap_on_queue', round(gap, 1))
PY
# PMC passes of the merged 16 GiB-batch launches (configs 4 / 5: two batches per launch)
for c in c4 c5; do
  CFG=$c TAG=r06_v22_pmc_$c bash scripts/gpu_pmc.sh || exit $?
  python3 scripts/pmc_summary.py gpurun_out r06_v22_pmc_$c > gpurun_out/r06_v22_pmc_$c.json
done

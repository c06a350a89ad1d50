cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v58
for rep in 1 2; do
  f=gpurun_out/${T}_full_q22_d20_$rep
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --hw-queues 22 --depth 20 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "
import json,sys;d=json.load(open(sys.argv[1]));c=d['concurrent'];e=c['e2e']
print(sys.argv[2], d['value'], d['batch_latency_ms'], d['stages_ms']['digest_timed'], {k:c[k] for k in c if k.startswith('K') and not k.endswith('detail')}, e['h2d_only'], e['K1'], e['K8'], e['K16'], e['one_caller_overlapped']['GiBps'], d['drop_in']['sha256']['K32']['gpu']['GiBps'], d['drop_in']['blake3']['K8']['gpu']['GiBps'])" $f.json rep$rep
done
f=gpurun_out/${T}_q22_d20_n200
timeout -k 10 300 python -u bench.py --steps 200 --warmup 5 --hw-queues 22 --depth 20 --no-cpu-baseline --no-concurrent --drop-in '' --e2e '' --no-clock > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
python3 scripts/depth_row.py $f.json c2 "q22 d20 n200"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/${T}_trace_c2" -o run --output-format csv -- python3 "$PWD/bench.py" --config c2 --steps 5 --warmup 2 --hw-queues 22 --depth 20 --no-cpu-baseline --no-concurrent --no-clock --e2e '' --drop-in '' > gpurun_out/${T}_trace.log 2>&1 || { tail -5 gpurun_out/${T}_trace.log; exit 1; }
grep '^{' gpurun_out/${T}_trace.log | cut -c1-200

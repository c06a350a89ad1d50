cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v48
for c in c2 c3 c5; do
  f=gpurun_out/${T}_$c
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-concurrent --drop-in '' --e2e '' --no-clock > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 scripts/depth_row.py $f.json $c pipeline
done
f=gpurun_out/${T}_c2_nooverlap
timeout -k 10 300 python -u bench.py --config c2 --steps 10 --warmup 2 --no-overlap --no-cpu-baseline --no-concurrent --drop-in '' --e2e '' --no-clock > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
python3 scripts/depth_row.py $f.json c2 no-overlap
timeout -k 10 300 python -u bench.py --gpus 1 --dist-force --steps 20 --warmup 5 --no-cpu-baseline --no-concurrent --drop-in '' --e2e '' --no-clock > gpurun_out/${T}_dist.json 2> gpurun_out/${T}_dist.err || { tail -5 gpurun_out/${T}_dist.err; exit 1; }
grep '^{' gpurun_out/${T}_dist.json | cut -c1-200
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 6 --warmup 2 --no-cpu-baseline --no-concurrent --drop-in '' --e2e '' --no-clock > gpurun_out/${T}_gloo.json 2> gpurun_out/${T}_gloo.err || { tail -5 gpurun_out/${T}_gloo.err; exit 1; }
python3 -c "
import json;d=json.loads([l for l in open('gpurun_out/${T}_gloo.json') if l.startswith('{')][-1]);print(d['n_gpus'], d['value'], d.get('gather_check'))"

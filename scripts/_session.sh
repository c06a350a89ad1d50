cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v47
timeout -k 10 400 python -u bench.py --gpus 8 --dist-backend gloo --depth 2 --hw-queues 4 --steps 4 --warmup 1 --no-cpu-baseline --no-concurrent --drop-in '' --e2e '' --no-clock > gpurun_out/${T}_g8_gloo.json 2> gpurun_out/${T}_g8_gloo.err || { tail -20 gpurun_out/${T}_g8_gloo.err; exit 1; }
grep '^{' gpurun_out/${T}_g8_gloo.json | cut -c1-300
python3 -c "
import json;d=json.loads([l for l in open('gpurun_out/${T}_g8_gloo.json') if l.startswith('{')][-1]);print(d['n_gpus'], d['value'], d.get('gather_check'), d.get('note'))"

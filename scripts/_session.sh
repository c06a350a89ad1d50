cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --concurrent '' --e2e 1,8,16 --drop-in '' --no-clock > gpurun_out/r05_v13_e2e.json 2> gpurun_out/r05_v13_e2e.err || { tail -20 gpurun_out/r05_v13_e2e.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r05_v13_e2e.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d['concurrent']))"

cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v34
f=gpurun_out/${T}_c2_long
timeout -k 10 300 python -u bench.py --config c2 --steps 200 --warmup 5 --no-cpu-baseline --no-concurrent --drop-in '' --e2e '' --no-clock > $f.json 2> $f.err || exit $?
python3 scripts/depth_row.py $f.json c2 "200 steps"
STEPS="bench configs" TAG=$T bash scripts/gpu_validate.sh
